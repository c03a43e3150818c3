# C3 bench (forward/backward kernel ms) for the in-tree library and variant libraries
# usage: bash tools/gpu_ab_lib.sh <tag> <variant names...>
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
for v in base "$@"; do
  if [ "$v" = base ]; then unset HYG_LIB_PATH; else export HYG_LIB_PATH=hygeia_amd/lib/libhygeia_amd_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/c3_$v.log 2>&1 || { tail -5 $O/c3_$v.log; exit 1; }
  grep '^{' $O/c3_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
done
