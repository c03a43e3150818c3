# C5 parity tests with a variant library, then the C5 bench for the in-tree and variant libraries
# usage: bash tools/gpu_ab_c5.sh <tag> <variant>
export TMPDIR=/tmp
tag=$1; v=$2
O=gpurun_out/$tag
mkdir -p $O
HYG_LIB_PATH=hygeia_amd/lib/libhygeia_amd_$v.so timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/t_c5.log 2>&1 || { tail -30 $O/t_c5.log; exit 1; }
tail -1 $O/t_c5.log
for lib in base $v; do
  if [ "$lib" = base ]; then unset HYG_LIB_PATH; else export HYG_LIB_PATH=hygeia_amd/lib/libhygeia_amd_$lib.so; fi
  timeout -k 10 300 python bench.py --job c5 --no-cpu-baseline --steps 1 --warmup 0 > $O/c5_$lib.log 2>&1 || { tail -5 $O/c5_$lib.log; exit 1; }
  grep '^{' $O/c5_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
done
