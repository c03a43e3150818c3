# two-group parity tests with a variant library, then the C3 bench alternating in-tree / variant
# usage: bash tools/gpu_ab_tg.sh <tag> <variant>
export TMPDIR=/tmp
tag=$1; v=$2
O=gpurun_out/$tag
mkdir -p $O
HYG_LIB_PATH=hygeia_amd/lib/libhygeia_amd_$v.so timeout -k 10 500 python -u -m pytest tests/test_gpu_two_group.py tests/test_gpu_tg_exact.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
i=0
for lib in base $v base $v; do
  i=$((i+1))
  if [ "$lib" = base ]; then unset HYG_LIB_PATH; else export HYG_LIB_PATH=hygeia_amd/lib/libhygeia_amd_$lib.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/c3_$i.log 2>&1 || { tail -5 $O/c3_$i.log; exit 1; }
  grep '^{' $O/c3_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
done
