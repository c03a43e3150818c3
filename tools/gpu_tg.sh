# two-group: parity tests (incl. the exact-model and config tests) and the C3 bench line
# usage: bash tools/gpu_tg.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_two_group.py tests/test_gpu_tg_exact.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
grep '^{' $O/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
