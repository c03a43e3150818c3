# two-group: parity tests, phase split (142 chains), C3 bench line
# usage: bash tools/gpu_fw.sh <tag> [skip-tests]
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
timeout -k 10 500 python -u -m pytest tests/test_gpu_two_group.py tests/test_gpu_tg_exact.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
HYG_DEBUG_PHASES=1 timeout -k 10 200 python bench.py --sites 6000000 --no-cpu-baseline --steps 1 --warmup 0 > $O/phases.log 2>&1 || { tail -5 $O/phases.log; exit 1; }
grep "phases" $O/phases.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
grep '^{' $O/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
if [ "$3" = "ab-shape" ]; then
HYG_NO_SHAPE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/c3_noshape.log 2>&1 || { tail -5 $O/c3_noshape.log; exit 1; }
grep '^{' $O/c3_noshape.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3 generic', round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
fi
