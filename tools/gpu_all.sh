# every GPU parity test, then the C3 and C2 bench lines (no CPU baselines)
# usage: bash tools/gpu_all.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
grep '^{' $O/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
timeout -k 10 400 python tools/bench_sg.py --no-cpu-baseline > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
grep '^{' $O/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', round(d['value']), d['roofline']['kernel_ms'], d['roofline'].get('us_per_step_longest_chain'))"
