# single-group: parity tests, phase split (chr1 prefix) and the C2 bench line
# usage: bash tools/gpu_sg.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_single_group.py tests/test_gpu_sg_pe.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
HYG_SG_PHASES=1 timeout -k 10 300 python tools/bench_sg.py --sites 3000000 --no-cpu-baseline > $O/phases.log 2>&1 || { tail -5 $O/phases.log; exit 1; }
grep "phases" $O/phases.log
timeout -k 10 400 python tools/bench_sg.py --no-cpu-baseline > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
grep '^{' $O/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', round(d['value']), d['roofline']['kernel_ms'], d['roofline'].get('us_per_step_longest_chain'))"
