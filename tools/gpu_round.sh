# One GPU call: parity tests, the default bench line (with CPU baselines), the
# 1-GPU C4 point, and the profile set of the default workload.
# usage: bash tools/gpu_round.sh <tag> [skip-tests]
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
( nproc; python3 -c 'import os; print(len(os.sched_getaffinity(0)), os.environ.get("OMP_NUM_THREADS"))'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo ) > $O/host.txt 2>&1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1
timeout -k 10 600 python bench.py --job c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log | tail -1
bash tools/gpu_profile.sh $tag > $O/profile.log 2>&1; rc=$?
cat $O/profile.log
exit $rc
