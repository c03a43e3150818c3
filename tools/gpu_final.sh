# The round's final measurement set on one GPU call, every step under its own
# time limit, stopping at the first crash / time-out (exit status other than 0):
#   parity tests; the default bench line (C3, CPU baselines); C4 and C5 on one
#   GPU; the C3 / C4 shares of 8 ranks (projections) and the C3 share's phase
#   split (tuning build); single group C2 and C1; the pipeline-level bench; the
#   rocprofv3 profile set of the default workload (tools/gpu_profile.sh).
# Outputs: gpurun_out/<tag>/* (only gpurun_out/ comes back from the box; copy
# gpurun_out/<tag>/out/* and gpurun_out/prof_<tag>/* into profiles/ afterwards).
# usage: bash tools/gpu_final.sh <tag> [no-profile|profile] [a|b|c|all]
#   (part a: tests, two-group benches and the phase split; part b: single
#   group and pipeline benches; part c: the 2- and 4-rank shares of C3 / C4;
#   all: a and b, the default)
set -u
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
TUNE=hygeia_amd/lib/var_tuning/libhygeia_amd.so
( nproc; python3 -c 'import os; print(len(os.sched_getaffinity(0)), os.environ.get("OMP_NUM_THREADS"))'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo ) > $O/host.txt 2>&1
step() {  # step <name> <seconds> <command...>
  local name=$1 secs=$2; shift 2
  echo "[$name] $*"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  grep '^{' $O/$name.log | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc: stop"; tail -20 $O/$name.log; exit $rc; fi
}
part=${3:-all}
if [ "$part" = "a" ] || [ "$part" = "all" ]; then
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
tail -2 $O/tests.log
step bench_c3 600 python bench.py
step bench_c4 600 python bench.py --job c4 --steps 1 --warmup 1 --no-cpu-baseline
step bench_c5 600 python bench.py --job c5 --steps 1 --warmup 1 --no-cpu-baseline
step bench_c3_shard0of8 300 python bench.py --shard 0/8 --no-cpu-baseline --steps 2
step bench_c4_shard0of8 300 python bench.py --job c4 --shard 0/8 --no-cpu-baseline --steps 1
# the tuning build must be of the benched sources (bash tools/build_variant.sh tuning -DHYG_TUNING)
SRC=$(python3 -c "from hygeia_amd import build; print(build.source_hash())")
if [ -f $TUNE ] && [ "$(cat $(dirname $TUNE)/source_hash 2>/dev/null)" != "$SRC" ]; then
  echo "[phases] the tuning library is not built from these sources ($SRC): skipped"
elif [ -f $TUNE ]; then
  step phases_c3_shard0of8 300 env HYG_LIB_PATH=$TUNE HYG_DEBUG_PHASES=1 python bench.py --shard 0/8 --no-cpu-baseline --steps 1 --warmup 0
fi
fi
if [ "$part" = "c" ]; then
for j in c3 c4; do for w in 2 4; do
  step bench_${j}_shard0of$w 300 python bench.py --job $j --shard 0/$w --no-cpu-baseline --steps 1
done; done
fi
if [ "$part" != "a" ] && [ "$part" != "c" ]; then
step bench_c2 600 python tools/bench_sg.py
step bench_c1 600 python tools/bench_sg.py --config c1
step bench_pipe 600 python tools/bench_pipeline.py
step bench_pipe_concurrent 600 python tools/bench_pipeline.py --concurrent 8,16
step bench_pipe_concurrent_cache 600 python tools/bench_pipeline.py --concurrent 16 --parse-cache
step bench_pipe_concurrent_server 600 python tools/bench_pipeline.py --concurrent 16 --parse-cache --server --gather 0.5
fi
rc=0
if [ "${2:-}" != "no-profile" ] && [ "$part" = "all" ]; then  # (the profile set can run as its own call: bash tools/gpu_profile.sh <tag>)
  bash tools/gpu_profile.sh $tag > $O/profile.log 2>&1; rc=$?
  tail -5 $O/profile.log
fi
mkdir -p $O/out
for n in bench_c3 bench_c4 bench_c5 bench_c3_shard0of8 bench_c4_shard0of8 bench_c3_shard0of2 bench_c3_shard0of4 bench_c4_shard0of2 bench_c4_shard0of4 bench_c2 bench_c1 bench_pipe bench_pipe_concurrent; do
  [ -f $O/$n.log ] && grep '^{' $O/$n.log | tail -1 > $O/out/${tag}_$n.json
done
[ -f $O/phases_c3_shard0of8.log ] && grep -h "phases" $O/phases_c3_shard0of8.log > $O/out/${tag}_phases_c3_shard0of8.log
cp $O/host.txt $O/out/${tag}_host.txt
exit $rc
