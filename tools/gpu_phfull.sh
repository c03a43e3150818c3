# per-step phase split (s_memtime ticks) of the forward and backward at full C3 occupancy (582 chains)
# usage: bash tools/gpu_phfull.sh <tag> [bench args...]
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
HYG_DEBUG_PHASES=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > $O/phfull.log 2>&1 || { tail -5 $O/phfull.log; exit 1; }
grep "phases" $O/phfull.log
