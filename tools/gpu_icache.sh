# Instruction-cache requests and misses per kernel (two SQC counters with the
# SQ wave / instruction / fetch counts, one pass).
# usage: bash tools/gpu_icache.sh <tag> [bench args]
export TMPDIR=/tmp
tag=$1; shift
P=gpurun_out/$tag
mkdir -p $P
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH -d $P/ic -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $P/ic.log 2>&1
rc=$?
python3 tools/sq_summary.py $(find $P/ic -name "*.db" | head -1)
find $P -name "*.db" -delete
exit $rc
