# Round profile set for one bench workload: rocprofv3 kernel trace + stats, the
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes), the SQ instruction /
# wait counters with GRBM_GUI_ACTIVE (clock). Summaries -> profiles/ via
# tools/prof_summary.py (tagged with the kernel build); large databases deleted.
# usage: bash tools/gpu_profile.sh <tag> [bench args...]
export TMPDIR=/tmp
tag=$1; shift
P=gpurun_out/prof_$tag
mkdir -p $P
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $*"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/trace -o run -- $B > $P/trace.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- $B > $P/fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- $B > $P/write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $P/sq -o run -- $B > $P/sq.log 2>&1
rc=$?
db() { find $P/$1 -name "*.db" | head -1; }
python3 tools/prof_summary.py --tag $tag --trace $(db trace) --fetch $(db fetch) --write $(db write) --sq $(db sq) --bench-log $P/trace.log > $P/summary.txt 2>&1
cp profiles/${tag}_kernel_stats.csv profiles/${tag}_pmc.csv profiles/${tag}_sq_summary.txt profiles/pmc_traffic.json profiles/pmc_issue.json $P/ 2>/dev/null
find $P -name "*.db" -delete; find $P -name "*.csv" -size +2M -delete
cat $P/summary.txt
echo "rc=$rc"
exit $rc
