# Round profile set: full C3 bench (with the CPU baseline), rocprofv3 kernel
# trace + stats, HBM PMC passes (FETCH_SIZE, WRITE_SIZE), SQ counters.
# Summaries go to gpurun_out/prof_<tag>/ (the large databases are deleted).
export TMPDIR=/tmp
tag=$1
P=gpurun_out/prof_$tag
mkdir -p $P
timeout -k 10 900 python bench.py > $P/bench.log 2>&1 && grep '^{' $P/bench.log | tail -1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/trace -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/trace.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $P/sq -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/sq.log 2>&1
rc=$?
python3 tools/prof_summary.py ${tag} $(find $P/trace -name "*.db" | head -1) $(find $P/fetch -name "*.db" | head -1) $(find $P/write -name "*.db" | head -1) > $P/summary.txt 2>&1
python3 tools/sq_summary.py $(find $P/sq -name "*.db" | head -1) > $P/sq_summary.txt 2>&1
cp profiles/${tag}_kernel_stats.csv profiles/${tag}_pmc.csv profiles/pmc_traffic.json $P/ 2>/dev/null
find $P -name "*.db" -delete; find $P -name "*.csv" -size +2M -delete
cat $P/summary.txt $P/sq_summary.txt
echo "rc=$rc"
