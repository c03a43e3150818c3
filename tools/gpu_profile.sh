# Round profile set: full C3 bench (with the CPU baseline), rocprofv3 kernel
# trace + stats (csv), HBM PMC passes (FETCH_SIZE, WRITE_SIZE), SQ counters.
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/prof_$tag
timeout -k 10 900 python bench.py > gpurun_out/prof_$tag/bench.log 2>&1 && grep '^{' gpurun_out/prof_$tag/bench.log | tail -1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/prof_$tag/trace -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$tag/trace.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$tag/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$tag/fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$tag/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$tag/write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/prof_$tag/sq -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$tag/sq.log 2>&1
echo "rc=$?"
find gpurun_out/prof_$tag -name "*.csv" | head
