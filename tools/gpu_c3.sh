export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_c3_256.log 2>&1 && tail -1 gpurun_out/bench_c3_256.log &&
HYG_THREADS=512 timeout -k 10 600 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/bench_c3_512.log 2>&1 && tail -1 gpurun_out/bench_c3_512.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
echo DONE rc=$?
