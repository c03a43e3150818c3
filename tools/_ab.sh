P=hygeia_amd/lib/var_nocheck/libhygeia_amd.so
bash tools/gpu_run.sh r05r --no-tests \
 "python tools/bench_sg.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python tools/bench_sg.py --no-cpu-baseline" \
 "python tools/bench_sg.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python tools/bench_sg.py --no-cpu-baseline"
