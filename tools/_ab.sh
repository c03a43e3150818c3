P=hygeia_amd/lib/var_prev/libhygeia_amd.so
T=hygeia_amd/lib/var_tuning/libhygeia_amd.so
bash tools/gpu_run.sh r05u \
 "python tools/bench_sg.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python tools/bench_sg.py --no-cpu-baseline" \
 "python tools/bench_sg.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python tools/bench_sg.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$T HYG_SG_PHASES=1 python tools/bench_sg.py --no-cpu-baseline"
