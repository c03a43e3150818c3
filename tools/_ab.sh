bash tools/gpu_run.sh r05e \
 "HYG_LIB_PATH=hygeia_amd/lib/var_tuning/libhygeia_amd.so HYG_SG_PHASES=1 python tools/bench_sg.py --no-cpu-baseline --sites 4000000" \
 "python tools/bench_sg.py --no-cpu-baseline" \
 "python tools/bench_sg.py --config c1 --no-cpu-baseline"
