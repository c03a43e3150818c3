T=hygeia_amd/lib/var_tuning/libhygeia_amd.so
bash tools/gpu_run.sh r05h --no-tests \
 "HYG_LIB_PATH=$T HYG_DEBUG_PHASES=1 python bench.py --job c5 --steps 1 --warmup 0 --no-cpu-baseline" \
 "HYG_LIB_PATH=$T HYG_THREADS_FWD=768 python bench.py --job c5 --steps 1 --warmup 1 --no-cpu-baseline" \
 "HYG_LIB_PATH=$T python bench.py --job c5 --steps 1 --warmup 1 --no-cpu-baseline"
