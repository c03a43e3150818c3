V=hygeia_amd/lib/var_bitonic/libhygeia_amd.so
bash tools/gpu_run.sh r05b \
 "python bench.py --shard 0/8 --no-cpu-baseline --steps 2" \
 "HYG_LIB_PATH=$V python bench.py --shard 0/8 --no-cpu-baseline --steps 2" \
 "python bench.py --shard 0/8 --no-cpu-baseline --steps 2" \
 "HYG_LIB_PATH=$V python bench.py --shard 0/8 --no-cpu-baseline --steps 2" \
 "python bench.py --job c5 --steps 1 --warmup 1 --no-cpu-baseline" \
 "HYG_LIB_PATH=$V python bench.py --job c5 --steps 1 --warmup 1 --no-cpu-baseline" \
 "HYG_LIB_PATH=hygeia_amd/lib/var_tuning/libhygeia_amd.so HYG_DEBUG_PHASES=1 python bench.py --shard 0/8 --no-cpu-baseline --steps 1 --warmup 0" \
 "HYG_LIB_PATH=hygeia_amd/lib/var_tunbit/libhygeia_amd.so HYG_DEBUG_PHASES=1 python bench.py --shard 0/8 --no-cpu-baseline --steps 1 --warmup 0"
