P=hygeia_amd/lib/var_prev/libhygeia_amd.so
bash tools/gpu_run.sh r05q \
 "python bench.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python bench.py --no-cpu-baseline" \
 "python bench.py --shard 0/8 --no-cpu-baseline --steps 2" \
 "HYG_LIB_PATH=$P python bench.py --shard 0/8 --no-cpu-baseline --steps 2" \
 "python bench.py --job c5 --steps 1 --warmup 1 --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python bench.py --job c5 --steps 1 --warmup 1 --no-cpu-baseline"
