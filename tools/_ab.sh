P=hygeia_amd/lib/var_prev/libhygeia_amd.so
bash tools/gpu_run.sh r05p \
 "python bench.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python bench.py --no-cpu-baseline" \
 "python bench.py --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python bench.py --no-cpu-baseline" \
 "python bench.py --job c4 --steps 1 --warmup 1 --no-cpu-baseline" \
 "HYG_LIB_PATH=$P python bench.py --job c4 --steps 1 --warmup 1 --no-cpu-baseline"
