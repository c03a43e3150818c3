bash tools/gpu_run.sh r05g --no-tests \
 "python -u -m pytest tests/test_gpu_single_group.py tests/test_gpu_sg_pe.py tests/test_gpu_single_group_cli.py tests/test_gpu_configs.py -k 'not c3 and not c5' -x -q --timeout 600 --timeout-method thread" \
 "HYG_LIB_PATH=hygeia_amd/lib/var_tuning/libhygeia_amd.so HYG_SG_PHASES=1 python tools/bench_sg.py --no-cpu-baseline --sites 4000000" \
 "python tools/bench_sg.py --no-cpu-baseline" \
 "HYG_LIB_PATH=hygeia_amd/lib/var_tuning/libhygeia_amd.so HYG_DEBUG_PHASES=1 python bench.py --no-cpu-baseline --steps 1 --warmup 0"
