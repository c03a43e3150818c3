P=hygeia_amd/lib/var_prev/libhygeia_amd.so
T=hygeia_amd/lib/var_tuning/libhygeia_amd.so
bash tools/gpu_run.sh r05n \
 "python tools/bench_sg.py" \
 "HYG_LIB_PATH=$P python tools/bench_sg.py" \
 "python tools/bench_sg.py --config c1" \
 "HYG_LIB_PATH=$P python tools/bench_sg.py --config c1" \
 "HYG_LIB_PATH=$T HYG_SG_PHASES=1 python tools/bench_sg.py" \
 "HYG_LIB_PATH=hygeia_amd/lib/var_prevtune/libhygeia_amd.so HYG_SG_PHASES=1 python tools/bench_sg.py"
