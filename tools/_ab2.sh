set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 600 python -u -m pytest tests/test_gpu_single_group.py tests/test_gpu_sg_pe.py tests/test_gpu_single_group_cli.py tests/test_gpu_configs.py -k "not c5 and not c3" -x -v --timeout 300 --timeout-method thread > gpurun_out/r05o/tests.log 2>&1 && tail -3 gpurun_out/r05o/tests.log && timeout -k 10 300 python tools/bench_sg.py --no-cpu-baseline > gpurun_out/r05o/c2.json 2> gpurun_out/r05o/c2.err; echo rc=$?; tail -c 300 gpurun_out/r05o/c2.json
