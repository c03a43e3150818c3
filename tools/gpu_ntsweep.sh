# C3 bench for forward/backward workgroup-size combinations
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_two_group.py -x -q > gpurun_out/t_sw.log 2>&1 || { tail -5 gpurun_out/t_sw.log; exit 1; }
tail -1 gpurun_out/t_sw.log
for combo in "256 256" "512 256" "512 128" "256 128"; do
set -- $combo
HYG_THREADS_FWD=$1 HYG_THREADS_BWD=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/b_sw_$1_$2.log 2>&1 || { tail -5 gpurun_out/b_sw_$1_$2.log; exit 1; }
python - "gpurun_out/b_sw_$1_$2.log" "$1/$2" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d=json.loads(l); print(sys.argv[2], round(d["value"]), {k: round(v) for k, v in d["roofline"]["kernel_ms"].items()})
PY
done
