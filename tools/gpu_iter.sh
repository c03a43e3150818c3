# parity tests (two-group), phase timing at 2M sites, C3 bench (no CPU baseline)
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_two_group.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$tag.log 2>&1; rc=$?
tail -3 gpurun_out/t_$tag.log
[ $rc -eq 0 ] || exit 1
HYG_DEBUG_PHASES=1 timeout -k 10 200 python bench.py --sites 2000000 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/p_$tag.log 2>&1 || { tail -5 gpurun_out/p_$tag.log; exit 1; }
grep "phases" gpurun_out/p_$tag.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/b_$tag.log 2>&1 || { tail -5 gpurun_out/b_$tag.log; exit 1; }
python - "gpurun_out/b_$tag.log" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d=json.loads(l); print("C3", round(d["value"]), {k: round(v) for k, v in d["roofline"]["kernel_ms"].items()})
PY
