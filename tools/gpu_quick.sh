# parity tests + C3 bench at the given thread counts (no CPU baseline)
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 400 python -m pytest tests/test_gpu_two_group.py -x -q > gpurun_out/t_$tag.log 2>&1; rc=$?
tail -2 gpurun_out/t_$tag.log
[ $rc -eq 0 ] || exit 1
for nt in "$@"; do
HYG_THREADS=$nt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/b_${tag}_$nt.log 2>&1 || { tail -5 gpurun_out/b_${tag}_$nt.log; exit 1; }
python - "gpurun_out/b_${tag}_$nt.log" "$nt" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d=json.loads(l); print("NT", sys.argv[2], round(d["value"]), {k: round(v) for k, v in d["roofline"]["kernel_ms"].items()})
PY
done
