export TMPDIR=/tmp
mkdir -p gpurun_out
HYG_THREADS=64 timeout -k 10 400 python -m pytest tests/test_gpu_two_group.py -x -q > gpurun_out/t8.log 2>&1; echo RC=$? >> gpurun_out/t8.log; tail -2 gpurun_out/t8.log
grep -q "RC=0" gpurun_out/t8.log || exit 1
for nt in 64 128; do
HYG_THREADS=$nt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/b8_$nt.log 2>&1 || exit 1
python - "$nt" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/b8_{sys.argv[1]}.log") if x.startswith("{")][-1]
d=json.loads(l); print(sys.argv[1], round(d["value"]), d["roofline"]["kernel_ms"])
PY
done
