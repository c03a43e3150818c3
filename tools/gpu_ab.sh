# A/B of an environment knob on the C3 bench: gpu_ab.sh VAR v1 v2 ...
export TMPDIR=/tmp
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
env $var=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
python - "gpurun_out/ab_$v.log" "$var=$v" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d=json.loads(l); print(sys.argv[2], round(d["value"]), {k: round(v) for k, v in d["roofline"]["kernel_ms"].items()})
PY
done
