# instruction-cache / fetch counters of the two-group kernels (142 chains, 6 M sites)
# usage: bash tools/gpu_icache.sh <tag>
export TMPDIR=/tmp
tag=$1
P=gpurun_out/$tag
mkdir -p $P
B="python3 bench.py --sites 6000000 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE -d $P/ic -o run --output-format csv -- $B > $P/ic.log 2>&1
rc=$?
f=$(find $P/ic -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
    tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(tot.items()):
    if "tg_" in k: print(f"{k:24s} {c:30s} {v:.4g}")
PY
find $P -name "*.csv" -size +2M -delete
echo rc=$rc
exit $rc
