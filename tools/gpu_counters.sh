# Lists the PMC counters of the box (rocprofv3 -L) matching a pattern.
# usage: bash tools/gpu_counters.sh <tag> <grep -E pattern>
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1
grep -oE "$2" $O/avail.txt | sort -u
