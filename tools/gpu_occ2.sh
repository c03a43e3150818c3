# two-group parity + C3 bench, then the forward per-step latency vs chains per CU
# (~256 / 512 / 768 chains of 25.6 M sites = 1, 2, 3 chains per CU)
# usage: bash tools/gpu_occ2.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
bash tools/gpu_tg.sh $tag || exit 1
for s in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --sites 25600000 --seeds $s > $O/occ_$s.log 2>&1 || { tail -5 $O/occ_$s.log; exit 1; }
grep '^{' $O/occ_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seeds', $s, d['config']['chains_per_gpu'], round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
done
