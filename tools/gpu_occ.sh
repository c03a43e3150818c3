# C5 parity (auto thread count) + forward per-step latency vs chains per CU
# usage: bash tools/gpu_occ.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k c5 > $O/t_c5.log 2>&1 || { tail -30 $O/t_c5.log; exit 1; }
tail -1 $O/t_c5.log
# ~256 / 512 / 768 chains: 1, 2, 3 chains per CU (longest first)
for cfg in "25600000 1" "25600000 2" "25600000 3"; do
set -- $cfg
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --sites $1 --seeds $2 > $O/occ_$2.log 2>&1 || { tail -5 $O/occ_$2.log; exit 1; }
grep '^{' $O/occ_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seeds', $2, d['config']['chains_per_gpu'], round(d['value']), {k: round(v) for k, v in d['roofline']['kernel_ms'].items()})"
done
