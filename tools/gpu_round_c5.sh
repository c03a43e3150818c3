# the round's final GPU call: tools/gpu_round.sh (parity tests, C3 line with CPU
# baselines, C4 1-GPU point, profile set), then the C5 line
# usage: bash tools/gpu_round_c5.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
bash tools/gpu_round.sh $tag || exit 1
timeout -k 10 500 python bench.py --job c5 --steps 1 --warmup 1 --cpu-seconds 5 > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log | tail -1 | cut -c1-400
