# Round measurements besides the default bench line: C4 1-GPU point, C5,
# single-group C2 / C2 + estimation / per-sample, pipeline-level drop-in.
# usage: bash tools/gpu_final2.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
run() { name=$1; shift; timeout -k 10 500 "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }; grep '^{' $O/$name.log | tail -1 | cut -c1-400; }
run c5 python bench.py --job c5 --steps 1 --warmup 1 --cpu-seconds 5
run c2 python tools/bench_sg.py
run c2pe python tools/bench_sg.py --estimate-parameters
run c2ps python tools/bench_sg.py --per-sample --no-cpu-baseline
run pipe python tools/bench_pipeline.py
