# rehearsal of bench.py's multi-rank path on a one-GPU box: 2 ranks on cuda:0 over gloo
# (everything but RCCL itself: init, barriers, sharding, counts all-reduce, max-over-ranks timing)
# usage: bash tools/gpu_dist.sh <tag>
export TMPDIR=/tmp
tag=$1
O=gpurun_out/$tag
mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517"
timeout -k 10 400 $R bench.py --gpus 2 --steps 1 --warmup 0 --sites 2000000 --dist-backend gloo --no-cpu-baseline > $O/c3_w2.log 2>&1 || { tail -20 $O/c3_w2.log; exit 1; }
grep '^{' $O/c3_w2.log | tail -1
timeout -k 10 400 $R bench.py --gpus 2 --job c4 --steps 1 --warmup 0 --sites 2000000 --dist-backend gloo --no-cpu-baseline > $O/c4_w2.log 2>&1 || { tail -20 $O/c4_w2.log; exit 1; }
grep '^{' $O/c4_w2.log | tail -1
