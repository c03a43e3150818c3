# SQ instruction / wait counters of the chain kernels (C3 workload, one step)
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/sq_$tag -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/sq_$tag.log 2>&1 || { tail -20 gpurun_out/sq_$tag.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU -d gpurun_out/sq2_$tag -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/sq2_$tag.log 2>&1 || { tail -20 gpurun_out/sq2_$tag.log; exit 1; }
echo ok
