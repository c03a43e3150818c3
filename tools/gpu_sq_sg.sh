# SQ instruction / wait counters of the single-group chain kernel (C2 workload at $2 sites)
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1
sites=${2:-2800000}
summ() {
  db=$(find $1 -name '*.db' | head -1)
  python3 tools/sq_summary.py "$db" sg_ > $1.txt && rm -rf $1 && cat $1.txt
}
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/sqsg_$tag -o run -- python3 tools/bench_sg.py --sites $sites --no-cpu-baseline > gpurun_out/sqsg_$tag.log 2>&1 || { tail -20 gpurun_out/sqsg_$tag.log; exit 1; }
summ gpurun_out/sqsg_$tag
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_FLAT -d gpurun_out/sqsg2_$tag -o run -- python3 tools/bench_sg.py --sites $sites --no-cpu-baseline > gpurun_out/sqsg2_$tag.log 2>&1 || { tail -20 gpurun_out/sqsg2_$tag.log; exit 1; }
summ gpurun_out/sqsg2_$tag
