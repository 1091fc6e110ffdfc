cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-counters"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/sqA -o a -- $B > gpurun_out/sqA.json 2>gpurun_out/sqA.err || { tail gpurun_out/sqA.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 --kernel-trace --output-format csv -d gpurun_out/sqB -o b -- $B > gpurun_out/sqB.json 2>gpurun_out/sqB.err || { tail gpurun_out/sqB.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH --kernel-trace --output-format csv -d gpurun_out/sqC -o c -- $B > gpurun_out/sqC.json 2>gpurun_out/sqC.err || { tail gpurun_out/sqC.err; exit 1; }
python scripts/pmc_sq.py gpurun_out/sqA gpurun_out/sqB gpurun_out/sqC
cat gpurun_out/sqA.json
