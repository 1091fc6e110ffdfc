# PMC: LDS activity of the path kernel for $CFG (profiling; is a walk LDS-bound?)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${CFG:-c5}
B="python bench.py --config $C --steps 1 --warmup 0 --cpu-seconds 0 --no-counters"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/lds_${C} -o a -- $B > /dev/null 2>gpurun_out/lds_${C}.err || { tail gpurun_out/lds_${C}.err; exit 1; }
python scripts/pmc_sq.py gpurun_out/lds_${C}
