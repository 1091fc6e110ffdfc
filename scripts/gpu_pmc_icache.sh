# PMC: instruction cache, LDS waits/conflicts and SQ basics for the C2 path kernel (profiling)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=${IPT_LIB_PATH:-ipt_amd/lib/libipt_hip.so}
T=${TAG:-ic}
B="python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-counters"
IPT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d gpurun_out/${T}_1 -o a -- $B > /dev/null 2>gpurun_out/${T}_1.err || { tail gpurun_out/${T}_1.err; exit 1; }
IPT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/${T}_2 -o a -- $B > /dev/null 2>gpurun_out/${T}_2.err || { tail gpurun_out/${T}_2.err; exit 1; }
IPT_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/${T}_3 -o a -- $B > /dev/null 2>gpurun_out/${T}_3.err || { tail gpurun_out/${T}_3.err; exit 1; }
python - <<PY
import csv, glob
tot = {}
for d in ("gpurun_out/${T}_1", "gpurun_out/${T}_2", "gpurun_out/${T}_3"):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "path_kernel" not in r.get("Kernel_Name", ""): continue
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot): print(f"{k:28s} {tot[k]:.4g}")
PY
