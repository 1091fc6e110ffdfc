# PMC: L1/L2 hit rates and L1->L2 read latency of the path kernel for $CFG (profiling)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${CFG:-c3}
B="python bench.py --config $C --steps 1 --warmup 0 --cpu-seconds 0 --no-counters"
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d gpurun_out/cache_${C}_1 -o a -- $B > /dev/null 2>gpurun_out/cache_${C}_1.err || { tail gpurun_out/cache_${C}_1.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/cache_${C}_2 -o a -- $B > /dev/null 2>gpurun_out/cache_${C}_2.err || { tail gpurun_out/cache_${C}_2.err; exit 1; }
python - <<PY
import csv, glob
tot = {}
for d in ("gpurun_out/cache_${C}_1", "gpurun_out/cache_${C}_2"):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "path_kernel" not in r.get("Kernel_Name", ""): continue
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot): print(f"{k:32s} {tot[k]:.4g}")
if tot.get("TCC_HIT_sum") is not None:
    print("L2 hit rate", tot["TCC_HIT_sum"] / max(1, tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"]))
    print("avg L1->L2 read latency (cycles)", tot.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / max(1, tot.get("TCP_TCC_READ_REQ_sum", 1)))
PY
