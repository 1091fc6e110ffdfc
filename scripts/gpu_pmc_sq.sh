# SQ counters of path_kernel per config (issue / wait / lane-utilisation
# breakdown), three passes of at most 8 SQ counters each.
# usage (on the GPU box): TAG=round3b CFGS="c2 c3" bash scripts/gpu_pmc_sq.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-latest}
for c in ${CFGS:-c2 c3 c5}; do
  B="python3 bench.py --config $c --steps 1 --warmup 0 --cpu-seconds 0 --no-counters"
  i=0
  for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS" \
              "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_IFETCH SQ_INST_CYCLES_SALU" \
              "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT" \
              "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/sq_${T}_${c}_$i -o run -- $B > gpurun_out/sq_${T}_${c}_$i.json 2> gpurun_out/sq_${T}_${c}_$i.err || { echo "$c pass $i failed"; tail -5 gpurun_out/sq_${T}_${c}_$i.err; exit 1; }
  done
  python3 scripts/pmc_sq.py gpurun_out/sq_${T}_${c}_* > gpurun_out/sq_${T}_${c}.json || exit 1
  python3 - <<PY
import json
d = json.load(open("gpurun_out/sq_${T}_${c}.json"))
b = json.loads(open("gpurun_out/sq_${T}_${c}_1.json").read().strip().splitlines()[-1])
paths = b["config"]["width"] * b["config"]["height"] * b["config"]["spp_per_step"]
out = {"config": "$c", "paths_per_launch": paths, "per_path": {k: v / paths for k, v in d.items()}, "raw": d}
wc = d.get("SQ_WAVE_CYCLES", 0)
if wc:
    out["wave_cycle_shares"] = {k: d[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in d}
if d.get("SQ_ACTIVE_INST_VALU"):
    out["valu_lane_utilisation"] = d.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * d["SQ_ACTIVE_INST_VALU"])
json.dump(out, open("gpurun_out/sq_${T}_${c}_summary.json", "w"), indent=1)
print("$c", json.dumps({k: out.get(k) for k in ("wave_cycle_shares", "valu_lane_utilisation")}),
      {k: round(v, 1) for k, v in out["per_path"].items()})
PY
done
