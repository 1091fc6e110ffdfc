# SQ / TCC counters of the stand-alone traversal kernel (walk_split_kernel) at
# the megakernel's occupancy (4 waves per SIMD) and at 8, per traced ray.
# usage (GPU box, after scripts/probes/build_walk_split.sh here):
#   bash scripts/probes/walk_split_sq.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "4,4,8" "8,8,8"; do
  t=w${cfg//,/_}
  i=0
  for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS" \
              "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_IFETCH SQ_INST_CYCLES_SALU" \
              "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
    i=$((i+1))
    WALK_RUNS=$cfg WALK_REPS=1 timeout -s KILL 240 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/wsq_${t}_$i -o run -- python3 scripts/probes/walk_split.py > gpurun_out/wsq_${t}_$i.jsonl 2> gpurun_out/wsq_${t}_$i.err || { echo "$cfg pass $i failed"; tail -5 gpurun_out/wsq_${t}_$i.err; exit 1; }
  done
  PMC_KERNEL=walk_split_kernel python3 scripts/pmc_sq.py gpurun_out/wsq_${t}_* > gpurun_out/wsq_${t}.json || exit 1
  python3 - <<PY
import json
d = json.load(open("gpurun_out/wsq_${t}.json"))
lines = [json.loads(l) for l in open("gpurun_out/wsq_${t}_1.jsonl")]
rays = lines[-1]["rays"]
out = {"config": "$cfg (wps, workgroups per CU, walk budget)", "rays": rays, "per_ray": {k: v / rays for k, v in d.items()},
       "raw": d}
wc = d.get("SQ_WAVE_CYCLES", 0)
if wc:
    out["wave_cycle_shares"] = {k: d[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in d}
if d.get("SQ_ACTIVE_INST_VALU"):
    out["valu_lane_utilisation"] = d.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * d["SQ_ACTIVE_INST_VALU"])
json.dump(out, open("gpurun_out/wsq_${t}_summary.json", "w"), indent=1)
print("$cfg", json.dumps({k: out.get(k) for k in ("wave_cycle_shares", "valu_lane_utilisation")}),
      {k: round(v, 2) for k, v in out["per_ray"].items()})
PY
done
