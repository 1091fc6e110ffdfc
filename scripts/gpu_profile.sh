# Round profile: rocprofv3 kernel stats + PMC passes (HBM bytes, occupancy) of
# the bench for each config, then the bench lines themselves (the c2 line with
# its cpu_baseline). usage (on the GPU box): TAG=round3a CFGS="c2 c3 c5" bash scripts/gpu_profile.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-latest}
for c in ${CFGS:-c2 c3 c5}; do
  # (--sync: counter collection serialises the dispatches, and a launch gated
  # on its predecessor's pool -- a polling wait kernel, DESIGN.md 4.7 -- then
  # never starts; bench.py runs synchronous steps under any rocprofv3 anyway)
  B="python3 bench.py --config $c --steps 2 --warmup 1 --cpu-seconds 0 --no-counters --sync"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_${c}_stats -o run -- $B > gpurun_out/${T}_${c}_stats.json 2> gpurun_out/${T}_${c}_stats.err || { echo "$c stats failed"; tail gpurun_out/${T}_${c}_stats.err; exit 1; }
  for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
              "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE" \
              "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"; do
    n=$(echo $pass | cut -d' ' -f1-2 | tr ' ' '+')
    timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/${T}_${c}_pmc_$n -o run -- $B > gpurun_out/${T}_${c}_pmc_$n.json 2> gpurun_out/${T}_${c}_pmc_$n.err || { echo "$c pmc $n failed"; tail gpurun_out/${T}_${c}_pmc_$n.err; exit 1; }
  done
  python3 scripts/summarize_rocprof.py $T $c gpurun_out/${T}_${c}_stats.json gpurun_out/${T}_${c}_stats gpurun_out/${T}_${c}_pmc_* || exit 1
done
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail gpurun_out/bench_$T.err; exit 1; }
for c in ${CFGS:-c2 c3 c5}; do
  [ "$c" = c2 ] && continue
  timeout -k 10 500 python3 bench.py --config $c > gpurun_out/bench_${T}_$c.json 2> gpurun_out/bench_${T}_$c.err || { echo "$c failed"; tail -5 gpurun_out/bench_${T}_$c.err; exit 1; }
done
python3 - <<PY
import json, glob
for f in sorted(glob.glob("gpurun_out/bench_${T}*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); r = d["roofline"] or {}; c = d.get("cpu_baseline") or {}
    print(f, round(d["value"], 3), d["unit"], "ms/step", round(d["ms_per_step"], 1), "hbm_frac", r.get("frac"), "valu_frac", (r.get("valu") or {}).get("frac"), "occ", r.get("occupancy"), "traffic", r.get("traffic"), "cpu", c.get("value"), c.get("cores"))
PY
# the summaries written into profiles/ on the box travel back via gpurun_out/
mkdir -p gpurun_out/profiles && cp profiles/${T}_* profiles/pmc_latest_* gpurun_out/profiles/ && cp gpurun_out/bench_${T}*.json gpurun_out/profiles/
