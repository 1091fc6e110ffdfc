# Round profile: GPU parity tests, rocprofv3 kernel stats + HBM PMC passes of
# the default bench, the default bench line (with cpu_baseline), C3 and C5.
# usage (on the GPU box): TAG=round1b bash scripts/gpu_profile.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-latest}
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu_$T.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$T -o bench -- python bench.py --steps 4 --cpu-seconds 0 --no-counters > gpurun_out/stats_${T}_bench.json 2> gpurun_out/stats_$T.err || { echo "rocprof stats failed"; tail gpurun_out/stats_$T.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fetch_$T -o fetch -- python bench.py --steps 2 --cpu-seconds 0 --no-counters > gpurun_out/fetch_$T.json 2> gpurun_out/fetch_$T.err || { echo "pmc fetch failed"; tail gpurun_out/fetch_$T.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/write_$T -o write -- python bench.py --steps 2 --cpu-seconds 0 --no-counters > gpurun_out/write_$T.json 2> gpurun_out/write_$T.err || { echo "pmc write failed"; tail gpurun_out/write_$T.err; exit 1; }
python scripts/summarize_rocprof.py $T gpurun_out/stats_$T gpurun_out/fetch_$T gpurun_out/write_$T gpurun_out/stats_${T}_bench.json || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail gpurun_out/bench_$T.err; exit 1; }
for c in c3 c5; do
  timeout -k 10 500 python bench.py --config $c --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_${T}_$c.json 2> gpurun_out/bench_${T}_$c.err || { echo "$c failed"; tail -5 gpurun_out/bench_${T}_$c.err; exit 1; }
done
python - <<PY
import json
for f in ("bench_$T", "bench_${T}_c3", "bench_${T}_c5"):
    d = json.load(open(f"gpurun_out/{f}.json")); r = d["roofline"] or {}; c = d.get("cpu_baseline") or {}
    print(f, round(d["value"], 3), d["unit"], "ms/step", round(d["ms_per_step"], 1), "hbm_frac", r.get("frac"), "valu_frac", (r.get("valu") or {}).get("frac"), "traffic", r.get("traffic"), "cpu", c.get("value"))
PY
# the summaries written into profiles/ on the box travel back via gpurun_out/
mkdir -p gpurun_out/profiles && cp profiles/${T}_* profiles/pmc_latest.json gpurun_out/profiles/
