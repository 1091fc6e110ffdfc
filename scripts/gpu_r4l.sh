# Round-4 checkpoint: the whole GPU suite, smoke, and the bench lines (CPU baselines included)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r4l_smoke.log; exit 1; }
tail -2 gpurun_out/r4l_smoke.log
T=round4l
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail gpurun_out/bench_$T.err; exit 1; }
for c in c3 c5; do
  timeout -k 10 500 python3 bench.py --config $c > gpurun_out/bench_${T}_$c.json 2> gpurun_out/bench_${T}_$c.err || { echo "$c failed"; tail -5 gpurun_out/bench_${T}_$c.err; exit 1; }
done
python3 - <<PY
import json, glob
for f in sorted(glob.glob("gpurun_out/bench_${T}*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); r = d["roofline"] or {}; c = d.get("cpu_baseline") or {}
    print(f, round(d["value"], 3), d["unit"], "ms/step", round(d["ms_per_step"], 1), "valu_frac", (r.get("valu") or {}).get("frac"), "cpu", c.get("value"), c.get("cores"), "1t", c.get("single_thread_paths_per_s"), "scal", c.get("thread_scaling"))
PY
cp gpurun_out/bench_${T}*.json gpurun_out/profiles/
