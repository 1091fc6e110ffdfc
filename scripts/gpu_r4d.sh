# Tail-overlap gating on the predecessor's unit counter: async tests, async vs sync benches, progressive callers
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_async.py -x -q --timeout 100 --timeout-method thread -m gpu > gpurun_out/r4d_async.log 2>&1 || { echo "async tests failed"; tail -30 gpurun_out/r4d_async.log; exit 1; }
tail -1 gpurun_out/r4d_async.log
for c in c3 c2 c5; do
  for m in "" "--sync"; do
    timeout -k 10 200 python bench.py --config $c --steps 2 --warmup 1 --cpu-seconds 0 --no-counters $m > gpurun_out/r4d_$c$m.json 2> gpurun_out/r4d_$c$m.err || { echo "bench $c $m failed"; tail -5 gpurun_out/r4d_$c$m.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4d_$c$m.json'));print('$c', '$m', round(d['value'],3), d['config']['calls'])"
  done
done
TAG=round4d OUT_DIR=gpurun_out/profiles timeout -k 10 300 python -u scripts/progressive.py c3 c2 > gpurun_out/r4d_prog.log 2>&1 || { echo "progressive failed"; tail -20 gpurun_out/r4d_prog.log; exit 1; }
cat gpurun_out/r4d_prog.log
