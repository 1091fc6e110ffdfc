# GPU parity tests (+ optional bench lines for the configs in $CONFIGS)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|Timeout" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for c in ${CONFIGS}; do
  timeout -k 10 500 python bench.py --config $c --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "$c failed"; tail -5 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));r=d['roofline'] or {};print('$c', round(d['value'],3), d['unit'], 'ms/step', round(d['ms_per_step'],1), 'hbm_frac', r.get('frac'), 'valu_frac', (r.get('valu') or {}).get('frac'))"
done
