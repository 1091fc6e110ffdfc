cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -x -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py ${BENCH_ARGS:---cpu-seconds 0} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open('gpurun_out/bench.json'))
r=d['roofline'] or {}
print('value', round(d['value'],2), 'Mpaths/s', 'ms/step', round(d['ms_per_step'],1), 'frac', r.get('frac'), 'launch_ms', r.get('launch_ms'))
PY
