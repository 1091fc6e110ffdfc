# Round 4: C3 VGPR/owner-search changes + two work slots (queued renders).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4c_async.log 2>&1 || { echo "async tests failed"; tail -40 gpurun_out/r4c_async.log; exit 1; }
tail -2 gpurun_out/r4c_async.log
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4c_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/r4c_gpu.log; exit 1; }
tail -2 gpurun_out/r4c_gpu.log
BENCH_EXTRA=--sync VARIANTS="base default base default" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
VARIANTS="default" CONFIGS="c3 c2 c5" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
TAG=round4c OUT_DIR=gpurun_out/profiles timeout -k 10 300 python -u scripts/progressive.py c3 c2 > gpurun_out/r4c_prog.log 2>&1 || { echo "progressive failed"; tail -20 gpurun_out/r4c_prog.log; exit 1; }
cat gpurun_out/r4c_prog.log
