# Round 4 checkpoint: GPU suite, smoke, progressive callers, profiles (stats + PMC incl. DRAM) and bench lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4f_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/r4f_gpu.log; exit 1; }
tail -1 gpurun_out/r4f_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
TAG=round4f OUT_DIR=gpurun_out/profiles timeout -k 10 300 python -u scripts/progressive.py c3 c2 > gpurun_out/r4f_prog.log 2>&1 || { echo "progressive failed"; tail -20 gpurun_out/r4f_prog.log; exit 1; }
cat gpurun_out/r4f_prog.log
TAG=round4f CFGS="c2 c3 c5" bash scripts/gpu_profile.sh
