cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo | grep -m3 -E "gfx9|Marketing" > gpurun_out/rocminfo.txt
nproc > gpurun_out/nproc.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/nproc.txt
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu1.log 2>&1
rc=$?
echo "pytest exit $rc"
tail -30 gpurun_out/pytest_gpu1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python tests/perf_probe.py 1024 4 > gpurun_out/perf1.log 2>&1; echo "perf exit $?"; cat gpurun_out/perf1.log
fi
