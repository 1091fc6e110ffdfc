# Round 4: async tests again (idle slots), then profiles (stats + PMC incl. DRAM, synchronous steps) and bench lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -m gpu -k "queued or interleaved or upload or chunked or counters or values_bit_exact_box" > gpurun_out/r4g_async.log 2>&1 || { echo "async tests failed"; tail -30 gpurun_out/r4g_async.log; exit 1; }
tail -1 gpurun_out/r4g_async.log
TAG=round4g CFGS="c2 c3 c5" bash scripts/gpu_profile.sh
