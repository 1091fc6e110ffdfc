# Round 4, first GPU call: the new deep/non-power-of-two parity tests, the
# whole GPU suite, the shard-balance measurement, then the C2 profile with
# the DRAM counter passes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_deep_trees.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4a_deep.log 2>&1 || { echo "deep tests failed"; tail -30 gpurun_out/r4a_deep.log; exit 1; }
tail -3 gpurun_out/r4a_deep.log
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r4a_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/r4a_gpu.log; exit 1; }
tail -3 gpurun_out/r4a_gpu.log
TAG=round4a OUT_DIR=gpurun_out/profiles timeout -k 10 300 python -u scripts/shard_balance.py c4 c5 > gpurun_out/r4a_shard.log 2>&1 || { echo "shard balance failed"; tail -20 gpurun_out/r4a_shard.log; exit 1; }
tail -2 gpurun_out/r4a_shard.log
TAG=round4a CFGS="c2" bash scripts/gpu_profile.sh
