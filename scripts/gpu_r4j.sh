# C3: range-free root in the wave walk's sphere tests (IPT_LIST_ROOT): parity, A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep_trees.py -x -q -m gpu --timeout 120 --timeout-method thread -k "spheres or sphere_grid or full_size or coincident" > gpurun_out/r4j_par.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/r4j_par.log; exit 1; }
tail -1 gpurun_out/r4j_par.log
VARIANTS="noroot default noroot default" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
