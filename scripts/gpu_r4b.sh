# C3 VGPR reduction + ds_permute owner search: sphere-list parity, then A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep_trees.py -x -q -m gpu --timeout 120 --timeout-method thread -k "spheres or sphere_grid or full_size or fractal or coincident or round_lights" > gpurun_out/r4b_parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/r4b_parity.log; exit 1; }
tail -1 gpurun_out/r4b_parity.log
VARIANTS="base default base default" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh
VARIANTS="base default" CONFIGS="c2" STEPS=1 bash scripts/gpu_variants_cfg.sh
