# C3 A/B: the wave walk's DDA step branch-free (IPT_GRID_WAVE_DDA_BF), then sphere parity with it
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default ddabf default ddabf" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
IPT_ABI_COMPAT=1 IPT_LIB_PATH=ipt_amd/lib/abl/libipt_ddabf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep_trees.py -x -q -m gpu --timeout 120 --timeout-method thread -k "spheres or sphere_grid or full_size or coincident" > gpurun_out/r4x_par.log 2>&1 || { tail -20 gpurun_out/r4x_par.log; exit 1; }
tail -1 gpurun_out/r4x_par.log
