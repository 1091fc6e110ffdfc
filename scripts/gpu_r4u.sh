# Uniform-region structurization adopted: the whole GPU suite, smoke, then A/B against the previous build (C2, C3, C5)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4u_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r4u_smoke.log; exit 1; }
tail -1 gpurun_out/r4u_smoke.log
VARIANTS="default prev default prev" CONFIGS="c2 c3 c5" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
