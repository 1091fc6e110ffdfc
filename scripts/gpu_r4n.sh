# C2 timing diagnostic: raygen records read from a 512 KiB region (wrong images, timing only)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default rgm default rgm" CONFIGS="c2" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
