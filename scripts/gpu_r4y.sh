# C3 walk budget 7 / 9 / 10 cells per step with the final build flags
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default b7 b9 b10 default b7 b9 b10" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
