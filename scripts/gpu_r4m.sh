# C2 timing diagnostic: frame-table / CosineDdf gathers confined to 512 KiB (wrong images, timing only)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default fm cm fcm default fm cm fcm" CONFIGS="c2" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
