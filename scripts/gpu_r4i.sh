# C3 re-sweep at 64-thread workgroups (walk budget, grid resolution) + N=2 rehearsal with queued steps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default bud6 bud12 cps12 cps20 default" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
bash scripts/gpu_r4h.sh
