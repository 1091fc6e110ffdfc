# A/B: raygen records read at the refill (IPT_RG_EARLY) vs the head, C2 / C5 / C3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default rge default rge" CONFIGS="c2 c5 c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
