# C3 A/B: the next cell located inside the first round's item-load latency (IPT_GRID_WAVE_DDA_LATE)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default ddal default ddal" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
