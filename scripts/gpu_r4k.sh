# C3 A/B: frame-angle table for the sphere lists, walk budget 6 / 12
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default ftab lag lagbf bf b6 b12 default ftab lag lagbf bf b6 b12" CONFIGS="c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
