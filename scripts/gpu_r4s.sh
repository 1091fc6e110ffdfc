# C2 A/B: compact LDS layout (16-bit stack meta, 9-row frames) at 5 waves per SIMD
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default cmp cmpnh cmp4 default cmp cmpnh cmp4" CONFIGS="c2" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
