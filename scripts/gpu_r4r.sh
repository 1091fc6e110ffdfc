# C2 layout probe: frame-column stride 264 vs 320, three vs four stack levels (n_rays 8 and 16)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default s4x264 s3x320 default s4x264 s3x320" CONFIGS="c2" STEPS=2 BENCH_EXTRA="--n-rays 8" bash scripts/gpu_variants_cfg.sh || exit 1
VARIANTS="default s4x264 default s4x264" CONFIGS="c2" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
