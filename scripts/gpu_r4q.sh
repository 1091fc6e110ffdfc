# C2-shaped occupancy probe (n_rays 8: three stack levels, 30.4 KiB LDS per workgroup): 4 vs 5 waves per SIMD, 8 steps each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default s3w4 s3w5 s3w5nh s3w4nh default s3w4 s3w5 s3w5nh s3w4nh default s3w4 s3w5 s3w5nh s3w4nh" CONFIGS="c2" STEPS=8 BENCH_EXTRA="--n-rays 8" bash scripts/gpu_variants_cfg.sh || exit 1
