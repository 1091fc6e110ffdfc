# Code-generation flags A/B (C2, C3): uniform-region structurization, AMDGPU RP trackers, schedule metric bias
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default sku trk skr mb0 default sku trk skr mb0" CONFIGS="c2 c3" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
