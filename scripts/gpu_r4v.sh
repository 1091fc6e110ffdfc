# Code-generation flags A/B, second set (C3, C2): relaxed occupancy, no high-RP reschedule, long-branch factor 0, kernarg preload
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="default rlx nohrp lbf0 kpl default rlx nohrp lbf0 kpl" CONFIGS="c3 c2" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
