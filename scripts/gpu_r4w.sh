# Final round-4 profiles: rocprof stats + PMC passes (DRAM split, occupancy) and bench lines for C2 / C3 / C5
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=round4w CFGS="c2 c3 c5" bash scripts/gpu_profile.sh
