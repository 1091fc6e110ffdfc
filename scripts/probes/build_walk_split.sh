#!/usr/bin/env bash
# Builds the split-traversal probe (scripts/probes/walk_split.hip): the product
# sources with the IPT_RAYLOG hook plus the probe's traversal kernel, as one
# library that also exports the C-ABI (loaded through IPT_LIB_PATH).
set -e
cd "$(dirname "$0")/../.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-memory-clause -Wno-unused-value \
  -DIPT_DIAGNOSTIC_BUILD -DIPT_RAYLOG=1 -Rpass-analysis=kernel-resource-usage \
  -o scripts/probes/libipt_walksplit.so scripts/probes/walk_split.hip ipt_amd/csrc/ipt_post.hip \
  2> scripts/probes/walk_split.resources.txt
grep -A12 "walk_split_kernel" scripts/probes/walk_split.resources.txt | grep -E "Function Name|VGPRs:|Occupancy|ScratchSize" || true
