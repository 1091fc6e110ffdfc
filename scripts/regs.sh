#!/usr/bin/env bash
# Register / spill / LDS report of the path_kernel instances (extra hipcc flags as args)
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-memory-clause -Wno-unused-value \
  --cuda-device-only -c ipt_amd/csrc/ipt_kernels.hip -o /tmp/ipt_regs.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 \
  | grep -E "Function Name|VGPRs:|ScratchSize|Occupancy|SGPRs:|Spill|LDS" \
  | sed -E 's/.*remark: //; s/\[-Rpass.*//; s/.*hip:[0-9]+:[0-9]+: +//' | paste - - - - - - - - | grep path_kernel \
  | sed -E 's/Function Name: _ZN12_GLOBAL__N_111path_kernelI//; s/EEvNS_7KParamsE//; s/ \[bytes\/[a-z]+\]//g' | awk '{$1=$1};1'
