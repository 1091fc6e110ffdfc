#!/usr/bin/env bash
# Profiling-only: build the per-phase lane-utilisation variant (-DIPT_PROF=1)
# and the step-segment stamp variant (-DIPT_STAMP=1) into ipt_amd/lib/abl/. Run with scripts/prof_phases.py on a GPU.
set -e
cd "$(dirname "$0")/.."
mkdir -p ipt_amd/lib/abl
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-memory-clause -Wno-unused-value"
/opt/rocm/bin/hipcc $F -DIPT_DIAGNOSTIC_BUILD -DIPT_PROF=1 -o ipt_amd/lib/abl/libipt_prof.so ipt_amd/csrc/ipt_kernels.hip ipt_amd/csrc/ipt_post.hip &
/opt/rocm/bin/hipcc $F -DIPT_DIAGNOSTIC_BUILD -DIPT_STAMP=1 -o ipt_amd/lib/abl/libipt_stamp.so ipt_amd/csrc/ipt_kernels.hip ipt_amd/csrc/ipt_post.hip &
wait
