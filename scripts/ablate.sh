#!/usr/bin/env bash
# Profiling-only: build the "duplicate one phase" variants into ipt_amd/lib/abl/.
set -e
cd "$(dirname "$0")/.."
mkdir -p ipt_amd/lib/abl
for n in 0 1 2 3 4 5 6 7; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -Wno-unused-value -DIPT_ABL=$n -o ipt_amd/lib/abl/libipt_abl$n.so ipt_amd/csrc/ipt_kernels.hip &
done
wait
ls ipt_amd/lib/abl
