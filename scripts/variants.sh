#!/usr/bin/env bash
# Experiment builds: sample_scenes[0]-only libraries (IPT_C2_ONLY) with extra
# -D flags, into ipt_amd/lib/abl/libipt_<name>.so.
# usage: bash scripts/variants.sh name1 "-DFOO=1" name2 "-DBAR=2 -DBAZ=0" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p ipt_amd/lib/abl
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-memory-clause \
    -Wno-unused-value -DIPT_AB_BUILD -DIPT_C2_ONLY=1 $f -o ipt_amd/lib/abl/libipt_$n.so ipt_amd/csrc/ipt_kernels.hip ipt_amd/csrc/ipt_post.hip &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "variant build failed"; exit 1; }; done
ls ipt_amd/lib/abl
