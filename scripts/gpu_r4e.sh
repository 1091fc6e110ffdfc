# 64 / 128-thread workgroups (finer slot release in launch tails): parity, then A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in b64 b128; do
  IPT_LIB_PATH=ipt_amd/lib/abl/libipt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py -x -q -m gpu --timeout 120 --timeout-method thread -k "spheres or sphere_grid or full_size or queued or values_bit_exact_box or light_grid or c1_config" > gpurun_out/r4e_par_$v.log 2>&1 || { echo "parity $v failed"; tail -20 gpurun_out/r4e_par_$v.log; exit 1; }
  tail -1 gpurun_out/r4e_par_$v.log
done
VARIANTS="default b64 b128 default b64" CONFIGS="c3 c2 c5" STEPS=2 bash scripts/gpu_variants_cfg.sh || exit 1
IPT_LIB_PATH=ipt_amd/lib/abl/libipt_b64.so TAG=round4e_b64 OUT_DIR=gpurun_out/profiles timeout -k 10 300 python -u scripts/progressive.py c3 c2 > gpurun_out/r4e_prog.log 2>&1 || { echo "progressive failed"; tail -20 gpurun_out/r4e_prog.log; exit 1; }
cat gpurun_out/r4e_prog.log
