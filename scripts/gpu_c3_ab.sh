# Per-config A/B: parity tests (PARITY_K, default the sphere-list ones) against
# each variant library, then throughput (CONFIGS, default c3).
# usage (GPU box): VARIANTS="f4 f4x2" [CONFIGS=c5 PARITY_K="light_grid"] bash scripts/gpu_c3_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  IPT_LIB_PATH=ipt_amd/lib/abl/libipt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
    --timeout 120 --timeout-method thread -k "${PARITY_K:-spheres_in_box or sphere_grid or full_size}" > gpurun_out/c3ab_pytest_$v.log 2>&1 \
    || { echo "parity $v failed"; tail -20 gpurun_out/c3ab_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/c3ab_pytest_$v.log
done
VARIANTS="default ${VARIANTS}" CONFIGS=${CONFIGS:-c3} STEPS=${STEPS:-2} bash scripts/gpu_variants_cfg.sh
