cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
echo "list rc=$? lines=$(wc -l < gpurun_out/pmc_list.txt)"
for bpc in 3 2 1; do
  IPT_BLOCKS_PER_CU=$bpc timeout -k 10 300 python bench.py --config c3 --steps 1 --warmup 1 --cpu-seconds 0 --no-counters > gpurun_out/r3e_bpc$bpc.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r3e_bpc$bpc.json'));print('c3 bpc $bpc', round(d['value'],3))"
done
VARIANTS="default inl" CONFIGS=c3 STEPS=1 bash scripts/gpu_variants_cfg.sh
