cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# profiling: C2 throughput vs resident blocks per CU (latency vs issue bound)
for b in 4 3 2; do
  IPT_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-counters > gpurun_out/occ_$b.json 2>gpurun_out/occ_$b.err || { echo "bpc $b failed"; tail -3 gpurun_out/occ_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/occ_$b.json'));print('blocks/CU $b', round(d['value'],2), 'Mpaths/s')"
done
