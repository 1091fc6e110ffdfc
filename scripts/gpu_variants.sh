cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# profiling: C2 throughput of library variants (IPT_LIB_PATH) against the default build
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then L=ipt_amd/lib/libipt_hip.so; else L=ipt_amd/lib/abl/libipt_$v.so; fi
  IPT_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-counters > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/var_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print('variant $v', round(d['value'],2), 'Mpaths/s')"
done
