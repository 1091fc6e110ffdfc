# variants x configs throughput (profiling): VARIANTS, CONFIGS, STEPS
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in ${CONFIGS:-c2}; do
for v in ${VARIANTS}; do
  if [ "$v" = default ]; then L=ipt_amd/lib/libipt_hip.so; else L=ipt_amd/lib/abl/libipt_$v.so; fi
  IPT_ABI_COMPAT=1 IPT_LIB_PATH=$L timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-2} --warmup 1 --cpu-seconds 0 --no-counters ${BENCH_EXTRA} > gpurun_out/var_${v}_$c.json 2>gpurun_out/var_${v}_$c.err || { echo "variant $v $c failed"; tail -3 gpurun_out/var_${v}_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/var_${v}_$c.json'));print('$c variant $v', round(d['value'],3), 'Mpaths/s')"
done
done
