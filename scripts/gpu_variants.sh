cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# profiling: C2 throughput of library variants (IPT_LIB_PATH) against the default build
# (COUNTERS=1: with the event counters, to check that a timing experiment kept the path statistics)
CF="--no-counters"; [ -n "$COUNTERS" ] && CF=""
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then L=ipt_amd/lib/libipt_hip.so; else L=ipt_amd/lib/abl/libipt_$v.so; fi
  IPT_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 $CF > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/var_$v.err; exit 1; }
  python scripts/print_var.py $v gpurun_out/var_$v.json
done
