cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in c3 c5; do
  timeout -k 10 500 python bench.py --config $c --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "$c failed"; tail -5 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', round(d['value'],3), 'Mpaths/s', round(d['ms_per_step'],1), 'ms/step', 'frac', d['roofline']['frac'])"
done
