# GPU parity tests, then C5 with the light lattice lookup (default) and with
# the light BVH (IPT_LIGHT_GRID=0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit 1
for g in 1 0; do
  IPT_LIGHT_GRID=$g timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/c5_grid$g.json 2> gpurun_out/c5_grid$g.err || { echo "c5 grid=$g failed"; tail -5 gpurun_out/c5_grid$g.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5_grid$g.json')); print('c5 grid=$g', round(d['value'],2), d['unit'], {k: round(v,2) for k,v in (d.get('events_per_path') or {}).items() if k in ('light_tests','light_nodes','traced_rays')})"
done
