cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for round in 1 2; do
for n in 0 1 2 3 4 5 6 7; do
  IPT_LIB_PATH=ipt_amd/lib/abl/libipt_abl$n.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-counters > gpurun_out/abl$n.json 2>/dev/null || { echo "abl $n failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl$n.json'));print('round $round abl $n', round(d['ms_per_step'],2))"
done
done
