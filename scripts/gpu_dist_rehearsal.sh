# N>1 bench path rehearsed on one GPU (all ranks on cuda:0, gloo collectives)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in ${NS:-2 4}; do
  IPT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n ${CFG:+--config $CFG} --steps 1 --warmup 1 --cpu-seconds 0 ${VERIFY:+--verify} > gpurun_out/dist_${CFG:-c2}_$n.json 2> gpurun_out/dist_${CFG:-c2}_$n.err || { echo "dist $n failed"; tail -20 gpurun_out/dist_${CFG:-c2}_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/dist_${CFG:-c2}_$n.json').read().strip().splitlines()[-1]);print('n', d['n_gpus'], 'value', round(d['value'],2), 'mean_pixel', d['mean_pixel'], 'H', d['config']['height'], 'events', round(d['events_per_path']['traced_rays'],3), 'verify', d.get('verify_whole_frame_bit_exact'), 'rank_imbalance', d.get('rank_imbalance'))"
done
