# N>1 bench path with queued steps, rehearsed on one GPU (both ranks on cuda:0, gloo), verified bit for bit
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in c5 c2; do
  IPT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config $c --steps 2 --warmup 1 --cpu-seconds 0 --verify > gpurun_out/r4h_$c.json 2> gpurun_out/r4h_$c.err || { echo "dist $c failed"; tail -20 gpurun_out/r4h_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r4h_$c.json').read().strip().splitlines()[-1]);print('$c', d['n_gpus'], round(d['value'],2), d['config']['calls'], 'verify', d.get('verify_whole_frame_bit_exact'), 'rank_imb', round(d['rank_imbalance'],3), 'work_imb', round(d['work_imbalance'],4))"
done
