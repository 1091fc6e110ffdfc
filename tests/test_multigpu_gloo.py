"""Multi-GPU path on CPU: world_size-2 gloo run of the shard plan + frame-end
assembly that bench.py performs over RCCL.

Each rank takes its tile plan from the product (ipt_shard_plan), forms the
GridRenderPlane rows it owns (here from the oracle; on the GPU box
test_gpu_parity.py::test_sharded_render_matches_whole_frame checks the
kernel's shard image equals exactly this), and rank 0 assembles the frame with
reduce(SUM) / reduce(MAX) — the collective bench.py issues. The assembled
frame must equal the single-rank frame bit-for-bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, TILE = 40, 48, 2, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    import oracle_binding as ob
    from ipt_amd import capi, scenes

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = capi.make_params(W, H, SPP, tile_rows=TILE, n_shards=world, shard_id=rank)
        owned, cand = capi.shard_plan(p)
        vals, codes = ob.render_values(scenes.make_scene_box(), capi.make_params(W, H, SPP))
        # every sample that lands in an owned row is traced by this rank
        for s in range(SPP):
            for iy in range(H):
                yn = max(H - 2 - iy, 0)
                for ix in range(W):
                    yi = yn + ((int(codes[s, iy, ix]) >> 2) & 3) - 1
                    if owned[yi]:
                        assert iy in cand, (rank, iy, yi)
        full = ob.accumulate(vals, codes)
        mask = np.repeat(owned, W)
        part = {k: torch.from_numpy(np.where(mask, v, 0).astype(v.dtype).view(
            np.int32 if v.dtype == np.uint32 else v.dtype)) for k, v in full.items()}
        dist.reduce(part["pixels"], 0, op=dist.ReduceOp.SUM)
        dist.reduce(part["counters"], 0, op=dist.ReduceOp.SUM)
        dist.reduce(part["sums"], 0, op=dist.ReduceOp.SUM)
        dist.reduce(part["pixel_max"], 0, op=dist.ReduceOp.MAX)
        if rank == 0:
            ok = all(np.array_equal(part[k].numpy().view(np.uint32),
                                    full[k].view(np.uint32)) for k in full)
            q.put(ok)
        own_count = torch.tensor([int(owned.sum())])
        dist.all_reduce(own_count)
        if rank == 0:
            q.put(int(own_count.item()))
    finally:
        dist.destroy_process_group()


def test_two_rank_frame_assembly(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=300)
        assert pr.exitcode == 0
    assert q.get(timeout=10) is True
    assert q.get(timeout=10) == H  # every destination row owned exactly once
