"""Multi-rank path: world_size-2 gloo runs of the tile plan
and the frame-end assembly (ipt_amd/tiles.py, the code bench.py runs over
RCCL).

* test_rank_frame_assembly (CPU, world_size 2 / 4 / 8, uneven shares): each rank takes its tile plan from the
  product (ipt_shard_plan), forms the GridRenderPlane rows it owns from the
  oracle's whole frame, and rank 0 assembles with tiles.assemble (one gather
  of owned rows); the result must equal the single-rank frame bit for bit.
* test_rank_sharded_render_on_gpu (GPU, world_size 2 / 4): the same run with the
  PRODUCT rendering each shard (both ranks on cuda:0, gloo for the frame
  end, as bench.py's IPT_BENCH_SHARE_GPU=1 rehearsal): the assembled frame
  must equal the whole-frame GPU render and the oracle's replay, bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, TILE = 40, 48, 2, 8
# (world, W, H, tile_rows) of the CPU assembly runs: H is not a multiple of
# tile_rows * world at 4 and 8 ranks, so the ranks' padded shares are uneven
# and the last tile is partial
CPU_PLANS = [(2, 40, 48, 8), (4, 36, 53, 4), (8, 32, 77, 4)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _setup(rank, world, port):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _state_of(img, h=H, w=W):
    return torch.from_numpy(np.stack([img[k].view(np.float32) for k in ("pixels", "counters", "sums", "pixel_max")])
                            .reshape(4, h, w).copy())


def _worker_cpu(rank, world, port, q, W=W, H=H, TILE=TILE):
    _setup(rank, world, port)
    import oracle_binding as ob
    from ipt_amd import capi, scenes, tiles

    try:
        owned = tiles.owned_rows(W, H, TILE, world)
        p = capi.make_params(W, H, SPP, tile_rows=TILE, n_shards=world, shard_id=rank)
        _, cand = capi.shard_plan(p)
        vals, codes = ob.render_values(scenes.make_scene_box(), capi.make_params(W, H, SPP))
        # every sample that lands in an owned row is traced by this rank
        for s in range(SPP):
            for iy in range(H):
                yn = max(H - 2 - iy, 0)
                for ix in range(W):
                    yi = yn + ((int(codes[s, iy, ix]) >> 2) & 3) - 1
                    if yi in owned[rank]:
                        assert iy in cand, (rank, iy, yi)
        full = _state_of(ob.accumulate(vals, codes), H, W)
        mine = torch.zeros_like(full)  # a rank's render writes only its owned rows
        mine[:, owned[rank]] = full[:, owned[rank]]
        tiles.assemble(dist, mine, owned, rank, host=True)
        if rank == 0:
            q.put(bool(torch.equal(mine.view(torch.int32), full.view(torch.int32))))
            q.put(sorted(np.concatenate(owned).tolist()) == list(range(H)))
    finally:
        dist.destroy_process_group()


def _worker_gpu(rank, world, port, q, W=W, H=H, TILE=TILE):
    _setup(rank, world, port)
    import oracle_binding as ob
    from ipt_amd import capi, scenes, tiles

    try:
        desc = scenes.make_scene_box()
        owned = tiles.owned_rows(W, H, TILE, world)
        ctx = capi.Context(0)
        ctx.upload_scene(desc)
        dev = torch.device("cuda", 0)
        state = torch.zeros(4, H, W, dtype=torch.float32, device=dev)

        def render(p, st):
            ctx.render_device(p, st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr())

        # two calls continue the same running mean, as bench.py's steps do
        for s0 in (0, SPP):
            render(capi.make_params(W, H, SPP, spp_offset=s0, tile_rows=TILE, n_shards=world, shard_id=rank), state)
        torch.cuda.synchronize(dev)
        others = np.setdiff1d(np.arange(H), owned[rank])
        wrote_outside = bool(state[:, others].any().item())
        tiles.assemble(dist, state, owned, rank, host=True)
        torch.cuda.synchronize(dev)
        if rank == 0:
            whole = torch.zeros_like(state)
            for s0 in (0, SPP):
                render(capi.make_params(W, H, SPP, spp_offset=s0), whole)
            torch.cuda.synchronize(dev)
            vals, codes = ob.render_values(desc, capi.make_params(W, H, 2 * SPP))
            ref = _state_of(ob.accumulate(vals, codes), H, W)
            got = state.cpu()
            q.put((wrote_outside, bool(torch.equal(got.view(torch.int32), whole.cpu().view(torch.int32))),
                   bool(torch.equal(got.view(torch.int32), ref.view(torch.int32)))))
        else:
            q.put((wrote_outside,))
        ctx.close()
    finally:
        dist.destroy_process_group()


def _run(target, world=2, extra=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(extra)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=300)
        assert pr.exitcode == 0
    return [q.get(timeout=10) for _ in range(world if target is _worker_gpu else 2)]


@pytest.mark.parametrize("world,w,h,tile", CPU_PLANS)
def test_rank_frame_assembly(oracle, world, w, h, tile):
    """world_size 2 / 4 / 8 over gloo: the tile plan of every rank and the
    frame-end gather of owned rows reproduce the single-rank frame bit for
    bit, with uneven padded shares (the bench's N = 8 path on the CPU)."""
    equal, partition = _run(_worker_cpu, world, (w, h, tile))
    assert equal is True
    assert partition is True  # every destination row owned exactly once


@pytest.mark.gpu
@pytest.mark.parametrize("world,w,h,tile", [(2, 40, 48, 8), (4, 36, 53, 4)])
def test_rank_sharded_render_on_gpu(oracle, world, w, h, tile):
    res = _run(_worker_gpu, world, (w, h, tile))
    full = [r for r in res if len(r) == 3]
    assert len(full) == 1
    assert not any(r[0] for r in res), "a shard wrote outside its rows"
    assert full[0][1], "assembled frame != whole-frame GPU render"
    assert full[0][2], "assembled frame != oracle"
