"""Full-size sharded parity (BASELINE.json configs[3] and
configs[4]): every shard of the n_shards = 8 tile plan rendered on the one
GPU, one pass each, at the configurations' own frame sizes.

The reference's only parallelism is whole-frame worker threads
(/root/reference/src/main.cpp:256-285); the multi-GPU path replaces it with
destination-row tiles dealt round-robin to the ranks (16-row tiles, shard t %
8). For each shard the test checks, bit for bit:
* the shard writes only its owned rows of the GridRenderPlane state (pixels,
  counters, sums, per-pixel max);
* the owned rows of the eight shards, assembled, equal the whole-frame
  render of the same pass;
* that whole-frame plane equals the oracle's GridRenderPlane::addRay replay
  (GridRenderPlane.cpp:61-75) of the frame's samples, whose values at strided
  source rows and columns the oracle recomputes from scratch.
C4 is the box at 4096^2 (one GPU's share of configs[3] would be its whole
frame at N = 1); C5 the 256-emitter lattice at 2048^2.
"""
import numpy as np
import pytest
import torch

import oracle_binding as ob
from ipt_amd import capi, scenes

pytestmark = pytest.mark.gpu

N_SHARDS, TILE = 8, 16


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_full_size_eight_shard_plan_bit_exact(gpu_ctx, oracle, cfg):
    if cfg == "c4":
        desc, W, rs, rp, cs, cp = scenes.make_scene_box(), 4096, 1024, 517, 4, 3
    else:
        desc, W, rs, rp, cs, cp = scenes.make_scene_box_lights(16), 2048, 512, 211, 4, 1
    H = W
    gpu_ctx.upload_scene(desc)
    dev = torch.device("cuda", 0)
    kw = dict(spp_offset=29, n_rays=16, depth_max=8)

    def render(p):
        st = torch.zeros(4, H, W, dtype=torch.float32, device=dev)
        gpu_ctx.render_device(p, st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr())
        torch.cuda.synchronize(dev)
        return st

    whole = render(capi.make_params(W, H, 1, **kw))
    assembled = torch.zeros_like(whole)
    covered = np.zeros(H, np.int32)
    for s in range(N_SHARDS):
        p = capi.make_params(W, H, 1, tile_rows=TILE, n_shards=N_SHARDS, shard_id=s, **kw)
        owned, _ = capi.shard_plan(p)
        covered += owned.astype(np.int32)
        part = render(p)
        own = torch.as_tensor(owned.astype(bool), device=dev)
        assert not part[:, ~own].any().item(), f"shard {s} wrote outside its rows"
        assembled[:, own] = part[:, own]
        del part
    assert (covered == 1).all(), "every destination row is owned exactly once"
    assert torch.equal(assembled.view(torch.int32), whole.view(torch.int32)), "assembled != whole frame"
    del assembled

    # the whole frame against the oracle: its samples, strided rows recomputed
    gv, gc = gpu_ctx.render_values(capi.make_params(W, H, 1, **kw))
    ov, rows, cols = ob.render_rows_values(desc, capi.make_params(W, H, 1, **kw), rs, rp, cs, cp, n_threads=16)
    sel = gv[:, rows, :][:, :, cols]
    assert np.array_equal(_bits(sel), _bits(ov)), int((_bits(sel) != _bits(ov)).sum())
    ref = ob.accumulate(gv, gc)
    got = whole.cpu().numpy().reshape(4, -1)
    for i, k in enumerate(("pixels", "counters", "sums", "pixel_max")):
        assert np.array_equal(_bits(got[i]), _bits(ref[k])), k
