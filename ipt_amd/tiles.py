"""Image-tile sharding across ranks (one rank per GPU) and the frame-end
assembly of the GridRenderPlane state.

The reference has no multi-device path (its only parallelism is whole-frame
threads, /root/reference/src/main.cpp:256-285). Every (pixel, pass) sample is
independent and its RNG stream depends only on (seed, pass, pixel), so the
destination rows are cut into tiles dealt round-robin to the ranks
(ipt_params.tile_rows / n_shards / shard_id, ipt_shard_plan); a rank's
ipt_render_device writes only its owned rows of a full-frame state, and the
frame is assembled on rank 0 by ONE gather of each rank's owned rows — 16 B
per owned pixel (pixels, counters, sums, max), no zero padding beyond the
largest share, no reduction arithmetic (every pixel has exactly one owner).
"""
from __future__ import annotations

import numpy as np

from . import capi

FIELDS = 4  # GridRenderPlane pixels (f32), counters (u32 bits), sums (f32), pixel_max (f32)


def owned_rows(width: int, height: int, tile_rows: int, world: int) -> list[np.ndarray]:
    """Destination rows owned by each rank (ipt_shard_plan, host only)."""
    if world <= 1:
        return [np.arange(height)]
    out = []
    for r in range(world):
        p = capi.make_params(width, height, 1, tile_rows=tile_rows, n_shards=world, shard_id=r)
        out.append(np.nonzero(capi.shard_plan(p)[0])[0])
    return out


def assemble(dist, state, owned: list[np.ndarray], rank: int, host: bool = False) -> None:
    """Frame end: rank 0's `state` [FIELDS][H][W] (float32 tensor; counters as
    their bits) receives every rank's owned rows. `host`: the collective runs
    on host copies (gloo); otherwise on the device tensors (RCCL)."""
    import torch

    world = len(owned)
    W = state.shape[2]
    dev = state.device
    max_own = max(len(o) for o in owned)
    mine = torch.as_tensor(owned[rank], dtype=torch.long, device=dev)
    packed = torch.zeros(FIELDS, max_own, W, dtype=state.dtype, device=dev)
    packed[:, :len(owned[rank])] = state.index_select(1, mine)
    src = packed.cpu() if host else packed
    parts = [torch.empty_like(src) for _ in range(world)] if rank == 0 else None
    dist.gather(src, parts, dst=0)
    if rank == 0:
        for r in range(1, world):
            idx = torch.as_tensor(owned[r], dtype=torch.long, device=dev)
            state.index_copy_(1, idx, parts[r].to(dev)[:, :len(owned[r])])


def payload_bytes(width: int, owned: list[np.ndarray]) -> int:
    """Bytes the gather moves to rank 0 (every rank's padded share)."""
    return 4 * FIELDS * width * max(len(o) for o in owned) * len(owned)
