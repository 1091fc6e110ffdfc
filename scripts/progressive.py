#!/usr/bin/env python3
"""Progressive callers (the reference's pass-per-call loop, main.cpp:256-285):
throughput of a frame rendered as many small calls -- queued
(ipt_render_device_async, launches overlapping through the two work slots)
and synchronous -- against the same frame in one call, and whether the
images are bit-identical.

usage: python3 scripts/progressive.py [c3 c2] -> $OUT_DIR/<tag>_progressive.json
"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

# config: (total spp of the frame, spp per call of the progressive caller)
PLANS = {"c3": (64, 16), "c2": (256, 32), "c5": (64, 16)}


def main():
    import torch

    from ipt_amd import capi

    tag = os.environ.get("TAG", "round4")
    out_dir = Path(os.environ.get("OUT_DIR", ROOT / "profiles"))
    out_dir.mkdir(parents=True, exist_ok=True)
    dev = torch.device("cuda", 0)
    ctx = capi.Context(0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    for cfg in sys.argv[1:] or ["c3", "c2"]:
        scene, W, H, _spp, _steps, depth, _sc, _cpu = bench.CONFIGS[cfg]
        total, per_call = PLANS[cfg]
        ctx.upload_scene(bench.make_desc(scene))

        def run(mode, calls_spp):
            st = torch.zeros(4, H, W, dtype=torch.float32, device=dev)
            ptr = (st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr())
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            off = 0
            for n in calls_spp:
                p = capi.make_params(W, H, n, spp_offset=off, n_rays=16, depth_max=depth)
                if mode == "async":
                    ctx.render_device_async(p, *ptr, stream)
                else:
                    ctx.render_device(p, *ptr, stream)
                off += n
            if mode == "async":
                ctx.wait()
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            return W * H * total / el / 1e6, st

        run("sync", [per_call])  # warm-up: tables, both slots' buffers
        run("async", [per_call, per_call])
        r = {}
        one_v, one = run("sync", [total])
        r["one_call"] = {"Mpaths_s": one_v, "calls": 1}
        for mode in ("async", "sync"):
            v, img = run(mode, [per_call] * (total // per_call))
            r[f"{mode}_{per_call}spp_calls"] = {
                "Mpaths_s": v, "calls": total // per_call, "vs_one_call": v / one_v,
                "bit_exact_vs_one_call": bool(torch.equal(img.view(torch.int32), one.view(torch.int32)))}
            del img
        r["workload"] = f"{scene} {W}x{H}, {total} spp, depth_max {depth}, n_rays 16"
        res[cfg] = r
        print(cfg, json.dumps(r), flush=True)
    f = out_dir / f"{tag}_progressive.json"
    f.write_text(json.dumps(res, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
