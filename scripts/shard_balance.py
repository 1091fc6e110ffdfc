#!/usr/bin/env python3
"""Per-shard work balance of the tile sharding, measured on ONE GPU.

For N in {2, 4, 8} every shard of the BASELINE config's frame (c4: the box at
4096^2 x 32 spp, c5: 256 emitters at 2048^2 x 64 spp, i.e. bench.py's strong-
scaling step) is rendered in turn on cuda:0, alone on the GPU, with the
kernel's event counters (IPT_FLAG_COUNTERS). Per shard: paths, traced rays,
light tests, the algorithmic op-eq (ipt_amd.roofline) and the path-kernel
time (HIP events; the shard had the whole GPU). The work imbalance
max/mean over shards is the predictor of the 8-GPU strong-scaling efficiency
(eff <= mean/max); T_whole / (N * max shard time) is the efficiency the
shards' own times predict (each shard launch also has its own tail).

usage: python3 scripts/shard_balance.py c4 [c5 ...] -> profiles/<tag>_shard_balance_<cfg>.json
"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402  (CONFIGS, make_desc)


def main():
    import torch

    from ipt_amd import capi, roofline

    tag = os.environ.get("TAG", "round4")
    out_dir = Path(os.environ.get("OUT_DIR", ROOT / "profiles"))
    out_dir.mkdir(parents=True, exist_ok=True)
    dev = torch.device("cuda", 0)
    ctx = capi.Context(0)
    for cfg in sys.argv[1:] or ["c4", "c5"]:
        scene, W, H, spp, _steps, depth, _scaling, _cpu = bench.CONFIGS[cfg]
        desc = bench.make_desc(scene)
        ctx.upload_scene(desc)
        state = torch.zeros(4, H, W, dtype=torch.float32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        n_sph, n_li = len(desc.get("spheres", [])), len(desc.get("lights", []))

        def run(n_shards, shard, flags):
            p = capi.make_params(W, H, spp, spp_offset=0, n_rays=16, depth_max=depth,
                                 tile_rows=16 if n_shards > 1 else 0, n_shards=n_shards, shard_id=shard, flags=flags)
            ctx.reset_counters()
            ctx.render_device(p, state[0].data_ptr(), state[1].data_ptr(), state[2].data_ptr(),
                              state[3].data_ptr(), stream)
            torch.cuda.synchronize(dev)
            return ctx.last_kernel_ms()[0], ctx.counters()

        run(1, 0, 0)  # warm-up (tables, work buffers)
        t_whole, _ = run(1, 0, 0)
        _, c_whole = run(1, 0, capi.IPT_FLAG_COUNTERS)
        rec = {"config": cfg, "workload": f"{scene} {W}x{H}, {spp} spp, depth_max {depth}, n_rays 16, 16-row tiles",
               "whole_frame": {"path_ms": t_whole, "paths": c_whole["paths"],
                               "traced_rays": c_whole["traced_rays"],
                               "ops": roofline.ops_from_counters(c_whole, n_sph, n_li)},
               "shards": {}}
        for n in (2, 4, 8):
            rows = []
            for s in range(n):
                ms, _ = run(n, s, 0)
                _, c = run(n, s, capi.IPT_FLAG_COUNTERS)
                rows.append({"shard": s, "path_ms": ms, "paths": c["paths"], "traced_rays": c["traced_rays"],
                             "light_tests": c["light_tests"], "sphere_tests": c["sphere_tests"],
                             "ops": roofline.ops_from_counters(c, n_sph, n_li)})
                print(cfg, n, s, round(ms, 1), c["paths"], c["traced_rays"], flush=True)

            def imb(k):
                v = [r[k] for r in rows]
                return max(v) / (sum(v) / len(v))

            tot = {k: sum(r[k] for r in rows) for k in ("paths", "traced_rays", "ops")}
            rec["shards"][str(n)] = {
                "per_shard": rows,
                "work_imbalance_paths": imb("paths"),
                "work_imbalance_traced_rays": imb("traced_rays"),
                "work_imbalance_ops": imb("ops"),
                "time_imbalance": imb("path_ms"),
                "sum_equals_whole": {k: tot[k] == rec["whole_frame"][k] if k != "ops" else
                                     abs(tot[k] / rec["whole_frame"][k] - 1) < 1e-9 for k in tot},
                "predicted_strong_efficiency_work": 1.0 / imb("ops"),
                "predicted_strong_efficiency_time": t_whole / (n * max(r["path_ms"] for r in rows)),
            }
        rec["measured_at"] = time.strftime("%Y-%m-%d %H:%M:%S")
        f = out_dir / f"{tag}_shard_balance_{cfg}.json"
        f.write_text(json.dumps(rec, indent=1))
        print(f, {n: (round(v["work_imbalance_ops"], 4), round(v["predicted_strong_efficiency_time"], 4))
                  for n, v in rec["shards"].items()}, flush=True)
        del state
    ctx.close()


if __name__ == "__main__":
    main()
