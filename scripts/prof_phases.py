#!/usr/bin/env python3
"""Per-phase lane utilisation of the path kernel (IPT_PROF build), C2 scene.
usage: IPT_LIB_PATH=ipt_amd/lib/abl/libipt_prof.so python scripts/prof_phases.py [config]"""
import json, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch
from ipt_amd import capi, scenes

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
desc = {"c2": scenes.make_scene_box, "c5": lambda: scenes.make_scene_box_lights(16),
        "c3": lambda: scenes.make_scene_spheres(10000, 1)}[cfg]()
W = H = 1024
spp = {"c2": 8, "c5": 1, "c3": 1}[cfg]
ctx = capi.Context(0)
ctx.upload_scene(desc)
px = torch.zeros(W * H, dtype=torch.float32, device="cuda")
cn = torch.zeros(W * H, dtype=torch.int32, device="cuda")
p = capi.make_params(W, H, spp)
st = torch.cuda.current_stream().cuda_stream
ctx.render_device(p, px.data_ptr(), cn.data_ptr(), stream=st)
torch.cuda.synchronize()
ctx.reset_counters()
ctx.render_device(p, px.data_ptr(), cn.data_ptr(), stream=st)
torch.cuda.synchronize()
prof = ctx.profile()
paths = W * H * spp
out = {}
stamps = prof.pop("stamps")
tot = sum(stamps.values())
if tot:
    for sg, v in stamps.items():
        print(f"segment {sg:22s} {100.0 * v / tot:6.2f} %")
for ph, (w, l) in prof.items():
    out[ph] = {"wave_execs_per_path": w / paths, "lanes_per_path": l / paths,
               "utilisation": (l / (64.0 * w)) if w else None}
    print(f"{ph:14s} wave-execs/path {w / paths:8.3f}  lanes/path {l / paths:8.3f}  util {out[ph]['utilisation'] or 0:6.3f}")
tag = Path(__import__("os").environ.get("IPT_LIB_PATH", "default")).stem
json.dump({"config": cfg, "paths": paths, "phases": out, "stamp_shares": {k: v / tot for k, v in stamps.items()} if tot else None}, open(f"gpurun_out/prof_{tag}_{cfg}.json", "w"), indent=1)
