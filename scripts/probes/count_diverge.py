"""Which samples differ between a library's counting instance (IPT_FLAG_COUNTERS)
and the oracle, and between its counting and product instances.

usage: IPT_LIB_PATH=ipt_amd/lib/abl/libipt_X.so python scripts/probes/count_diverge.py
Prints, per scene, the number of differing samples of each instance against
the oracle's per-path values and the first few (pass, row, col, gpu, oracle).
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
os.environ.setdefault("IPT_ABI_COMPAT", "1")

from ipt_amd import capi, scenes  # noqa: E402
import oracle_binding as ob  # noqa: E402


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def main():
    ctx = capi.Context(0)
    cases = [("box", scenes.make_scene_box(), 32, 32, 2),
             ("box_lights16", scenes.make_scene_box_lights(4), 24, 20, 2),
             ("box_lights256", scenes.make_scene_box_lights(16), 24, 20, 2)]
    for name, desc, W, H, spp in cases:
        ctx.upload_scene(desc)
        ov, oc, ev = ob.render_events(desc, capi.make_params(W, H, spp), 0)
        for flags, tag in ((0, "product"), (capi.IPT_FLAG_COUNTERS, "counting")):
            ctx.reset_counters()
            vals, codes = ctx.render_values(capi.make_params(W, H, spp, flags=flags))
            vals = np.asarray(vals).reshape(ov.shape)
            bad = np.argwhere(bits(vals) != bits(ov))
            print(f"{name} {tag}: {len(bad)} of {vals.size} samples differ", flush=True)
            for s, y, x in bad[:6]:
                e = dict(zip(ob.EVENT_NAMES, ev[s, y, x].tolist()))
                print(f"   pass {s} row {y} col {x}: gpu {vals[s, y, x]!r} oracle {ov[s, y, x]!r} "
                      f"oracle events {e}", flush=True)
            if flags:
                g = ctx.counters()
                tot = ev.reshape(-1, ev.shape[-1]).sum(0)
                print("   counters gpu:", {k: g[k] for k in ("paths", "traced_rays", "iterations", "skipped")},
                      "oracle:", dict(zip(ob.EVENT_NAMES, tot.tolist())), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
