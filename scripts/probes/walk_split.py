"""The split-traversal measurement for C3 (scripts/probes/walk_split.hip).

Renders one pass of the C3 frame (1024 x 1024, n_rays 16, depth_max 8, the
10 000-sphere scene) with the IPT_RAYLOG build, which logs every k-th finished
sphere-list trace, then re-traces the logged rays with the stand-alone
traversal kernel at several occupancies and walk budgets. Every line reports
the rays/s of the traversal alone and the rays whose (t, hit) differ from the
megakernel's (must be 0). GPU box: bash scripts/probes/build_walk_split.sh
first (CPU container), then python scripts/probes/walk_split.py.
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
os.environ["IPT_LIB_PATH"] = str(ROOT / "scripts/probes/libipt_walksplit.so")
sys.path.insert(0, str(ROOT))

from ipt_amd import capi, scenes  # noqa: E402


def main():
    every = int(os.environ.get("WALK_EVERY", "4"))
    cap = int(os.environ.get("WALK_CAP", str(160 << 20)))
    ctx = capi.Context(0)
    lib = ctx.lib
    lib.probe_raylog_arm.argtypes = [C.c_ulonglong, C.c_uint]
    lib.probe_raylog_count.argtypes = [C.c_void_p, C.c_void_p]
    lib.probe_walk.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_ulonglong, C.c_void_p,
                               C.c_void_p]
    assert lib.probe_raylog_arm(cap, every) == 0
    ctx.upload_scene(scenes.make_scene_spheres(10000, seed=1))
    p = capi.make_params(1024, 1024, 1, n_rays=16, depth_max=8)
    ctx.render_values(p)
    seen, held = C.c_ulonglong(), C.c_ulonglong()
    assert lib.probe_raylog_count(C.byref(seen), C.byref(held)) == 0
    print(json.dumps({"logged_from": "c3 1024x1024 x 1 spp, n_rays 16, depth_max 8", "traces_seen": seen.value,
                      "traces_per_path": seen.value / (1024 * 1024), "records": held.value, "every": every}),
          flush=True)
    n = held.value
    runs = [(4, 4, 8), (4, 5, 8), (4, 6, 8), (4, 7, 8), (8, 8, 8), (4, 4, 32), (4, 7, 32), (4, 4, 64), (4, 7, 64), (8, 8, 64)]
    # WALK_RUNS="wps,wgs,budget;..." (counter passes: one run each, no counting runs)
    if os.environ.get("WALK_RUNS"):
        runs = [tuple(int(x) for x in r.split(",")) for r in os.environ["WALK_RUNS"].split(";")]
    reps = int(os.environ.get("WALK_REPS", "3"))
    for count in (() if os.environ.get("WALK_RUNS") else (1,)) + (0,):
        for wps, wgs, budget in runs if not count else [(4, 4, 8), (4, 7, 64)]:
            best_ms = None
            for _ in range(1 if count else reps):
                ms = C.c_float()
                out = (C.c_ulonglong * 4)()
                rc = lib.probe_walk(ctx.h, wps, count, wgs, budget, n, C.byref(ms), out)
                if rc != 0:
                    print(json.dumps({"wps": wps, "wgs_per_cu": wgs, "budget": budget, "rc": rc}), flush=True)
                    break
                if out[0] != 0:
                    print(json.dumps({"wps": wps, "wgs_per_cu": wgs, "budget": budget, "MISMATCH": out[0]}),
                          flush=True)
                    sys.exit(1)
                assert out[3] == n, (out[3], n)
                best_ms = ms.value if best_ms is None else min(best_ms, ms.value)
            else:
                line = {"wps": wps, "wgs_per_cu": wgs, "waves_per_simd_cap": min(wgs, 8), "budget": budget,
                        "count": count, "rays": n, "ms": best_ms, "Grays_per_s": n / best_ms / 1e6,
                        "mismatches": 0}
                if count:
                    line["cells_per_ray"] = out[1] / n
                    line["tests_per_ray"] = out[2] / n
                print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
