"""Quick perf probe (not a test): renders sample_scenes[0] at W x W x spp."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
from ipt_amd import capi, scenes
W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ctx = capi.Context(0)
ctx.upload_scene(scenes.make_scene_box())
img = {k: np.zeros(W * W, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32))}
ctx.render(capi.make_params(W, W, 1), img)  # warmup
for rep in range(2):
    t = time.time()
    ctx.render(capi.make_params(W, W, spp, spp_offset=1 + rep * spp, flags=capi.IPT_FLAG_COUNTERS), img)
    dt = time.time() - t
    pm, am = ctx.last_kernel_ms()
    paths = W * W * spp
    print(f"W={W} spp={spp}: wall {dt*1e3:.1f} ms, path kernel {pm:.1f} ms, acc {am:.2f} ms, "
          f"{paths/pm/1e3:.2f} Mpaths/s (kernel)", flush=True)
print(ctx.counters())
print("mean", img["pixels"].mean())
