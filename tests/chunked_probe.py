"""Helper (not a test): one synchronous render split into several launches
(IPT_TEST_CHUNK_UNITS), checked bit for bit against the oracle; exit 0 when
equal. test_gpu_async.py runs it under `rocprofv3 --pmc`, whose dispatch
serialisation must make the library gate launches on events (ipt_create)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import numpy as np

import oracle_binding as ob
from ipt_amd import capi, scenes

W, H, SPP = 36, 28, 7
ctx = capi.Context(0)
desc = scenes.make_scene_box()
ctx.upload_scene(desc)
p = capi.make_params(W, H, SPP, spp_offset=5)
img = {k: np.zeros(W * H, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32),
                                            ("sums", np.float32), ("pixel_max", np.float32))}
ctx.render(p, img)
ov, oc = ob.render_values(desc, p)
ref = ob.accumulate(ov, oc)
ok = all(np.array_equal(img[k].view(np.uint32), ref[k].view(np.uint32)) for k in img)
ctx.close()
print("chunked render", "bit-exact" if ok else "DIFFERS", flush=True)
sys.exit(0 if ok else 1)
