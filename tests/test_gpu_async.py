"""Queued renders and chunked launches (the two work slots).

Consecutive launches alternate between two work slots with their own
streams, so a launch fills the CUs its predecessor's tail leaves idle; the
GridRenderPlane replays stay on the caller's stream in call order. The
reference's progressive loop renders pass after pass into one GridRenderPlane
(/root/reference/src/main.cpp:256-285, render_sample per pass): every queued
sequence here must leave the image bit-identical to one synchronous call
over the same passes, and to the oracle's replay of GridRenderPlane::addRay
(GridRenderPlane.cpp:61-75).
"""
import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi, scenes

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _state(W, H):
    import torch

    return torch.zeros(4, H, W, dtype=torch.float32, device="cuda")


def _ptrs(st):
    return st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr()


def _host(st):
    import torch

    torch.cuda.synchronize()
    a = st.cpu().numpy()
    return {"pixels": a[0].reshape(-1), "counters": a[1].view(np.uint32).reshape(-1),
            "sums": a[2].reshape(-1), "pixel_max": a[3].reshape(-1)}


def _assert_same(a, b):
    for k in ("pixels", "sums", "pixel_max"):
        assert np.array_equal(_bits(a[k]), _bits(b[k])), k
    assert np.array_equal(a["counters"], b["counters"])


def _stream():
    import torch

    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("scene", ["box", "spheres", "lights"])
def test_queued_calls_equal_one_call(gpu_ctx, oracle, scene):
    """Four queued 2-spp calls == one synchronous 8-spp call == the oracle."""
    desc = {"box": scenes.make_scene_box, "spheres": lambda: scenes.make_scene_spheres(3000, seed=1),
            "lights": lambda: scenes.make_scene_box_lights(16)}[scene]()
    W, H = (48, 40) if scene != "spheres" else (24, 20)
    gpu_ctx.upload_scene(desc)
    one = _state(W, H)
    gpu_ctx.render_device(capi.make_params(W, H, 8), *_ptrs(one), _stream())
    q = _state(W, H)
    for c in range(4):
        gpu_ctx.render_device_async(capi.make_params(W, H, 2, spp_offset=2 * c), *_ptrs(q), _stream())
    gpu_ctx.wait()
    a, b = _host(one), _host(q)
    _assert_same(a, b)
    ov, oc = ob.render_values(desc, capi.make_params(W, H, 8))
    _assert_same(a, ob.accumulate(ov, oc))
    pm, am = gpu_ctx.last_kernel_ms()
    assert pm > 0 and am > 0


def test_interleaved_images_and_stream_order(gpu_ctx):
    """Calls into two images, queued alternately, each equal to its own
    sequential render; the image is complete in `stream` order (a torch
    operation queued after the calls sees the final image without a wait)."""
    import torch

    W, H = 40, 32
    gpu_ctx.upload_scene(scenes.make_scene_box())
    A, B = _state(W, H), _state(W, H)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()  # a real stream (torch's default one is handle 0 = the context's own)
    with torch.cuda.stream(s):
        for c in range(3):
            gpu_ctx.render_device_async(capi.make_params(W, H, 2, spp_offset=2 * c), *_ptrs(A), s.cuda_stream)
            gpu_ctx.render_device_async(capi.make_params(W, H, 1, spp_offset=50 + c), *_ptrs(B), s.cuda_stream)
        snap = A.clone()  # queued on the same stream, after the accumulates
    gpu_ctx.wait()
    ra, rb = _state(W, H), _state(W, H)
    gpu_ctx.render_device(capi.make_params(W, H, 6), *_ptrs(ra), _stream())
    for c in range(3):
        gpu_ctx.render_device(capi.make_params(W, H, 1, spp_offset=50 + c), *_ptrs(rb), _stream())
    _assert_same(_host(A), _host(ra))
    _assert_same(_host(B), _host(rb))
    _assert_same(_host(snap), _host(ra))
    torch.cuda.synchronize()


def test_upload_between_queued_calls(gpu_ctx):
    """ipt_upload_scene waits for the queued launches that read the old scene."""
    W, H = 32, 24
    box, lit = scenes.make_scene_box(), scenes.make_scene_lit_corner()
    gpu_ctx.upload_scene(box)
    X = _state(W, H)
    gpu_ctx.render_device_async(capi.make_params(W, H, 3), *_ptrs(X), _stream())
    gpu_ctx.upload_scene(lit)
    Y = _state(W, H)
    gpu_ctx.render_device_async(capi.make_params(W, H, 3), *_ptrs(Y), _stream())
    gpu_ctx.wait()
    for desc, img in ((box, X), (lit, Y)):
        ov, oc = ob.render_values(desc, capi.make_params(W, H, 3))
        _assert_same(_host(img), ob.accumulate(ov, oc))


@pytest.mark.parametrize("gate", ["pool", "IPT_NO_TAIL_OVERLAP", "ROCPROF_COUNTER_COLLECTION"])
@pytest.mark.parametrize("units", [1, 3000, 5000])
def test_chunked_launches_bit_exact(oracle, monkeypatch, units, gate):
    """IPT_TEST_CHUNK_UNITS caps a launch (at least one pass): a call split
    into many launches, alternating slots and overlapping, gives the same
    image and the same per-sample values as the oracle -- with the launches
    gated on the predecessor's drained pool (the default) and on its end
    event (IPT_NO_TAIL_OVERLAP, or a counter-collecting profiler detected at
    ipt_create)."""
    monkeypatch.setenv("IPT_TEST_CHUNK_UNITS", str(units))
    if gate != "pool":
        monkeypatch.setenv(gate, "1")
    ctx = capi.Context(0)
    try:
        desc = scenes.make_scene_box()
        W, H = 36, 28
        ctx.upload_scene(desc)
        p = capi.make_params(W, H, 7, spp_offset=5)
        gv, gc = ctx.render_values(p)
        ov, oc = ob.render_values(desc, p)
        assert np.array_equal(gc, oc)
        assert np.array_equal(_bits(gv), _bits(ov))
        img = {k: np.zeros(W * H, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32),
                                                    ("sums", np.float32), ("pixel_max", np.float32))}
        ctx.render(p, img)
        _assert_same(img, ob.accumulate(ov, oc))
        # sharded + chunked: the slots' candidate-row tables follow the shard
        for sid in (0, 1):
            part = {k: np.zeros_like(v) for k, v in img.items()}
            ctx.render(capi.make_params(W, H, 7, spp_offset=5, tile_rows=4, n_shards=2, shard_id=sid), part)
            owned, _ = capi.shard_plan(capi.make_params(W, H, 1, tile_rows=4, n_shards=2, shard_id=sid))
            m = np.repeat(owned, W)
            for k in img:
                assert np.array_equal(_bits(part[k][m]), _bits(img[k][m])), (sid, k)
    finally:
        ctx.close()


def test_counters_after_queued_calls(gpu_ctx, oracle):
    """The event counters read after queued calls include all of them."""
    desc = scenes.make_scene_box()
    W, H = 24, 20
    gpu_ctx.upload_scene(desc)
    gpu_ctx.reset_counters()
    X = _state(W, H)
    for c in range(3):
        gpu_ctx.render_device_async(capi.make_params(W, H, 1, spp_offset=c, flags=capi.IPT_FLAG_COUNTERS),
                                    *_ptrs(X), _stream())
    g = gpu_ctx.counters()  # waits for the queued calls
    _, _, o = ob.render_values(desc, capi.make_params(W, H, 3), 0, with_counters=True)
    for k in ("paths", "traced_rays", "iterations", "light_traces"):
        assert g[k] == o[k], (k, g[k], o[k])


def test_chunked_call_under_counter_collection(tmp_path):
    """A synchronous call split into several launches completes under
    rocprofv3's counter collection (which serialises dispatches: a launch
    gated on a stream value wait behind it was never released)
    and stays bit-exact: the library must detect the tool and gate on events.
    A hang is killed by the timeout and fails the test."""
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not Path(prof).exists():
        pytest.skip("rocprofv3 not installed")
    probe = Path(__file__).resolve().parent / "chunked_probe.py"
    env = dict(__import__("os").environ, IPT_TEST_CHUNK_UNITS="3000", TMPDIR="/tmp")
    r = subprocess.run(["timeout", "-s", "KILL", "150", prof, "--pmc", "SQ_WAVES", "--kernel-trace",
                        "--output-format", "csv", "-d", str(tmp_path / "prof"), "-o", "run", "--",
                        sys.executable, str(probe)], capture_output=True, text=True, env=env, timeout=200)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "bit-exact" in r.stdout


def test_chunked_call_under_pool_gate_traced(tmp_path):
    """A synchronous call split into several launches with the pool gate on
    (each launch's stream waits on its predecessor's pool-drained flag,
    hipStreamWaitValue64 on signal memory) completes bit-exact under a
    trace-only rocprofv3 run (--kernel-trace: no dispatch serialisation, so the
    gate stays on), and the trace shows the runtime's wait kernel
    (__amd_rocclr_streamOpsWait): the stream wait runs as a polling kernel,
    which is why a dispatch-serialising tool deadlocks it."""
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not Path(prof).exists():
        pytest.skip("rocprofv3 not installed")
    probe = Path(__file__).resolve().parent / "chunked_probe.py"
    env = dict(__import__("os").environ, IPT_TEST_CHUNK_UNITS="3000", TMPDIR="/tmp")
    r = subprocess.run(["timeout", "-s", "KILL", "150", prof, "--kernel-trace", "--stats", "--output-format", "csv",
                        "-d", str(tmp_path / "prof"), "-o", "run", "--", sys.executable, str(probe)],
                       capture_output=True, text=True, env=env, timeout=200)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "bit-exact" in r.stdout
    stats = list((tmp_path / "prof").rglob("*kernel_stats.csv"))
    assert stats, "no kernel stats written"
    names = stats[0].read_text()
    assert "path_kernel" in names and "streamOpsWait" in names
