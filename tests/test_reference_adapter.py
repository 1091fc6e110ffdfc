"""the reference-side adapter (integration/render_gpu.cpp),
compiled against the REFERENCE's own headers and linked with its own TUs
(oracle/build_ref.sh -> oracle/_ref/adapter_check; the only change is the
three AreaLight accessors the adapter documents, patched into a temporary
copy of lighting.h, and FractalSpheres' sphere-list accessors). The check
harness builds each scene with the reference's own sample_scenes code and a
reference GridRenderPlane, then calls render_samples_gpu twice (progressive
passes).

* CPU: the adapter type-checks and links (the binary exists whenever the
  reference tree is present) and, without a GPU, fails loudly with the
  library's IPT_E_DEVICE message (no CPU fallback).
* GPU: the reference's own GridRenderPlane, filled through the adapter, is
  bit-identical to the oracle's replay of the same passes.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi, scenes

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "oracle" / "_ref" / "adapter_check"
W, H, SPP, CALLS = 40, 32, 2, 2


def _need_bin():
    if not BIN.exists():
        if Path("/root/reference/src").is_dir():
            pytest.fail("oracle/_ref/adapter_check was not built (oracle/build_ref.sh)")
        pytest.skip("reference tree absent and adapter_check not shipped")


def test_adapter_builds_against_reference_and_fails_loudly_without_gpu(tmp_path):
    _need_bin()
    r = subprocess.run([str(BIN), "box", str(W), str(H), str(SPP), str(CALLS), str(tmp_path / "a")],
                       capture_output=True, text=True, timeout=120)
    if r.returncode == 3:
        assert "no HIP device" in r.stderr or "gfx950" in r.stderr, r.stderr
    else:
        assert r.returncode == 0, r.stderr  # a GPU is present: the render itself is checked below


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["box", "lit_corner", "fractal", "smallpt", "square_lit_by_square"])
def test_adapter_renders_reference_plane_bit_exact(oracle, tmp_path, scene):
    """Every sample_scenes entry (sample_scenes.cpp:20-108), built by the
    reference's own code and flattened by the adapter (AreaLight square and
    triangle, SphereLight; GeometrySphereInBox, GeometryCorner,
    FractalSpheres, GeometrySmallPt, GeometryFloor): the reference
    GridRenderPlane after two progressive calls is bit-identical to the
    oracle's replay, and the scene was uploaded once."""
    _need_bin()
    r = subprocess.run([str(BIN), scene, str(W), str(H), str(SPP), str(CALLS), str(tmp_path / "a")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    px = np.fromfile(tmp_path / "a.f32", np.float32)
    cnt = np.fromfile(tmp_path / "a.u32", np.uint32)
    desc = getattr(scenes, f"make_scene_{scene}")()
    ov, oc = ob.render_values(desc, capi.make_params(W, H, SPP * CALLS))
    ref = ob.accumulate(ov, oc)
    assert np.array_equal(cnt, ref["counters"])
    assert np.array_equal(px.view(np.uint32), ref["pixels"].view(np.uint32))
    out = r.stdout.split()
    mx = float(out[out.index("max_value") + 1])
    assert np.float32(mx) == ref["pixel_max"].max()
    assert int(out[out.index("uploads") + 1]) == 1  # unchanged scene: not re-uploaded
    # device-resident plane: a later call moves 12 B per pixel down (pixels,
    # counters, per-pixel max) and at most 4 B up (the zeroed max, for row runs
    # whose previous maxima were not all zero), not the whole plane both ways
    assert 12 * W * H <= int(out[out.index("last_call_transfer_bytes") + 1]) <= 16 * W * H


@pytest.mark.gpu
@pytest.mark.parametrize("scene,devices,tile", [("box", "0,0,0", 4), ("lit_corner", "0,0", 16), ("box", "0", 16)])
def test_adapter_multi_context_bit_exact(oracle, tmp_path, scene, devices, tile):
    """render_samples_multi_gpu (the adapter's N-device form for the
    reference's main, main.cpp:256-285): one context per listed device (all
    on device 0 here), tile shards rendered by one host thread each, owned
    rows written into the reference's GridRenderPlane (a one-entry list renders
    on the listed device). Two progressive calls at
    a height that is not a multiple of tile x N: bit-identical to the oracle,
    each context uploaded the scene once."""
    _need_bin()
    Hm = 53
    r = subprocess.run([str(BIN), scene, str(W), str(Hm), str(SPP), str(CALLS), str(tmp_path / "a"), "16", "8",
                        devices, str(tile)], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    px = np.fromfile(tmp_path / "a.f32", np.float32)
    cnt = np.fromfile(tmp_path / "a.u32", np.uint32)
    desc = getattr(scenes, f"make_scene_{scene}")()
    ov, oc = ob.render_values(desc, capi.make_params(W, Hm, SPP * CALLS))
    ref = ob.accumulate(ov, oc)
    assert np.array_equal(cnt, ref["counters"])
    assert np.array_equal(px.view(np.uint32), ref["pixels"].view(np.uint32))
    out = r.stdout.split()
    assert np.float32(float(out[out.index("max_value") + 1])) == ref["pixel_max"].max()
    assert int(out[out.index("uploads") + 1]) == 1
    # each context keeps its own rows on its device: a later call moves at
    # most 16 B per pixel of the frame in all (each pixel by its one owner)
    assert 12 * W * Hm <= int(out[out.index("last_call_transfer_bytes") + 1]) <= 16 * W * Hm
