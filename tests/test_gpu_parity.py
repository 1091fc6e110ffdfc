"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar: bit-exact. Per-sample radiance values and GridRenderPlane drift codes
must be identical to the oracle's, and the accumulated GridRenderPlane state
(running-mean pixels, counters, sums, per-pixel max) identical to the
oracle's replay of GridRenderPlane::addRay (GridRenderPlane.cpp:61-75).
The BASELINE tolerance (<=1e-3 per-pixel L-inf) is asserted as well, but the
test requires 0.
"""
import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi, scenes

pytestmark = pytest.mark.gpu

L_INF_TOL = 1e-3  # BASELINE.json north_star per-channel tolerance


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _render_both(ctx, desc, p, oracle):
    ctx.upload_scene(desc)
    gv, gc = ctx.render_values(p)
    ov, oc = ob.render_values(desc, p, 0)
    return gv, gc, ov, oc


@pytest.mark.parametrize("n_rays,depth_max", [(16, 8), (16, 4), (4, 8), (16, 0), (1, 3), (0, 5)])
def test_values_bit_exact_box(gpu_ctx, oracle, n_rays, depth_max):
    desc = scenes.make_scene_box()
    p = capi.make_params(48, 40, 3, spp_offset=7, n_rays=n_rays, depth_max=depth_max)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), (
        f"{int((_bits(gv) != _bits(ov)).sum())} of {gv.size} samples differ; "
        f"max |d| = {np.abs(gv - ov).max()}")


def test_image_bit_exact_box(gpu_ctx, oracle):
    desc = scenes.make_scene_box()
    W, H = 64, 64
    gpu_ctx.upload_scene(desc)
    img = {k: np.zeros(W * H, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32),
                                                ("sums", np.float32), ("pixel_max", np.float32))}
    # two calls continue the same running mean (spp_offset)
    gpu_ctx.render(capi.make_params(W, H, 3, spp_offset=0), img)
    gpu_ctx.render(capi.make_params(W, H, 2, spp_offset=3), img)
    ov, oc = ob.render_values(desc, capi.make_params(W, H, 5, spp_offset=0))
    ref = ob.accumulate(ov, oc)
    for k in ("pixels", "sums", "pixel_max"):
        assert np.array_equal(_bits(img[k]), _bits(ref[k])), k
    assert np.array_equal(img["counters"], ref["counters"])
    assert np.abs(img["pixels"] - ref["pixels"]).max() <= L_INF_TOL


def test_counters_match_oracle(gpu_ctx, oracle):
    """The counting instance (IPT_FLAG_COUNTERS, 128 VGPRs) renders the same
    samples as the product instance and the oracle, and counts the oracle's
    events. (Round 5's frame-fallback code motion, built with
    -structurizecfg-skip-uniform-regions, broke exactly this: 10 of these 2048
    samples and traced_rays 338 341 vs 338 173)"""
    desc = scenes.make_scene_box()
    p = capi.make_params(32, 32, 2, flags=capi.IPT_FLAG_COUNTERS)
    gpu_ctx.upload_scene(desc)
    gpu_ctx.reset_counters()
    cv, cc = gpu_ctx.render_values(p)
    g = gpu_ctx.counters()
    pv, pc = gpu_ctx.render_values(capi.make_params(32, 32, 2))
    ov, oc, o = ob.render_values(desc, capi.make_params(32, 32, 2), 0, with_counters=True)
    assert np.array_equal(_bits(cv), _bits(pv)) and np.array_equal(cc, pc)
    assert np.array_equal(_bits(cv), _bits(ov)) and np.array_equal(cc, oc)
    for k in ("paths", "traced_rays", "surface_hits", "light_hits", "expanded_nodes",
              "iterations", "light_samples", "skipped", "light_traces", "drifted"):
        assert g[k] == o[k], (k, g[k], o[k])


@pytest.mark.parametrize("name", ["box_lights16", "box_lights256", "random64", "lit_corner", "square", "spheres300"])
def test_counters_match_oracle_scenes(gpu_ctx, oracle, name):
    """The oracle's event counts in the other instances: the single-light and
    lattice instances that take certain skips ahead in the prologue and at the
    end of the step (skip-ahead, pre-skip), and the generic ones that do not.
    Every skipped iteration must be counted as the reference counts it."""
    desc = {"box_lights16": lambda: scenes.make_scene_box_lights(4),
            "box_lights256": lambda: scenes.make_scene_box_lights(16),
            "random64": lambda: scenes.make_scene_random_lights(64),
            "lit_corner": scenes.make_scene_lit_corner,
            "square": scenes.make_scene_square_lit_by_square,
            "spheres300": lambda: scenes.make_scene_spheres(300)}[name]()
    W, H = 24, 20
    gpu_ctx.upload_scene(desc)
    gpu_ctx.reset_counters()
    vals, codes = gpu_ctx.render_values(capi.make_params(W, H, 2, flags=capi.IPT_FLAG_COUNTERS))
    g = gpu_ctx.counters()
    ov, oc, o = ob.render_values(desc, capi.make_params(W, H, 2), 0, with_counters=True)
    assert np.array_equal(_bits(vals), _bits(ov))
    for k in ("paths", "traced_rays", "surface_hits", "light_hits", "expanded_nodes",
              "iterations", "light_samples", "skipped", "drifted"):
        assert g[k] == o[k], (name, k, g[k], o[k])


@pytest.mark.parametrize("fn", sorted(capi.MATH_FNS.values()))
def test_device_math_matches_host(gpu_ctx, fn):
    """Device build of ipt_math.h == host build (which equals glibc, see
    test_math_exhaustive.py): all 2^24 RNG-reachable inputs + a strided sweep."""
    u = (np.arange(1 << 24, dtype=np.float32) * np.float32(2.0 ** -24))
    sweep = np.arange(0, 0x42f00000, 997, dtype=np.uint64).astype(np.uint32).view(np.float32)
    neg = -sweep[::7]
    for x in (u, np.sqrt(u, dtype=np.float32), sweep, neg):
        d = gpu_ctx.math_device(fn, x)
        h = capi.math_host(fn, x)
        same = (_bits(d) == _bits(h)) | (np.isnan(d) & np.isnan(h))
        if fn == capi.MATH_FNS["div_inrange_pairs"]:
            same |= (d == 0) & (h == 0)  # a zero quotient's sign is never observed (ipt_math.h)
        assert same.all(), (fn, x[~same][:4], d[~same][:4], h[~same][:4])


def test_cli_render_matches_oracle(gpu_ctx, oracle, tmp_path):
    """The C++ host path end to end: ipt_render (ipt_amd/host/, scene built by
    the C++ sample scenes, two progressive batches) writes the same
    GridRenderPlane pixels and counters as the oracle's accumulate."""
    import subprocess
    import __graft_entry__ as ge
    ge.build_host()
    W, H, spp, passes = 48, 40, 2, 2
    r = subprocess.run([str(ge.HOST_BIN), "--scene", "box", "--width", str(W), "--height", str(H),
                        "--spp", str(spp), "--passes", str(passes), "--out", str(tmp_path / "r.png"),
                        "--pfm", str(tmp_path / "r.pfm"), "--counts", str(tmp_path / "r.u32")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = (tmp_path / "r.pfm").read_bytes()
    hdr_end = raw.index(b"-1.0\n") + 5
    px = np.frombuffer(raw[hdr_end:], np.float32).reshape(H, W)[::-1].reshape(-1)
    cnt = np.fromfile(tmp_path / "r.u32", np.uint32)
    ov, oc = ob.render_values(scenes.make_scene_box(), capi.make_params(W, H, spp * passes))
    ref = ob.accumulate(ov, oc)
    assert np.array_equal(cnt, ref["counters"])
    assert np.array_equal(_bits(px), _bits(ref["pixels"]))
    assert (tmp_path / "r.png").read_bytes()[:4] == b"\x89PNG"


@pytest.mark.parametrize("devices,tile", [("0,0", 16), ("0,0,0", 4)])
def test_cli_multi_context_matches_oracle(gpu_ctx, oracle, tmp_path, devices, tile):
    """The C++ N-context renderer (MultiGpuRenderer, ipt_render --devices):
    one context per listed device (all on device 0 here), rows dealt in tiles,
    each context writing its own rows of the caller's plane; two progressive batches at a
    height that is not a multiple of tile_rows x N. Pixels and counters equal
    the oracle's replay (the reference's threads, main.cpp:256-285, write one
    plane; so do the contexts here)."""
    import subprocess
    import __graft_entry__ as ge
    ge.build_host()
    W, H, spp, passes = 40, 53, 2, 2
    r = subprocess.run([str(ge.HOST_BIN), "--scene", "box", "--width", str(W), "--height", str(H),
                        "--spp", str(spp), "--passes", str(passes), "--devices", devices, "--tile-rows", str(tile),
                        "--out", "", "--pfm", str(tmp_path / "r.pfm"), "--counts", str(tmp_path / "r.u32")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = (tmp_path / "r.pfm").read_bytes()
    px = np.frombuffer(raw[raw.index(b"-1.0\n") + 5:], np.float32).reshape(H, W)[::-1].reshape(-1)
    cnt = np.fromfile(tmp_path / "r.u32", np.uint32)
    ov, oc = ob.render_values(scenes.make_scene_box(), capi.make_params(W, H, spp * passes))
    ref = ob.accumulate(ov, oc)
    assert np.array_equal(cnt, ref["counters"])
    assert np.array_equal(_bits(px), _bits(ref["pixels"]))
    assert '"devices": %d' % len(devices.split(",")) in r.stdout
    # the contexts keep their rows on the device between batches: the last
    # batch moved 12 B per pixel down and at most 4 B up (the zeroed per-pixel
    # max, for the row runs whose previous maxima were not all zero)
    import json
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["last_batch_d2h_bytes"] == 12 * W * H
    assert js["last_batch_h2d_bytes"] <= 4 * W * H


@pytest.mark.parametrize("fn", ["acos_f64_f32", "sqrtf", "div_pairs", "div_inrange_pairs", "longer_pairs",
                                "udiv_exact_pairs", "sqrt_inrange", "frame_angle_sin", "frame_angle_cos"])
def test_fast_math_exhaustive(gpu_ctx, fn):
    """The device fast paths equal their exact references on all 2^32 inputs:
    (float)acos((double)x) (Ziv test + exact fallback) vs the fdlibm
    restatement (== glibc on every float, test_math_exhaustive.py); sqrtf and
    a/b (range-guarded correction cores, ipt_math.h) vs the compiler's IEEE
    sequences (division over 2^32 in-range / zero-numerator pairs); the
    range-free division of the box planes (div_inrange_) over the same pairs;
    the squares-first length comparison (longer_sq) against sqrtf(x) >
    sqrtf(y) over 2^32 near-tie and unrelated pairs; the 32-bit work-unit
    decomposition (udiv_exact) against integer division over 2^32 pairs; the
    range-free root (frame builds) against sqrtf on its range; the frame
    table's (sin, cos) of the RotateDdf angle, looked up by to.z's bits,
    against the computed angle for every float z (incl. the table's ends
    2^-8 and 1, the computed |z| < 2^-8 and NaN)."""
    bad, first = gpu_ctx.math_selfcheck(capi.MATH_FNS[fn])
    assert bad == 0, (fn, bad, hex(first))


@pytest.mark.parametrize("fn", ["SELFCHECK_RCP1", "SELFCHECK_RCP2", "SELFCHECK_DIV_PAIRS", "SELFCHECK_DIV_ONES"])
def test_short_division_exhaustive(gpu_ctx, fn):
    """The round-5 range-free reciprocal (the hardware rcp and one Newton
    correction) equals the round-4 three-correction sequence on all 2^32
    floats (17; 18: two corrections), and the range-free division with one
    quotient residual step equals IEEE a/b on 2^32 hashed pairs over its range
    (19) and on 2^32 pairs whose divisors have all-ones-like significands
    (20, the hard case of Markstein's one-step theorem)."""
    bad, first = gpu_ctx.math_selfcheck(getattr(capi, fn))
    assert bad == 0, (fn, bad, hex(first))


def test_short_division_every_significand_pair(gpu_ctx):
    """the one-residual-step division (div_inrange_) is proved, not
    sampled. Every pair of significands a, b in [1, 2) -- all 2^46 -- gives
    IEEE a/b (21), and the reciprocal it starts from scales exactly over the
    operand range [2^-40, 2^41) for all 2^32 floats (22); the other operations
    are IEEE and commute with scaling by powers of two in that range, so the
    division equals a/b on every in-range operand pair (ipt_math.h
    div_inrange_). Run in 2^40-pair slices (about a second each)."""
    bad, first = gpu_ctx.math_selfcheck(capi.SELFCHECK_RCP_SCALING)
    assert bad == 0, ("rcp scaling", bad, hex(first))
    step = 1 << 40
    for lo in range(0, 1 << 46, step):
        bad, first = gpu_ctx.math_selfcheck(capi.SELFCHECK_DIV_ALL_SIGNIFICANDS, lo, lo + step)
        assert bad == 0, ("division", lo, bad, hex(first))


def test_fast_frame_matches_exact(gpu_ctx):
    """The sphere-in-box frame without glm's zero terms (make_frame_sc_fast)
    equals the exact RotateDdf build (make_frame_sc<true>) bit for bit on every
    direction where it reports ok: 2^32 directions hashed from the bit
    pattern, a quarter of them edge cases (zero, -0, tiny or ~1e-7 x and y,
    x = +-y) that must either match or be handed to the exact build."""
    bad, first = gpu_ctx.math_selfcheck(capi.SELFCHECK_FRAME_FAST)
    assert bad == 0, (bad, hex(first))


@pytest.mark.parametrize("n_shards", [2, 3])
def test_sharded_render_matches_whole_frame(gpu_ctx, oracle, n_shards):
    """Tile-sharded rendering (one shard per call, as one rank per GPU does)
    assembled by summation equals the whole-frame render bit-for-bit."""
    desc = scenes.make_scene_box()
    W, H, tile = 40, 50, 8
    gpu_ctx.upload_scene(desc)

    def blank():
        return {k: np.zeros(W * H, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32),
                                                     ("sums", np.float32), ("pixel_max", np.float32))}

    whole = blank()
    gpu_ctx.render(capi.make_params(W, H, 3), whole)
    acc = blank()
    for s in range(n_shards):
        part = blank()
        p = capi.make_params(W, H, 3, tile_rows=tile, n_shards=n_shards, shard_id=s)
        gpu_ctx.render(p, part)
        owned, _ = capi.shard_plan(p)
        mask = np.repeat(owned, W)
        for k in acc:
            assert not part[k][~mask].any(), "shard wrote outside its rows"
            acc[k] = acc[k] + part[k]
    for k in ("pixels", "sums", "pixel_max"):
        assert np.array_equal(_bits(acc[k]), _bits(whole[k])), k
    assert np.array_equal(acc["counters"], whole["counters"])


@pytest.mark.parametrize("k", [2, 4, 16])
def test_many_lights_bit_exact(gpu_ctx, oracle, k):
    """BASELINE configs[4] scene family: the [0] light split into k x k
    co-planar squares (k=16: 256 emitters, global-memory light mode)."""
    desc = scenes.make_scene_box_lights(k)
    p = capi.make_params(24, 20, 2, n_rays=16, depth_max=8)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


@pytest.mark.parametrize("n", [17, 64, 300])
def test_random_lights_bit_exact(gpu_ctx, oracle, n):
    """Overlapping emitters of random shape/orientation above kLdsLights: the
    index-ordered light BVH must reproduce the full scan's nearest-light rule
    and the running UnionDdf sum with several hits per ray."""
    desc = scenes.make_scene_random_lights(n, seed=7)
    p = capi.make_params(20, 16, 2, n_rays=8, depth_max=6)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


def _light_counters(ctx, desc):
    ctx.upload_scene(desc)
    p = capi.make_params(32, 32, 1, n_rays=16, depth_max=8, flags=capi.IPT_FLAG_COUNTERS)
    img = {"pixels": np.zeros(32 * 32, np.float32), "counters": np.zeros(32 * 32, np.uint32)}
    ctx.reset_counters()
    ctx.render(p, img)
    return ctx.counters()


def test_light_bvh_active(monkeypatch):
    """With the lattice lookup off (IPT_LIGHT_GRID=0) the 256-emitter scene runs
    the light BVH: far fewer light tests than the reference's L traces per ray,
    and the reference event count intact."""
    monkeypatch.setenv("IPT_LIGHT_GRID", "0")
    ctx = capi.Context(0)
    try:
        c = _light_counters(ctx, scenes.make_scene_box_lights(16))
    finally:
        ctx.close()
    assert c["light_nodes"] > 0
    assert c["light_tests"] < 0.1 * 256 * c["traced_rays"]
    assert c["light_traces"] >= 256 * c["traced_rays"]


def test_light_grid_active(gpu_ctx):
    """The 256 co-planar emitters lie on a lattice: each ray tests the lights of
    the one to four cells around its plane point (no BVH nodes), and the
    reference event count stays intact."""
    c = _light_counters(gpu_ctx, scenes.make_scene_box_lights(16))
    assert c["light_nodes"] == 0
    assert 0 < c["light_tests"] < 1.2 * c["traced_rays"]
    assert c["light_traces"] >= 256 * c["traced_rays"]


@pytest.mark.parametrize("k", [5, 8, 16, 32])
def test_light_grid_bit_exact(gpu_ctx, oracle, k):
    """kLightsGridA10: the lattice lookup finds every light the full scan hits
    (k x k emitters, 25 to 1 024 lights) -- bit-exact vs the oracle, with more
    samples per pixel so that many plane points fall within the lookup's
    margin of a cell edge."""
    desc = scenes.make_scene_box_lights(k)
    p = capi.make_params(32, 24, 4, n_rays=8, depth_max=6)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


@pytest.mark.parametrize("k", [8, 16])
def test_light_grid_lds_and_global_records_bit_exact(oracle, monkeypatch, k):
    """The lattice instances with the records in LDS (one 1024-thread workgroup
    per CU, the default where the LDS fits) and in global memory
    (IPT_LATTICE_LDS=0, 256-thread workgroups) give the same bits as the
    oracle, at depth 8 / 16 rays (C5's stack depth)."""
    desc = scenes.make_scene_box_lights(k)
    p = capi.make_params(24, 16, 2, n_rays=16, depth_max=8)
    out = []
    for lds in ("1", "0"):
        monkeypatch.setenv("IPT_LATTICE_LDS", lds)
        ctx = capi.Context(0)
        try:
            gv, gc, ov, oc = _render_both(ctx, desc, p, oracle)
        finally:
            ctx.close()
        assert np.array_equal(gc, oc)
        assert np.array_equal(_bits(gv), _bits(ov)), (lds, int((_bits(gv) != _bits(ov)).sum()))
        out.append(gv)
    assert np.array_equal(_bits(out[0]), _bits(out[1]))


@pytest.mark.parametrize("variant", ["nudged", "gap", "mixed_axes"])
def test_light_grid_fallback_bit_exact(gpu_ctx, oracle, variant):
    """Light sets that are not a lattice (one emitter moved by a tenth of a
    cell, one emitter with swapped axes) take the light BVH; a lattice with an
    empty row keeps the cell lookup (empty cells): all bit-exact."""
    desc = scenes.make_scene_box_lights(8)
    L = [dict(l) for l in desc["lights"]]
    if variant == "nudged":
        c = list(L[9]["position"])
        c[1] = float(np.float32(c[1] + np.float32(0.0025)))
        L[9]["position"] = c
    elif variant == "gap":
        L = L[:8] + L[16:]
    else:
        L[3]["x_axis"], L[3]["y_axis"] = L[3]["y_axis"], L[3]["x_axis"]
    desc = dict(desc, lights=L)
    p = capi.make_params(24, 20, 2, n_rays=8, depth_max=6)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


@pytest.mark.parametrize("name", ["make_scene_square_lit_by_square", "make_scene_lit_corner"])
@pytest.mark.parametrize("n_rays,depth_max", [(16, 8), (4, 5)])
def test_sample_scenes_floor_corner_bit_exact(gpu_ctx, oracle, name, n_rays, depth_max):
    """sample_scenes.cpp:73-108: GeometryFloor (unrotated CosineDdf, identity
    frame) with a square light; GeometryCorner (three faces, strict-<) with
    a triangle light."""
    desc = getattr(scenes, name)()
    p = capi.make_params(40, 32, 2, n_rays=n_rays, depth_max=depth_max)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())
    assert (ov > 0).mean() > 0.05  # the scene is lit


@pytest.mark.parametrize("n_rays,depth_max", [(16, 8), (4, 6)])
def test_sample_scene_fractal_bit_exact(gpu_ctx, oracle, n_rays, depth_max):
    """sample_scenes.cpp:43-55: FractalSpheres (sphere list, no walls) lit by a
    SphereLight (its own intersection and sampler, lighting.cpp:11-36,146-193)."""
    desc = scenes.make_scene_fractal()
    p = capi.make_params(48, 40, 2, n_rays=n_rays, depth_max=depth_max)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())
    assert (ov > 0).any()  # the sphere light reaches the camera


@pytest.mark.parametrize("n_rays,depth_max", [(16, 8), (8, 5)])
def test_sample_scene_smallpt_bit_exact(gpu_ctx, oracle, n_rays, depth_max):
    """sample_scenes.cpp:57-71: smallpt's room (GeometrySmallPt, double
    precision Sphere::intersect, flipped room normals) with a square light."""
    desc = scenes.make_scene_smallpt()
    p = capi.make_params(40, 32, 2, n_rays=n_rays, depth_max=depth_max)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())
    assert (ov > 0).mean() > 0.05


@pytest.mark.parametrize("geom", ["box", "fractal"])
def test_round_lights_bit_exact(gpu_ctx, oracle, geom):
    """Sphere, point and inverted-sphere (outer) lights mixed with area lights:
    CollectionLighting's nearest rule, UnionDdf over all of them, the point
    light never hit (lighting.h:31-73)."""
    base = scenes.make_scene_box() if geom == "box" else scenes.make_scene_fractal()
    desc = dict(base)
    desc["lights"] = list(base["lights"]) + [
        scenes.sphere_light((0.3, 0.2, 0.4), 0.15, 0.7),
        scenes.point_light((-0.4, 0.3, -0.2), 0.05, 0.5),
        scenes.outer_light(9.0, 0.05),
        scenes.sphere_light((-0.5, -0.6, 0.5), 0.2, 1.3),
    ]
    p = capi.make_params(40, 32, 2, n_rays=8, depth_max=6)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


def test_spheres_in_box_c3_scene(gpu_ctx, oracle):
    """The full 10k-sphere scene of BASELINE configs[2] (bench C3): BVH walk
    (octant orders, open-floor rays with best = inf) against the oracle's scan."""
    desc = scenes.make_scene_spheres(10000, seed=1)
    p = capi.make_params(12, 10, 1, n_rays=8, depth_max=4)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


@pytest.mark.parametrize("n", [1, 50, 400, 3000])
def test_spheres_in_box_bit_exact(gpu_ctx, oracle, n):
    """BASELINE configs[2] scene family: box planes + n seeded spheres with
    FractalSpheres' acceptance rule."""
    desc = scenes.make_scene_spheres(n, seed=1)
    p = capi.make_params(20, 16, 1, n_rays=16, depth_max=8)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


@pytest.mark.parametrize("lds", ["0", "1"])
@pytest.mark.parametrize("desc_fn", [lambda: scenes.make_scene_box_lights(16),
                                     lambda: scenes.make_scene_random_lights(300, seed=7)])
def test_light_bvh_in_lds_bit_exact(oracle, monkeypatch, desc_fn, lds):
    """The light BVH staged in LDS (default) and kept in global memory
    (IPT_LNODES_LDS=0, read at ipt_create) walk the same nodes: bit-exact vs
    the oracle."""
    monkeypatch.setenv("IPT_LNODES_LDS", lds)
    monkeypatch.setenv("IPT_LIGHT_GRID", "0")  # the lattice scene would not walk the BVH
    ctx = capi.Context(0)
    try:
        desc = desc_fn()
        p = capi.make_params(20, 16, 2, n_rays=8, depth_max=6)
        gv, gc, ov, oc = _render_both(ctx, desc, p, oracle)
        assert np.array_equal(gc, oc)
        assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())
    finally:
        ctx.close()


def _lattice_scene(k, r, cam_pos, cam_dir):
    sp = []
    for i in range(k):
        for j in range(k):
            for m in range(k):
                c = [float(np.float32(-0.8 + 1.6 * (q + 0.5) / k)) for q in (i, j, m)]
                sp.append((c, float(np.float32(r))))
    d = scenes.make_scene_spheres(1, seed=1)
    d["spheres"] = sp
    d["camera"] = scenes.simple_camera(cam_pos, cam_dir)
    return d


@pytest.mark.parametrize("k,r,cam_pos,cam_dir", [
    (10, 0.03, (0.0, -3.0, 0.0), (0.0, 1.0, 0.0)),      # axis-aligned camera, rays along lattice rows
    (8, 0.09, (0.05, 0.0, 0.05), (0.3, 1.0, 0.2)),      # overlapping spheres, camera inside the grid
    (12, 0.02, (-0.95, -0.95, -0.95), (1.0, 1.0, 1.0)),  # diagonal through cell corners
])
def test_sphere_grid_adversarial_bit_exact(gpu_ctx, oracle, k, r, cam_pos, cam_dir):
    """The uniform sphere grid (> 256 spheres inside the box) on lattices whose
    rows line up with the camera, overlapping spheres around an inside camera,
    and a diagonal view through cell corners: the DDA walk with its outward
    registration and stopping margin must reproduce the oracle's linear scan
    (FractalSpheres.cpp:75-84) bit for bit."""
    desc = _lattice_scene(k, r, cam_pos, cam_dir)
    p = capi.make_params(16, 12, 1, n_rays=8, depth_max=5)
    gpu_ctx.upload_scene(desc)
    gpu_ctx.reset_counters()
    gv, gc = gpu_ctx.render_values(p)
    ov, oc = ob.render_values(desc, p, 0)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


@pytest.mark.parametrize("fail_at", [1, 2, 7])
def test_failed_upload_leaves_no_scene(gpu_ctx, oracle, monkeypatch, fail_at):
    """ipt_upload_scene is transactional (ipt_capi.h): an allocation failure in
    the second upload (injected at its k-th device allocation) returns an error
    and leaves the context with no scene, so the next render fails with
    IPT_E_NOSCENE instead of launching on freed or null scene buffers; a later
    upload recovers and renders bit-exactly."""
    desc = scenes.make_scene_spheres(400, seed=1)  # sphere grid + lights + spheres: 7 device buffers
    p = capi.make_params(16, 12, 1, n_rays=8, depth_max=5)
    gpu_ctx.upload_scene(scenes.make_scene_box())
    gpu_ctx.render_values(p)
    monkeypatch.setenv("IPT_TEST_FAIL_UPLOAD_ALLOC", str(fail_at))
    with pytest.raises(capi.IptError) as e:
        gpu_ctx.upload_scene(desc)
    assert e.value.code == capi.IPT_E_OOM
    monkeypatch.delenv("IPT_TEST_FAIL_UPLOAD_ALLOC")
    with pytest.raises(capi.IptError) as e:
        gpu_ctx.render_values(p)
    assert e.value.code == capi.IPT_E_NOSCENE
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov))


@pytest.mark.parametrize("light", [
    # x along y, y along x, facing down: sample_scenes[0]'s pattern (kLightsOneA10)
    {"position": [-0.3, 0.2, 0.7], "x_axis": [0.0, 0.3, 0.0], "y_axis": [0.25, 0.0, 0.0], "power": 2.0, "type": 0},
    # x along x, y along -y, facing down (kLightsOneA01)
    {"position": [-0.2, 0.4, 0.6], "x_axis": [0.3, 0.0, 0.0], "y_axis": [0.0, -0.3, 0.0], "power": 1.0, "type": 0},
    # triangle with the A10 pattern
    {"position": [0.3, -0.5, 0.5], "x_axis": [0.0, 0.4, 0.0], "y_axis": [0.4, 0.0, 0.0], "power": 1.0, "type": 1},
    # a corner component exactly 0: the generic code (the reduced forms need P != 0)
    {"position": [0.0, -0.9, -0.15], "x_axis": [0.0, 0.2, 0.0], "y_axis": [0.2, 0.0, 0.0], "power": 1.0, "type": 0},
    # facing up (A10 axes swapped sign): light seen from below only by its back
    {"position": [0.1, -0.9, -0.6], "x_axis": [0.0, -0.2, 0.0], "y_axis": [0.2, 0.0, 0.0], "power": 1.0, "type": 0},
])
def test_axis_aligned_single_light_bit_exact(gpu_ctx, oracle, light):
    """A single axis-aligned AreaLight runs the reduced light trace / pdf /
    sample forms (light_trace_ax etc., ipt_path.h: the zero components'
    products dropped where they are exact no-ops); the images must stay
    bit-identical to the oracle's generic arithmetic, incl. the fallback cases."""
    desc = scenes.make_scene_box()
    desc["lights"] = [light]
    p = capi.make_params(40, 32, 2, n_rays=16, depth_max=8)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())


@pytest.mark.parametrize("cfg", ["c2", "c4", "c5", "c3"])
def test_full_size_rows_bit_exact(gpu_ctx, oracle, cfg):
    """BASELINE.json configs at their full frame sizes, one pass each (C2: the
    box at 1024^2, n_rays 16, depth 8; C4: the box at 4096^2 (one GPU's whole
    frame); C5: 256 emitters at 2048^2, the light lattice; C3: 10 000 spheres
    at 1024^2, the sphere grid): every sample of the frame rendered on the GPU,
    and strided source pixels of it recomputed by the oracle, bit-exact."""
    # (rows, columns) sampled so that the oracle's share stays a few seconds
    if cfg == "c2":
        desc, W, rs, rp, cs, cp = scenes.make_scene_box(), 1024, 128, 37, 1, 0
    elif cfg == "c4":
        desc, W, rs, rp, cs, cp = scenes.make_scene_box(), 4096, 1024, 333, 2, 1
    elif cfg == "c5":
        desc, W, rs, rp, cs, cp = scenes.make_scene_box_lights(16), 2048, 1024, 101, 4, 3
    else:
        desc, W, rs, rp, cs, cp = scenes.make_scene_spheres(10000, seed=1), 1024, 1024, 517, 32, 5
    p = capi.make_params(W, W, 1, spp_offset=17, n_rays=16, depth_max=8)
    gpu_ctx.upload_scene(desc)
    gv, gc = gpu_ctx.render_values(p)
    ov, rows, cols = ob.render_rows_values(desc, p, rs, rp, cs, cp, n_threads=16)
    sel = gv[:, rows, :][:, :, cols]
    assert np.array_equal(_bits(sel), _bits(ov)), int((_bits(sel) != _bits(ov)).sum())
    assert (gc != 0xFF).mean() > 0.99


def test_c1_config_bit_exact(gpu_ctx, oracle):
    """BASELINE.json configs[0] verbatim (C1, the reference's CPU-runnable
    case): sample_scenes[0] at 256^2, 16 spp, 4 bounces (depth_max 4, the
    reference default, /root/reference/src/main.cpp:95), n_rays 16. All
    1 048 576 samples of the frame rendered on the GPU are bit-identical to
    the oracle's, and so is the accumulated GridRenderPlane (pixels,
    counters, sums, max) of the same frame rendered by ipt_render."""
    desc = scenes.make_scene_box()
    p = capi.make_params(256, 256, 16, n_rays=16, depth_max=4)
    gv, gc, ov, oc = _render_both(gpu_ctx, desc, p, oracle)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), int((_bits(gv) != _bits(ov)).sum())
    img = {k: np.zeros(256 * 256, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32),
                                                    ("sums", np.float32), ("pixel_max", np.float32))}
    gpu_ctx.render(p, img)
    ref = ob.accumulate(ov, oc)
    for k in ("pixels", "sums", "pixel_max"):
        assert np.array_equal(_bits(img[k]), _bits(ref[k])), k
    assert np.array_equal(img["counters"], ref["counters"])
    assert abs(float(ref["pixels"].mean()) - 0.0654) < 0.002  # 0.06535 at 640^2


def _jittered_powers(desc, rel, seed=3):
    """desc with every light's power scaled by 1 + rel*u, u uniform in [-1, 1)."""
    rng = np.random.default_rng(seed)
    for L in desc["lights"]:
        L["power"] = float(np.float32(L["power"]) * np.float32(1.0 + rel * (2.0 * rng.random() - 1.0)))
    return desc


@pytest.mark.parametrize("case", ["lattice_equal", "lattice_jitter", "random_jitter", "lattice_uneven"])
def test_near_uniform_cdf_pick(gpu_ctx, oracle, case):
    """The many-light pick from floor(r 2^e) and two cdf entries (IPT_CDF_POW2):
    nearly equal powers (the 256-emitter lattice's own rounding, or powers
    jittered by 1e-4 so that entries sit on both sides of (i+1) 2^-e), on the
    lattice and on the light-BVH instance; and powers too uneven for it (the
    bucket-table pick). Values and counters bit-exact against the oracle."""
    desc = {"lattice_equal": lambda: scenes.make_scene_box_lights(16),
            "lattice_jitter": lambda: _jittered_powers(scenes.make_scene_box_lights(16), 1e-4),
            "random_jitter": lambda: _jittered_powers(
                {**scenes.make_scene_random_lights(64), "lights": [
                    {**L, "power": 0.5} for L in scenes.make_scene_random_lights(64)["lights"]]}, 1e-4),
            "lattice_uneven": lambda: _jittered_powers(scenes.make_scene_box_lights(16), 0.5)}[case]()
    W, H = 32, 24
    gpu_ctx.upload_scene(desc)
    gpu_ctx.reset_counters()
    vals, _ = gpu_ctx.render_values(capi.make_params(W, H, 2, flags=capi.IPT_FLAG_COUNTERS))
    g = gpu_ctx.counters()
    ov, _, o = ob.render_values(desc, capi.make_params(W, H, 2), 0, with_counters=True)
    assert np.array_equal(_bits(vals), _bits(ov))
    for k in ("iterations", "light_samples", "skipped", "light_hits"):
        assert g[k] == o[k], (case, k, g[k], o[k])


@pytest.mark.parametrize("n_shards", [1, 3])
def test_resident_render_sees_caller_changes(oracle, n_shards):
    """ipt_render keeps the rows a context accumulates on its device between
    calls (ABI 5). The caller's host plane stays the truth: rows the caller
    changes between calls are uploaded again, rows it leaves alone are not,
    and the result equals a fresh context's render of the same plane. Shards
    (one context each) share one host plane and touch only their own rows."""
    desc = scenes.make_scene_box()
    W, H, tile = 40, 37, 4
    ctxs = [capi.Context(0) for _ in range(n_shards)]
    fresh = [capi.Context(0) for _ in range(n_shards)]
    try:
        for c in ctxs + fresh:
            c.upload_scene(desc)

        def params(spp, off, k):
            return capi.make_params(W, H, spp, spp_offset=off, tile_rows=tile if n_shards > 1 else 0,
                                    n_shards=n_shards, shard_id=k)

        img = {k: np.zeros(W * H, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32),
                                                    ("pixel_max", np.float32))}
        for k, c in enumerate(ctxs):
            c.render(params(2, 0, k), img)
        # an untouched plane: the next call uploads nothing but the zeroed max
        img["pixel_max"][:] = 0
        before = {k: v.copy() for k, v in img.items()}
        for k, c in enumerate(ctxs):
            c.render(params(1, 2, k), img)
            h2d, d2h = c.transfer_bytes()
            assert h2d <= 4 * W * H and d2h > 0
        # the caller edits the plane (a row of pixels, some counters), then renders on
        img["pixels"][5 * W:6 * W] = 0.25
        img["counters"][17 * W + 3:17 * W + 9] += 7
        img["pixel_max"][:] = 0
        edited = {k: v.copy() for k, v in img.items()}
        for k, c in enumerate(ctxs):
            c.render(params(2, 3, k), img)
        ref = {k: v.copy() for k, v in edited.items()}
        for k, c in enumerate(fresh):
            c.render(params(2, 3, k), ref)
        for k in img:
            assert np.array_equal(_bits(img[k]), _bits(ref[k])), k
        assert not np.array_equal(_bits(before["pixels"]), _bits(img["pixels"]))
    finally:
        for c in ctxs + fresh:
            c.close()
