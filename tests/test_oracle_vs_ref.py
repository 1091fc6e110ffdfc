"""The CPU oracle against the reference's OWN compiled code.

tests/golden/ref_*.bin were produced by oracle/ref_kat.cpp linked with the
reference translation units (oracle/build_ref.sh, -O2, from /root/reference).
Every comparison is bit-exact (float32 bit patterns).
"""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

import oracle_binding as ob

GOLD = Path(__file__).resolve().parent / "golden"


def load(name, width):
    a = np.fromfile(GOLD / name, dtype=np.float32)
    assert a.size % width == 0
    return a.reshape(-1, width)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def arr(v):
    return np.ascontiguousarray(v, np.float32)


@pytest.fixture(scope="module")
def lib(oracle):
    return ob.setup_probes()


def test_box_plane(lib):
    R = load("ref_box_plane.bin", 10)
    got = np.array([lib.ipt_oracle_box_plane(ob.fptr(arr(r[0:3])), ob.fptr(arr(r[3:6])),
                                              ob.fptr(arr(r[6:9]))) for r in R], np.float32)
    assert np.array_equal(bits(got), bits(R[:, 9]))
    assert np.isfinite(R[:, 9]).sum() > 200  # the fixture does exercise hits


def test_sphere(lib):
    R = load("ref_sphere.bin", 8)
    got = np.array([lib.ipt_oracle_sphere(float(r[0]), ob.fptr(arr(r[1:4])), ob.fptr(arr(r[4:7])))
                    for r in R], np.float32)
    assert np.array_equal(bits(got), bits(R[:, 7]))
    assert np.isfinite(R[:, 7]).sum() > 200


def test_area_light_ctor_and_trace(lib):
    R = load("ref_area_light.bin", 24)
    hits = 0
    for r in R:
        L = ob.area_light_struct(r[0:3], r[3:6], r[6:9], r[9], int(r[10]))
        asp = np.zeros(2, np.float32)
        lib.ipt_oracle_area_light(C.byref(L), ob.fptr(asp))
        assert np.array_equal(bits(asp), bits(r[17:19]))
        pos = np.zeros(3, np.float32)
        h = lib.ipt_oracle_light_trace(C.byref(L), ob.fptr(arr(r[11:14])), ob.fptr(arr(r[14:17])),
                                       ob.fptr(pos))
        assert h == int(r[19])
        if h:
            hits += 1
            assert np.array_equal(bits(pos), bits(r[20:23]))
    assert hits > 500


def test_area_light_sample(lib):
    R = load("ref_light_sample.bin", 18)
    for r in R:
        L = ob.area_light_struct(r[0:3], r[3:6], r[6:9], 1.0, int(r[9]))
        out = np.zeros(6, np.float32)
        lib.ipt_oracle_light_sample_uv(C.byref(L), float(r[10]), float(r[11]), ob.fptr(out))
        assert np.array_equal(bits(out), bits(r[12:18]))


def test_simple_camera(lib):
    R = load("ref_camera.bin", 23)
    for r in R:
        ru = np.zeros(6, np.float32)
        lib.ipt_oracle_camera(ob.fptr(arr(r[0:3])), ob.fptr(arr(r[3:6])), ob.fptr(arr(r[6:9])),
                              ob.fptr(ru))
        assert np.array_equal(bits(ru), bits(r[11:17]))
        d = np.zeros(3, np.float32)
        lib.ipt_oracle_camera_ray(ob.fptr(arr(r[3:6])), ob.fptr(arr(r[11:14])),
                                  ob.fptr(arr(r[14:17])), float(r[9]), float(r[10]), ob.fptr(d))
        assert np.array_equal(bits(d), bits(r[20:23]))
        assert np.array_equal(bits(r[17:20]), bits(r[0:3]))  # origin = position


def test_scene_box_flattening(lib):
    """ipt_amd.scenes.make_scene_box() reproduces make_scene_box()'s objects."""
    from ipt_amd import scenes

    R = np.fromfile(GOLD / "ref_scene_box.bin", dtype=np.float32)
    desc = scenes.make_scene_box()
    cam = desc["camera"]
    mine = np.array(cam["position"] + cam["direction"] + cam["right"] + cam["up"], np.float32)
    assert np.array_equal(bits(mine), bits(R[0:12]))
    assert int(R[12]) == 1
    L = desc["lights"][0]
    asp = np.zeros(2, np.float32)
    Ls = ob.area_light_struct(L["position"], L["x_axis"], L["y_axis"], L["power"], L["type"])
    lib.ipt_oracle_area_light(C.byref(Ls), ob.fptr(asp))
    assert np.array_equal(bits(np.array(L["position"] + [L["power"], asp[0]], np.float32)),
                          bits(R[13:18]))
    probes = R[18:].reshape(-1, 11)
    n_hit = 0
    for r in probes:
        out = np.zeros(4, np.float32)
        h = lib.ipt_oracle_collection_trace(C.byref(Ls), 1, ob.fptr(arr(r[0:3])),
                                            ob.fptr(arr(r[3:6])), ob.fptr(out))
        assert h == int(r[6])
        if h:
            n_hit += 1
            assert np.array_equal(bits(out), bits(r[7:11]))
    assert n_hit > 20


def test_collection_lighting_nearest(lib):
    R = np.fromfile(GOLD / "ref_collection.bin", dtype=np.float32)
    lights = R[:160].reshape(16, 10)
    from ipt_amd.capi import AreaLight

    arrL = (AreaLight * 16)()
    for i, l in enumerate(lights):
        arrL[i] = ob.area_light_struct(l[0:3], l[3:6], l[6:9], l[9], 0)
    probes = R[160:].reshape(-1, 11)
    hits = 0
    for r in probes:
        out = np.zeros(4, np.float32)
        h = lib.ipt_oracle_collection_trace(arrL, 16, ob.fptr(arr(r[0:3])), ob.fptr(arr(r[3:6])),
                                            ob.fptr(out))
        assert h == int(r[6])
        if h:
            hits += 1
            assert np.array_equal(bits(out), bits(r[7:11]))
    assert hits > 500


def _mat_vec(m9, v):
    """glm mat3*vec3 in float32, operation order of type_mat3x3.inl:468-474."""
    m = m9.reshape(3, 3)  # m[c][r]
    f = np.float32
    return np.array([f(f(m[0, r] * v[0]) + f(m[1, r] * v[1])) + f(m[2, r] * v[2])
                     for r in range(3)], np.float32)


def test_rotate_ddf(lib):
    R = load("ref_rotate.bin", 33)
    for r in R:
        m = np.zeros(18, np.float32)
        lib.ipt_oracle_rotate(ob.fptr(arr(r[0:3])), ob.fptr(m))
        assert np.array_equal(bits(m[:9]), bits(r[3:12])), r[0:3]
        assert np.array_equal(bits(m[9:]), bits(r[12:21])), r[0:3]
        assert np.array_equal(bits(_mat_vec(m[:9], r[21:24])), bits(r[24:27]))
        assert np.array_equal(bits(_mat_vec(m[9:], r[27:30])), bits(r[30:33]))


def test_grid_render_plane(lib):
    R = np.fromfile(GOLD / "ref_grid.bin", dtype=np.float32)
    W, H, n = int(R[0]), int(R[1]), int(R[2])
    xyv = arr(R[3:3 + 3 * n])
    ref_px = R[3 + 3 * n:3 + 3 * n + W * H]
    ref_cnt = R[3 + 3 * n + W * H:3 + 3 * n + 2 * W * H]
    ref_max = R[-1]
    px = np.zeros(W * H, np.float32)
    cnt = np.zeros(W * H, np.uint32)
    mx = np.zeros(1, np.float32)
    lib.ipt_oracle_grid_addray(W, H, n, ob.fptr(xyv), ob.fptr(px),
                               cnt.ctypes.data_as(C.POINTER(C.c_uint32)), ob.fptr(mx))
    assert np.array_equal(bits(px), bits(ref_px))
    assert np.array_equal(cnt.astype(np.float32), ref_cnt)
    assert mx[0] == ref_max
    # the off-by-one of GridRenderPlane.cpp:67: row H-1 only receives samples
    # with y*H landing exactly on an integer
    assert ref_cnt.reshape(H, W)[0].sum() > ref_cnt.reshape(H, W)[H // 2].sum()


def _ref_scenes():
    """ref_scenes.bin: square_lit_by_square, lit_corner, fractal, smallpt."""
    R = np.fromfile(GOLD / "ref_scenes.bin", dtype=np.float32)
    n, pos, out = int(R[0]), 1, []
    for _ in range(n):
        head = R[pos:pos + 13]
        pos += 13
        nl = int(head[12])
        lights = R[pos:pos + 5 * nl].reshape(nl, 5)
        pos += 5 * nl
        probes = R[pos:pos + 200 * 11].reshape(200, 11)
        pos += 200 * 11
        out.append((head[:12], lights, probes))
    assert pos == R.size
    return out


@pytest.mark.parametrize("idx,name", [(0, "make_scene_square_lit_by_square"), (1, "make_scene_lit_corner"),
                                      (2, "make_scene_fractal"), (3, "make_scene_smallpt")])
def test_area_light_scenes_flattening(lib, idx, name):
    """ipt_amd.scenes reproduces sample_scenes.cpp's floor, corner and fractal
    scenes: camera fields, light fields (AreaLight, triangle AreaLight,
    SphereLight) and the light's own traceRay on probes."""
    from ipt_amd import scenes

    cam_ref, lights_ref, probes = _ref_scenes()[idx]
    desc = getattr(scenes, name)()
    cam = desc["camera"]
    mine = np.array(cam["position"] + cam["direction"] + cam["right"] + cam["up"], np.float32)
    assert np.array_equal(bits(mine), bits(cam_ref))
    assert len(desc["lights"]) == len(lights_ref) == 1
    L = desc["lights"][0]
    asp = np.zeros(2, np.float32)
    Ls = ob.area_light_struct(L["position"], L["x_axis"], L["y_axis"], L["power"], L["type"])
    lib.ipt_oracle_area_light(C.byref(Ls), ob.fptr(asp))
    assert np.array_equal(bits(np.array(L["position"] + [L["power"], asp[0]], np.float32)), bits(lights_ref[0]))
    n_hit = 0
    for r in probes:
        out = np.zeros(4, np.float32)
        h = lib.ipt_oracle_collection_trace(C.byref(Ls), 1, ob.fptr(arr(r[0:3])), ob.fptr(arr(r[3:6])),
                                            ob.fptr(out))
        assert h == int(r[6])
        if h:
            n_hit += 1
            assert np.array_equal(bits(out), bits(r[7:11]))
    assert n_hit > 20


def test_fractal_spheres_generator():
    """ipt_amd.scenes.fractal_spheres() == the reference's generate_spheres
    driven as FractalSpheres' constructor does (ref_fractal_spheres.bin)."""
    from ipt_amd import scenes

    R = np.fromfile(GOLD / "ref_fractal_spheres.bin", dtype=np.float32)
    mine = np.array([v for c, r in scenes.fractal_spheres() for v in (*c, r)], np.float32)
    assert int(R[0]) == len(mine) // 4 and np.array_equal(bits(mine), bits(R[1:]))
