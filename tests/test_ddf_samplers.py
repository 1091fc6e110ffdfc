"""the path's DDF samplers, validated on the device.

* Bit-exact: the device sampler and value functions (ipt_ddf_sample /
  ipt_ddf_value, the same code the path kernel runs) against the oracle
  restatement, on shared uniforms (including 0 and the largest draw).
* Statistically: the reference's chi^2 harness (check_ddf.cpp:114-203,
  restated in tests/ddf_check.py) on device samples for RotateDdf(CosineDdf)
  (test_ddf.cpp:229), DdfFromLight of test_lighting.cpp:77-89's area light at
  its origins (0,0,0.6), (0.5,0,0.5) and twice those, and the UnionDdf
  mixture of sample_scenes[0] at wall and sphere points.
The CPU half runs the same chi^2 checks on the oracle's samplers."""
import ctypes as C

import numpy as np
import pytest

import oracle_binding as ob
from ddf_check import check_ddf
from ipt_amd import capi, scenes

N = 100000  # check_ddf.cpp:11


def _bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def _lib():
    lib = ob.load()
    for f in (lib.ipt_oracle_ddf_sample, lib.ipt_oracle_ddf_value):
        f.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        f.restype = C.c_int
    return lib


def light_scene():
    # test_lighting.cpp:77: AreaLight(vec3(-0.5,-0.5,0), vec3(1,0,0), vec3(0,1,0), 1.0f)
    L = {"position": [-0.5, -0.5, 0.0], "x_axis": [1.0, 0.0, 0.0], "y_axis": [0.0, 1.0, 0.0], "power": 1.0,
         "type": capi.IPT_LIGHT_AREA_DIAMOND}
    return {"geometry_kind": capi.IPT_GEOM_SPHERE_IN_BOX, "lights": [L], "spheres": [],
            "camera": scenes.box_camera()}


def _uniforms(n, seed):
    u = (np.random.default_rng(seed).integers(0, 1 << 24, size=(n, 3)) * 2.0 ** -24).astype(np.float32)
    u[:8] = [[0, 0, 0], [0, 0.5, 0.5], [0.5, 0.999999940, 0.999999940], [0.999999940, 0, 0.25],
             [0.25, 0.999999940, 0], [0.75, 0.3, 0.0], [0.5, 0.0, 0.999999940], [0.49999997, 0.2, 0.7]]
    return u


def oracle_sample(desc, kind, params, u):
    sc, keep = capi.make_scene(desc)
    pr = np.pad(np.asarray(params, np.float32), (0, 8))[:8]
    out = np.empty((len(u), 3), np.float32)
    _lib().ipt_oracle_ddf_sample(C.addressof(sc), kind, pr.ctypes.data, np.ascontiguousarray(u).ctypes.data,
                                 len(u), out.ctypes.data)
    return out


def oracle_value(desc, kind, params, dirs):
    sc, keep = capi.make_scene(desc)
    pr = np.pad(np.asarray(params, np.float32), (0, 8))[:8]
    dd = np.ascontiguousarray(dirs, np.float32)
    out = np.empty(len(dd), np.float32)
    _lib().ipt_oracle_ddf_value(C.addressof(sc), kind, pr.ctypes.data, dd.ctypes.data, len(dd), out.ctypes.data)
    return out


def _grid(kind, params=None):
    """check_ddf's 20x20 buckets with centre values for the z-up cosine DDF
    (test_ddf.cpp:229); for the tilted cosine (whose horizon cuts bucket
    interiors), light and mixture DDFs the 40x40 variant the
    reference uses for unions (test_ddf.cpp:265), with bucket-integrated
    expectations (a light spans about one 20x20 bucket, and at ~40 DoF the
    [0.70, 1.35] x DoF window rejects a correct sampler ~6% of the time)."""
    if kind == capi.IPT_DDF_COSINE and list(params) == [0, 0, 1]:
        return dict(size_alpha=20, size_phi=20, sub=1)  # exactly test_ddf.cpp:229's check
    return dict(size_alpha=40, size_phi=40, sub=8)


# (scene, kind, params, strict integral): the chi^2 cases
NZ = float(np.float32(1.0) / np.sqrt(np.float32(3.0)))
CASES = {
    "cosine_z": (scenes.make_scene_box, capi.IPT_DDF_COSINE, [0, 0, 1], True),
    "cosine_tilted": (scenes.make_scene_box, capi.IPT_DDF_COSINE, [NZ, -NZ, NZ], True),
    "light_a": (light_scene, capi.IPT_DDF_LIGHT, [0, 0, 0.6, 0], False),
    "light_a2": (light_scene, capi.IPT_DDF_LIGHT, [0, 0, 1.2, 0], False),
    "light_b": (light_scene, capi.IPT_DDF_LIGHT, [0.5, 0, 0.5, 0], False),
    "mixture_wall": (scenes.make_scene_box, capi.IPT_DDF_MIXTURE, [0.2, -0.4, -1.0, 0, 0, 1], False),
    "mixture_sphere": (scenes.make_scene_box, capi.IPT_DDF_MIXTURE, [0.0, -0.5, 0.0, 0, -1, 0], False),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_chi2_oracle_samplers(oracle, case):
    make, kind, params, strict = CASES[case]
    desc = make()
    s = oracle_sample(desc, kind, params, _uniforms(3 * N, 3))
    ok, info = check_ddf(s, lambda d: oracle_value(desc, kind, params, d), N=N, strict_integral=strict,
                         **_grid(kind, params))
    assert ok, (case, info)


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_device_samplers_bit_exact_and_chi2(gpu_ctx, oracle, case):
    make, kind, params, strict = CASES[case]
    desc = make()
    gpu_ctx.upload_scene(desc)
    u = _uniforms(3 * N, 11)
    d = gpu_ctx.ddf_sample(kind, params, u)
    o = oracle_sample(desc, kind, params, u)
    assert np.array_equal(_bits(d), _bits(o)), int((_bits(d) != _bits(o)).any(1).sum())
    probe = np.concatenate([d[:20000], np.random.default_rng(1).normal(size=(20000, 3)).astype(np.float32)])
    probe[20000:] /= np.linalg.norm(probe[20000:], axis=1, keepdims=True)
    dv, ov = gpu_ctx.ddf_value(kind, params, probe), oracle_value(desc, kind, params, probe)
    assert np.array_equal(_bits(dv), _bits(ov))
    ok, info = check_ddf(d, lambda x: gpu_ctx.ddf_value(kind, params, x), N=N, strict_integral=strict,
                         **_grid(kind, params))
    assert ok, (case, info)


@pytest.mark.gpu
@pytest.mark.parametrize("to", [[0, 0, 1], [NZ, -NZ, NZ]])
def test_cosine_table_sampler_exhaustive(gpu_ctx, oracle, to):
    """The path kernel's CosineDdf tables (every one of the 2^24 values each of
    u1 and u2 can take, paired by an odd-multiplier permutation) against the
    oracle's glibc CosineDdf::sample (ddf.cpp:223-231): bit-identical. With
    to = +z the frame is the identity, so the table entries themselves are
    compared."""
    gpu_ctx.upload_scene(scenes.make_scene_box())
    n = 1 << 24 if to == [0, 0, 1] else 1 << 20
    i1 = np.arange(n, dtype=np.uint64) * ((1 << 24) // n)
    i2 = (i1 * 7919 + 12345) % (1 << 24)
    u = np.zeros((n, 3), np.float32)
    u[:, 1] = i1.astype(np.float32) * np.float32(2.0 ** -24)
    u[:, 2] = i2.astype(np.float32) * np.float32(2.0 ** -24)
    d = gpu_ctx.ddf_sample(capi.IPT_DDF_COSINE_TABLE, to, u)
    o = oracle_sample(scenes.make_scene_box(), capi.IPT_DDF_COSINE, to, u)
    bad = (_bits(d) != _bits(o)).any(1)
    assert not bad.any(), (int(bad.sum()), u[bad][:3], d[bad][:3], o[bad][:3])


@pytest.mark.gpu
def test_cosine_table_sampler_rejects_off_grid(gpu_ctx):
    gpu_ctx.upload_scene(scenes.make_scene_box())
    with pytest.raises(capi.IptError):
        gpu_ctx.ddf_sample(capi.IPT_DDF_COSINE_TABLE, [0, 0, 1], np.array([[0, 0.1, 0.5]], np.float32))
