"""The reference's own unit tests, restated against the oracle and the
product's host build of the portable math.

test_ddf.cpp:16-20 (eq, EPS), :205-216 (CosineDdf values), :225-229 (chi^2 of
CosineDdf via check_ddf.cpp:114-203); test_lighting.cpp:130-144 (AreaLight).
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi

EPS = 1e-6  # test_ddf.cpp:16


def eq(a, b):  # test_ddf.cpp:18-20
    return abs(a - b) < EPS


@pytest.fixture(scope="module")
def lib(oracle):
    return ob.setup_probes()


def _cos_value_product(z):
    # CosineDdf::value in the product = z < 0 ? 0 : (float)(z/M_PI) (ipt_path.h)
    if z < 0:
        return 0.0
    return float(capi.math_host(capi.MATH_FNS["div_pi"], np.array([z], np.float32))[0])


def test_cosine_ddf_values(lib):
    # CosineDdf cd; cd.value(0,0,1) == M_1_PI; cd.value(1,0,EPS/10) == 0;
    # cd.value(normalize(1,1,-1)) == 0        (test_ddf.cpp:213-215)
    for f in (lib.ipt_oracle_cosine_value, _cos_value_product):
        assert eq(f(1.0), 1.0 / math.pi)
        assert eq(f(np.float32(EPS / 10.0)), 0.0)
        assert f(np.float32(-1.0 / math.sqrt(3.0))) == 0.0
    to = np.array([0, 0, 1], np.float32)
    for d, want in (((0, 0, 1), 1.0 / math.pi), ((1, 0, EPS / 10), 0.0)):
        v = lib.ipt_oracle_cosine_ddf_value(ob.fptr(to), ob.fptr(np.array(d, np.float32)))
        assert eq(v, want)


def test_area_light_basic(lib):
    # AreaLight diag(vec3(1,1,1), vec3(-1,-1,-1), vec3(0,-1,0), 4)   test_lighting.cpp:131-143
    L = ob.area_light_struct((1, 1, 1), (-1, -1, -1), (0, -1, 0), 4.0, 0)
    asp = np.zeros(2, np.float32)
    lib.ipt_oracle_area_light(C.byref(L), ob.fptr(asp))
    sin_alpha = np.sqrt(np.float32(2.0) / np.float32(3.0), dtype=np.float32)
    diag_length = np.sqrt(np.float32(3.0), dtype=np.float32)
    assert abs(asp[0] - diag_length * sin_alpha) <= 1e-6
    pos = np.zeros(3, np.float32)
    h = lib.ipt_oracle_light_trace(C.byref(L), ob.fptr(np.array([0, 0, 0.1], np.float32)),
                                   ob.fptr(np.array([1.1, 0, 0], np.float32)), ob.fptr(pos))
    assert h == 1
    assert abs(asp[1] - 4.0 / asp[0]) <= 1e-6


def _check_ddf(samples, value_fn, size_alpha=20, size_phi=20, strict_integral=True):
    """check_ddf.cpp:114-203 restated (N = number of samples)."""
    N = len(samples)
    rng = np.random.default_rng(7)
    # mc_integral_and_max: uniform sphere samples (SphericalDdf, value 1/4pi)
    u1 = rng.random(100000) * 2 - 1
    u2 = rng.random(100000)
    r = np.sqrt(1 - u1 * u1)
    sph = np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2), u1], 1)
    vals = np.array([value_fn(v) for v in sph])
    ddf_integral = float(np.mean(vals / (0.25 / np.pi)))
    buckets = np.zeros((size_alpha, size_phi))
    total_tries = 0
    for v in samples:
        total_tries += 1
        alpha = math.acos(max(-1.0, min(1.0, float(v[2]))))
        rr = math.hypot(float(v[0]), float(v[1]))
        phi = math.asin(max(-1.0, min(1.0, v[1] / rr))) if v[0] >= 0 else math.pi - math.asin(
            max(-1.0, min(1.0, v[1] / rr)))
        if phi < 0:
            phi += 2 * math.pi
        if phi >= 2 * math.pi:
            phi -= 2 * math.pi
        buckets[min(int(alpha / math.pi * size_alpha), size_alpha - 1),
                min(int(phi / 2 / math.pi * size_phi), size_phi - 1)] += 1

    def a_i(i):
        return (i + 0.5) / size_alpha * math.pi

    def p_j(j):
        return (j + 0.5) / size_phi * 2 * math.pi

    def polar(a, p):
        s = math.sin(a)
        return np.array([s * math.cos(p), s * math.sin(p), math.cos(a)], np.float32)

    def area(i):
        return (2 * math.pi * math.sin(a_i(i)) / size_phi) * (math.pi / size_alpha)

    def zero_neighbour(i, j):
        for ii, jj in ((i + 1, j), (i - 1, j), (i, (j + 1) % size_phi), (i, (j - 1) % size_phi)):
            if 0 <= ii < size_alpha and (buckets[ii, jj] == 0 or value_fn(polar(a_i(ii), p_j(jj))) == 0):
                return True
        return False

    chi2 = 0.0
    skip = 0
    for i in range(size_alpha):
        for j in range(size_phi):
            theor = value_fn(polar(a_i(i), p_j(j))) * area(i) * N / ddf_integral
            exper = buckets[i, j]
            if theor > 2 and exper >= 2 and not zero_neighbour(i, j):
                chi2 += (exper - theor) ** 2 / theor
            else:
                skip += 1
    dof = size_alpha * size_phi - skip
    lo, hi = 70 * dof / 100.0, 135 * dof / 100.0
    success = N / total_tries
    ok = (lo < chi2 < hi and 0.95 < success / ddf_integral < 1.05
          and (not strict_integral or 0.95 < ddf_integral < 1.05))
    return ok, chi2, dof, ddf_integral


@pytest.mark.parametrize("seed", [1, 2])
def test_chi2_cosine_ddf(lib, seed):
    """CHECK(check_ddf(CosineDdf()))  (test_ddf.cpp:229) on the restated sampler,
    which the GPU reproduces bit-for-bit (test_gpu_parity.py)."""
    N = 100000  # check_ddf.cpp:11
    to = np.array([0, 0, 1], np.float32)
    out = np.zeros(3 * N, np.float32)
    lib.ipt_oracle_cosine_samples(seed, ob.fptr(to), N, ob.fptr(out))
    samples = out.reshape(N, 3)

    def value(v):
        return max(float(v[2]), 0.0) / math.pi

    ok, chi2, dof, integ = _check_ddf(samples, value)
    assert ok, (chi2, dof, integ)
