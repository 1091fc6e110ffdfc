"""ipt_math.h (host build of the product library) against the host glibc libm
the reference calls, bit-for-bit.

Default run: every input the path tracer can produce for the RNG-driven
functions (all 2^24 draws u = k*2^-24 through CosineDdf::sample's chain) and a
strided sweep (1 float in 61) of every function's full domain.
IPT_EXHAUSTIVE=1: every float of every domain (~1.4e10 evaluations, ~2 min on
8 cores; last full run: 0 mismatches, recorded in DESIGN.md).
"""
import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from ipt_amd import capi

HERE = Path(__file__).resolve().parent
STRIDE = 1 if os.environ.get("IPT_EXHAUSTIVE") == "1" else 61
F = capi.MATH_FNS


@pytest.fixture(scope="module")
def libm(tmp_path_factory):
    so = tmp_path_factory.mktemp("libm") / "libm_ref.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-fno-builtin", "-o",
                    str(so), str(HERE / "native" / "libm_ref.c"), "-lm", "-lpthread"], check=True)
    lib = C.CDLL(str(so))
    lib.libm_eval.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_int]
    return lib


def ref(libm, fn, x):
    out = np.empty_like(x)
    libm.libm_eval(fn, x.ctypes.data, out.ctypes.data, x.size, min(16, os.cpu_count() or 1))
    return out


def compare(libm, fn, x):
    a = capi.math_host(fn, x)
    b = ref(libm, fn, x)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), (fn, x[~same][:5], a[~same][:5], b[~same][:5])


def sweep(libm, fn, lo_bits, hi_bits):
    chunk = 1 << 24
    for s in range(lo_bits, hi_bits, chunk * STRIDE):
        e = min(hi_bits, s + chunk * STRIDE)
        x = np.arange(s, e, STRIDE, dtype=np.uint64).astype(np.uint32).view(np.float32)
        compare(libm, fn, x)


U = np.arange(1 << 24, dtype=np.float32) * np.float32(2.0 ** -24)  # every RNG draw


def test_cosine_sample_chain_reachable(libm):
    """cos_alpha = sqrtf(u1); alpha = acosf(cos_alpha); r = sinf(alpha);
    phi = (float)(2*M_PI*u2); sincosf(phi)  — ddf.cpp:223-231, every u."""
    compare(libm, F["sqrtf"], U)
    ca = capi.math_host(F["sqrtf"], U)
    compare(libm, F["acosf"], ca)
    alpha = capi.math_host(F["acosf"], ca)
    compare(libm, F["sinf"], alpha)
    compare(libm, F["two_pi_times"], U)
    phi = capi.math_host(F["two_pi_times"], U)
    for fn in ("sinf", "cosf", "sincosf_sin", "sincosf_cos"):
        compare(libm, F[fn], phi)


def test_acosf_domain(libm):
    sweep(libm, F["acosf"], 0, 0x3f800001)
    sweep(libm, F["acosf"], 0x80000000, 0xbf800001)
    compare(libm, F["acosf"], np.array([2.0, -2.0, np.inf, np.nan], np.float32))


def test_sin_cos_domain(libm):
    for fn in ("sinf", "cosf", "sincosf_sin", "sincosf_cos"):
        sweep(libm, F[fn], 0, 0x42f00000)  # |x| < 120: every angle the path tracer makes
        sweep(libm, F[fn], 0x80000000, 0xc2f00000)
    for fn in ("sinf", "cosf"):  # large-argument reduction
        sweep(libm, F[fn], 0x42f00000, 0x7f800000)


def test_acos_double_rounded_to_float(libm):
    """(float)acos((double)cosinus) of RotateDdf (ddf_detail.h:82)."""
    sweep(libm, F["acos_f64_f32"], 0, 0x3f800001)
    sweep(libm, F["acos_f64_f32"], 0x80000000, 0xbf800001)


def test_mixed_precision_helpers(libm):
    sweep(libm, F["div_pi"], 0, 0x40000001)  # CosineDdf::value z/M_PI in f64
    sweep(libm, F["sqrtf"], 0, 0x7f800000)


def test_frame_angle_and_range_free_root(libm):
    """Host build of the RotateDdf angle's (sin, cos) (the frame table's
    entries, ipt_path.h frame_angle_sc) against glibc, and the range-free root
    probe against sqrtf (its fast sequence is proven on the GPU)."""
    for fn in ("frame_angle_sin", "frame_angle_cos"):
        sweep(libm, F[fn], 0, 0x3f800001)
        sweep(libm, F[fn], 0x80000000, 0xbf800001)
    sweep(libm, F["sqrt_inrange"], 0, 0x7f800000)


def test_two_pi_times_from_24_bit_draw():
    """two_pi_times_u24(g) (ipt_math.h) == two_pi_times(u01(g << 8)) for every
    24-bit g: (float)(2pi * (g 2^-24)) in double equals (float)((2pi 2^-24) *
    g), the same real product with the constant scaled by a power of two."""
    import struct
    two_pi = struct.unpack("<d", struct.pack("<Q", 0x401921FB54442D18))[0]
    scaled = struct.unpack("<d", struct.pack("<Q", 0x3E9921FB54442D18))[0]
    assert scaled == two_pi * 2.0 ** -24
    g = np.arange(1 << 24, dtype=np.uint64)
    u = g.astype(np.float32) * np.float32(2.0 ** -24)
    a = (two_pi * u.astype(np.float64)).astype(np.float32)
    b = (scaled * g.astype(np.float64)).astype(np.float32)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
