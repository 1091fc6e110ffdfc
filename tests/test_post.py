"""Image post-process: GridRenderPlane::smooth /
computeSmoothedMax and Gui's glare, on the GPU (ipt_amd/csrc/ipt_post.hip),
bit-exact. CPU: the oracle restatement against the reference's own compiled
GridRenderPlane (tests/golden/ref_smooth.bin from oracle/ref_kat.cpp), against
the reference's own gui.cpp glare() (tests/golden/ref_glare.bin from
oracle/ref_glare.cpp) and the hypot identity the glare kernel uses. GPU:
kernels against both golden files and the oracle."""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi

HERE = Path(__file__).resolve().parent
GOLD = HERE / "golden" / "ref_smooth.bin"
GOLD_GLARE = HERE / "golden" / "ref_glare.bin"  # reference gui.cpp glare(), oracle/ref_glare.cpp


def _lib():
    lib = ob.load()
    lib.ipt_oracle_smooth.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int,
                                      C.POINTER(C.c_float)]
    lib.ipt_oracle_smooth.restype = C.c_int
    lib.ipt_oracle_glare.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_float]
    return lib


def oracle_smooth(px, W, H, side, in_place):
    p = np.ascontiguousarray(px, np.float32).copy()
    mx = C.c_float()
    assert _lib().ipt_oracle_smooth(p.ctypes.data, W, H, side, 1 if in_place else 0, C.byref(mx)) == 0
    return p, mx.value


def oracle_glare(img, W, H, cutoff):
    src = np.ascontiguousarray(img, np.float32)
    out = np.empty_like(src)
    _lib().ipt_oracle_glare(src.ctypes.data, out.ctypes.data, W, H, C.c_float(cutoff))
    return out


def _bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def _cases():
    d = np.fromfile(GOLD, np.float32)
    n, pos, out = int(d[0]), 1, []
    for _ in range(n):
        W, H, side = (int(v) for v in d[pos:pos + 3])
        pos += 3
        inp = d[pos:pos + W * H]; pos += W * H
        sm = d[pos:pos + W * H]; pos += W * H
        out.append((W, H, side, inp, sm, d[pos], d[pos + 1]))
        pos += 2
    return out


def _glare_cases():
    d = np.fromfile(GOLD_GLARE, np.float32)
    n, pos, out = int(d[0]), 1, []
    for _ in range(n):
        W, H, cutoff = int(d[pos]), int(d[pos + 1]), d[pos + 2]
        pos += 3
        inp = d[pos:pos + W * H]; pos += W * H
        ref = d[pos:pos + W * H]; pos += W * H
        out.append((W, H, cutoff, inp, ref))
    return out


def test_oracle_glare_matches_reference(oracle):
    """The oracle's glare against the reference's own gui.cpp glare() (9 cases:
    single hot pixel at the GUI cutoff 1.01, random hot fractions, a pixel at /
    just above the cutoff, negative pixels, +inf and NaN sources, 1x1, 1xN)."""
    cases = _glare_cases()
    assert len(cases) == 9
    assert any(np.isnan(r).all() for *_, r in cases)
    for W, H, cutoff, inp, ref in cases:
        got = oracle_glare(inp, W, H, float(cutoff))
        assert np.array_equal(_bits(got), _bits(ref)), (W, H, float(cutoff))


def test_oracle_smooth_matches_reference(oracle):
    cases = _cases()
    assert len(cases) == 6
    for W, H, side, inp, sm, mx_s, mx_c in cases:
        got, mx = oracle_smooth(inp, W, H, side, True)
        assert np.array_equal(_bits(got), _bits(sm)), (W, H, side)
        assert _bits(mx) == _bits(mx_s)
        same, mx2 = oracle_smooth(inp, W, H, side, False)
        assert np.array_equal(_bits(same), _bits(inp)) and _bits(mx2) == _bits(mx_c)


def test_hypot_identity(tmp_path):
    exe = tmp_path / "hypot_check"
    subprocess.run(["gcc", "-O2", "-fno-builtin", "-o", str(exe), str(HERE / "native" / "hypot_check.c"), "-lm"],
                   check=True)
    assert subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.strip() == "0"


def test_oracle_glare_basics(oracle):
    """A single bright pixel: halo falls off as C/(0.25+r)^2 and the result is
    cut to [0, cutoff]."""
    W, H = 9, 7
    img = np.zeros(W * H, np.float32)
    img[3 * W + 4] = 10.0
    out = oracle_glare(img, W, H, 1.0).reshape(H, W)
    assert out[3, 4] == np.float32(1.0)          # cut at the cutoff
    assert out[3, 5] > out[3, 6] > out[3, 8] > 0  # monotone fall-off
    assert np.array_equal(out, out[:, ::-1][:, ::-1])


@pytest.mark.gpu
def test_gpu_smooth_matches_reference_and_oracle(gpu_ctx, oracle):
    for W, H, side, inp, sm, mx_s, mx_c in _cases():
        got, mx = gpu_ctx.smooth(inp, W, H, side, True)
        assert np.array_equal(_bits(got), _bits(sm)) and _bits(mx) == _bits(mx_s), (W, H, side)
        same, mx2 = gpu_ctx.smooth(inp, W, H, side, False)
        assert np.array_equal(_bits(same), _bits(inp)) and _bits(mx2) == _bits(mx_c)
    rng = np.random.default_rng(11)
    for W, H, side in ((640, 640, 2), (640, 640, 5), (1000, 37, 16), (300, 200, 3)):
        px = (rng.random(W * H, dtype=np.float32) * 3).astype(np.float32)
        px[rng.random(W * H) < 0.05] = 0.0
        px[7] = np.nan
        ref, rmx = oracle_smooth(px, W, H, side, True)
        got, mx = gpu_ctx.smooth(px, W, H, side, True)
        assert np.array_equal(_bits(got), _bits(ref)) and _bits(mx) == _bits(rmx), (W, H, side)
    with pytest.raises(capi.IptError):
        gpu_ctx.smooth(px, W, H, 1, True)


@pytest.mark.gpu
def test_gpu_glare_matches_reference(gpu_ctx):
    for W, H, cutoff, inp, ref in _glare_cases():
        got = gpu_ctx.glare(inp, W, H, float(cutoff))
        assert np.array_equal(_bits(got), _bits(ref)), (W, H, float(cutoff))


@pytest.mark.gpu
def test_gpu_glare_matches_oracle(gpu_ctx, oracle):
    rng = np.random.default_rng(5)
    for W, H, frac in ((64, 48, 0.03), (97, 33, 0.2)):
        img = (rng.random(W * H, dtype=np.float32) * np.float32(0.5)).astype(np.float32)
        hot = rng.random(W * H) < frac
        img[hot] = (rng.random(int(hot.sum()), dtype=np.float32) * 40 + 1).astype(np.float32)
        cutoff = np.float32(1.0)
        ref = oracle_glare(img, W, H, cutoff)
        got = gpu_ctx.glare(img, W, H, float(cutoff))
        assert np.array_equal(_bits(got), _bits(ref)), int((_bits(got) != _bits(ref)).sum())
