"""The C++ host layer (ipt_amd/host/: reference-named scene classes,
sample scenes, flattening to the C-ABI, Gui-style PNG output) without a GPU:
its scenes must be bit-identical to the Python builders the parity tests use
(ipt_amd/scenes.py), and its 8-bit output must follow gui.cpp/CImg's
normalisation. The GPU half (ipt_render CLI vs the oracle image) is
tests/test_gpu_parity.py::test_cli_render_matches_oracle."""
import ctypes as C
import json
import struct
import subprocess
import zlib
from pathlib import Path

import numpy as np
import pytest

import __graft_entry__ as ge
from ipt_amd import capi, scenes

HERE = Path(__file__).resolve().parent


@pytest.fixture(scope="module")
def dump(tmp_path_factory):
    ge.build_lib()
    ge.build_host()
    exe = tmp_path_factory.mktemp("host") / "host_scene_dump"
    subprocess.run(["g++", *ge.GXX_FLAGS, "-o", str(exe), str(HERE / "native" / "host_scene_dump.cpp"),
                    f"-I{ge.HOST}", f"-L{ge.LIB.parent}", "-lipt_host", "-lipt_hip",
                    f"-Wl,-rpath,{ge.LIB.parent}", "-Wl,-rpath-link,/opt/rocm/lib"], check=True)
    return exe


def _b(x):
    return int(np.float32(x).view(np.uint32))


def _py_flat(desc):
    cam = desc["camera"]
    return {
        "geometry_kind": desc["geometry_kind"],
        "camera": [[_b(v) for v in cam[k]] for k in ("position", "direction", "right", "up")],
        "lights": [[[_b(v) for v in L["position"]], [_b(v) for v in L["x_axis"]],
                    [_b(v) for v in L["y_axis"]], _b(L["power"]), L["type"]] for L in desc["lights"]],
        "spheres": [[[_b(v) for v in c], _b(r)] for c, r in desc.get("spheres", [])],
    }


@pytest.mark.parametrize("name,desc_fn", [
    ("box", scenes.make_scene_box),
    ("box_lights:4", lambda: scenes.make_scene_box_lights(4)),
    ("box_lights:16", lambda: scenes.make_scene_box_lights(16)),
    ("spheres:300:1", lambda: scenes.make_scene_spheres(300, 1)),
    ("random_lights:17:7", lambda: scenes.make_scene_random_lights(17, 7)),
    ("square_lit_by_square", scenes.make_scene_square_lit_by_square),
    ("lit_corner", scenes.make_scene_lit_corner),
    ("fractal", scenes.make_scene_fractal),
    ("smallpt", scenes.make_scene_smallpt),
])
def test_cpp_scenes_match_python(dump, name, desc_fn):
    out = subprocess.run([str(dump), "scene", name], check=True, capture_output=True, text=True).stdout
    assert json.loads(out) == _py_flat(desc_fn())


@pytest.mark.parametrize("name", ["open_spheres", "nonexistent"])
def test_unknown_scenes_fail_loudly(dump, name):
    out = subprocess.run([str(dump), "scene-error", name], check=True, capture_output=True, text=True).stdout
    assert int(out) == capi.IPT_E_INVALID


def _read_png_gray8(path):
    data = Path(path).read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body)
        chunks.setdefault(typ, b"")
        chunks[typ] += body
        pos += 12 + n
    w, h, depth, ctype = struct.unpack(">IIBB", chunks[b"IHDR"][:10])
    assert (depth, ctype) == (8, 0)
    raw = np.frombuffer(zlib.decompress(chunks[b"IDAT"]), np.uint8).reshape(h, w + 1)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:]


def test_gray8_png_follows_gui_save(dump, tmp_path):
    """gui.cpp:11-16 + 133-135: (v/max)^(1/2.2) cut [0,1], CImg normalize(0,255),
    (unsigned char) cast; restated here in numpy float32."""
    rng = np.random.default_rng(3)
    W, H = 37, 23
    px = (rng.random(W * H, dtype=np.float32) * np.float32(3.0)).astype(np.float32)
    px[5] = 0.0
    px.tofile(tmp_path / "p.f32")
    subprocess.run([str(dump), "gray8", str(W), str(H), str(tmp_path / "p.f32"), str(tmp_path / "o.png")],
                   check=True)
    got = _read_png_gray8(tmp_path / "o.png")
    v = px / px.max()
    v = np.power(v, np.float32(1.0) / np.float32(2.2)).astype(np.float32)
    v = np.clip(v, np.float32(0), np.float32(1))
    m, M = v.min(), v.max()
    v = ((v - m) / (M - m) * np.float32(255.0)).astype(np.float32)
    assert np.array_equal(got.reshape(-1), v.astype(np.uint8))


def test_pgm_follows_main_cpp(dump, tmp_path):
    """main.cpp:225-235,297-309: n_val with contrast 500, gamma 0.6, float
    logf/powf (the reference's `using namespace std` overloads), ASCII P2."""
    libm = C.CDLL("libm.so.6")
    libm.logf.restype = libm.powf.restype = C.c_float
    libm.logf.argtypes = [C.c_float]
    libm.powf.argtypes = [C.c_float, C.c_float]
    rng = np.random.default_rng(9)
    W, H = 13, 7
    px = (rng.random(W * H, dtype=np.float32) * np.float32(2.0)).astype(np.float32)
    px.tofile(tmp_path / "p.f32")
    mx = float(px.max())
    subprocess.run([str(dump), "pgm", str(W), str(H), str(tmp_path / "p.f32"), repr(mx), str(tmp_path / "o.pgm")],
                   check=True)
    txt = (tmp_path / "o.pgm").read_text().split()
    assert txt[:4] == ["P2", str(W), str(H), "255"]
    contrast, gamma = np.float32(500.0), np.float32(0.6)
    exp = []
    for v in px:
        adj = np.float32(np.float32(v * contrast) / np.float32(mx))
        adj = min(adj, contrast)
        adj = max(adj, np.float32(1.0))
        fn = np.float32(np.float32(libm.logf(adj)) / np.float32(libm.logf(contrast)))
        fn = np.float32(libm.powf(fn, gamma))
        n = int(np.float32(256) * fn)
        exp.append(str(min(255, max(0, n))))
    assert txt[4:] == exp


def test_cli_requires_gpu():
    """No CPU fallback: without a gfx950 device the CLI exits non-zero."""
    ge.build_host()
    r = subprocess.run([str(ge.HOST_BIN), "--width", "4", "--height", "4", "--out", ""],
                       capture_output=True, text=True)
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present: covered by test_gpu_parity.py::test_cli_render_matches_oracle")
    assert r.returncode == 1 and "no HIP device" in r.stderr
