"""Test-side binding of oracle/libipt_oracle.so (the CPU restatement checker).

Test infrastructure only: loaded by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_SO = ROOT / "oracle" / "libipt_oracle.so"

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not ORACLE_SO.exists():
        build()
    from ipt_amd.capi import Counters, Params, Scene  # struct layouts only

    lib = C.CDLL(str(ORACLE_SO))
    lib.ipt_oracle_render_values.argtypes = [C.POINTER(Scene), C.POINTER(Params), C.c_void_p,
                                             C.c_void_p, C.c_int, C.POINTER(Counters)]
    lib.ipt_oracle_accumulate.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    f3 = C.POINTER(C.c_float)
    lib.ipt_oracle_box_plane.argtypes = [f3, f3, f3]
    lib.ipt_oracle_box_plane.restype = C.c_float
    lib.ipt_oracle_sphere.argtypes = [C.c_float, f3, f3]
    lib.ipt_oracle_sphere.restype = C.c_float
    lib.ipt_oracle_trace_box.argtypes = [f3, f3, f3]
    lib.ipt_oracle_light_trace.argtypes = [C.c_void_p, f3, f3, f3]
    lib.ipt_oracle_area_light.argtypes = [C.c_void_p, f3]
    lib.ipt_oracle_area_light.restype = None
    lib.ipt_oracle_rotate.argtypes = [f3, f3]
    lib.ipt_oracle_rotate.restype = None
    lib.ipt_oracle_camera.argtypes = [f3, f3, f3, f3]
    lib.ipt_oracle_camera.restype = None
    lib.ipt_oracle_mixture_weights.argtypes = [f3, C.c_int, f3]
    lib.ipt_oracle_mixture_weights.restype = None
    lib.ipt_oracle_cosine_value.argtypes = [C.c_float]
    lib.ipt_oracle_cosine_value.restype = C.c_float
    lib.ipt_oracle_randf.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.ipt_oracle_randf.restype = C.c_float
    _lib = lib
    return lib


def fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _threads(n: int) -> int:
    """0 = the host's cores, capped at 16 (a GPU box's CPU share)."""
    import os

    return n if n > 0 else max(1, min(16, os.cpu_count() or 1))


def render_values(scene_desc: dict, p, n_threads: int = 0, with_counters: bool = False):
    from ipt_amd.capi import Counters, make_scene

    lib = load()
    s, keep = make_scene(scene_desc)
    n = p.spp * p.width * p.height
    vals = np.zeros(n, np.float32)
    codes = np.zeros(n, np.uint8)
    cnt = Counters()
    rc = lib.ipt_oracle_render_values(C.byref(s), C.byref(p), vals.ctypes.data, codes.ctypes.data,
                                      _threads(n_threads), C.byref(cnt) if with_counters else None)
    assert rc == 0, rc
    shape = (p.spp, p.height, p.width)
    out = (vals.reshape(shape), codes.reshape(shape))
    return out + (cnt.as_dict(),) if with_counters else out


def render_rows_values(scene_desc: dict, p, row_step: int, row_phase: int, col_step: int = 1,
                       col_phase: int = 0, n_threads: int = 0):
    """Oracle values of the source pixels iy = row_phase (mod row_step),
    ix = col_phase (mod col_step) of every pass: array [spp][rows][cols] and
    the row and column indices."""
    from ipt_amd.capi import make_scene

    lib = load()
    lib.ipt_oracle_render_rows_values.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                                  C.c_int, C.c_void_p]
    s, keep = make_scene(scene_desc)
    rows = list(range(row_phase, p.height, row_step))
    cols = list(range(col_phase, p.width, col_step))
    vals = np.zeros(p.spp * len(rows) * len(cols), np.float32)
    rc = lib.ipt_oracle_render_rows_values(C.addressof(s), C.addressof(p), row_step, row_phase, col_step,
                                           col_phase, _threads(n_threads), vals.ctypes.data)
    assert rc == 0, rc
    return vals.reshape(p.spp, len(rows), len(cols)), rows, cols


def accumulate(values: np.ndarray, codes: np.ndarray, img: dict | None = None):
    """GridRenderPlane::addRay replay; returns dict(pixels, counters, sums, pixel_max)."""
    lib = load()
    spp, H, W = values.shape
    if img is None:
        img = {k: np.zeros(H * W, dt) for k, dt in
               (("pixels", np.float32), ("counters", np.uint32), ("sums", np.float32),
                ("pixel_max", np.float32))}
    v = np.ascontiguousarray(values, np.float32)
    c = np.ascontiguousarray(codes, np.uint8)
    rc = lib.ipt_oracle_accumulate(W, H, spp, v.ctypes.data, c.ctypes.data,
                                   img["pixels"].ctypes.data, img["counters"].ctypes.data,
                                   img["sums"].ctypes.data, img["pixel_max"].ctypes.data)
    assert rc == 0, rc
    return img


def setup_probes():
    """argtypes for the KAT probes added for the reference-pinning tests."""
    lib = load()
    f3 = C.POINTER(C.c_float)
    lib.ipt_oracle_light_sample_uv.argtypes = [C.c_void_p, C.c_float, C.c_float, f3]
    lib.ipt_oracle_light_sample_uv.restype = None
    lib.ipt_oracle_camera_ray.argtypes = [f3, f3, f3, C.c_float, C.c_float, f3]
    lib.ipt_oracle_camera_ray.restype = None
    lib.ipt_oracle_collection_trace.argtypes = [C.c_void_p, C.c_int, f3, f3, f3]
    lib.ipt_oracle_grid_addray.argtypes = [C.c_int, C.c_int, C.c_int, f3, f3,
                                           C.POINTER(C.c_uint32), f3]
    lib.ipt_oracle_grid_addray.restype = None
    lib.ipt_oracle_cosine_samples.argtypes = [C.c_uint64, f3, C.c_int, f3]
    lib.ipt_oracle_cosine_samples.restype = None
    lib.ipt_oracle_cosine_ddf_value.argtypes = [f3, f3]
    lib.ipt_oracle_cosine_ddf_value.restype = C.c_float
    return lib


def area_light_struct(P, x, y, power, typ):
    from ipt_amd.capi import AreaLight

    a = AreaLight()
    a.position[:] = [float(v) for v in P]
    a.x_axis[:] = [float(v) for v in x]
    a.y_axis[:] = [float(v) for v in y]
    a.power = float(power)
    a.type = int(typ)
    return a


EVENT_NAMES = ("traced_rays", "surface_hits", "light_hits", "expanded_nodes", "iterations", "light_samples",
               "skipped", "light_traces", "nonfinite_sums", "nonfinite_mults", "draws")


def render_events(scene_desc: dict, p, n_threads: int = 0):
    """Per-path values and drift codes [spp][H][W] and event counts
    [spp][H][W][len(EVENT_NAMES)] (ipt_oracle_render_events)."""
    from ipt_amd.capi import make_scene

    lib = load()
    lib.ipt_oracle_render_events.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                             C.c_void_p]
    assert lib.ipt_oracle_nev() == len(EVENT_NAMES)
    s, keep = make_scene(scene_desc)
    n = p.spp * p.width * p.height
    vals = np.zeros(n, np.float32)
    codes = np.zeros(n, np.uint8)
    ev = np.zeros((n, len(EVENT_NAMES)), np.uint32)
    rc = lib.ipt_oracle_render_events(C.addressof(s), C.addressof(p), _threads(n_threads), vals.ctypes.data,
                                      codes.ctypes.data, ev.ctypes.data)
    assert rc == 0, rc
    shape = (p.spp, p.height, p.width)
    return vals.reshape(shape), codes.reshape(shape), ev.reshape(shape + (len(EVENT_NAMES),))


def philox(ctr, key):
    """Philox4x32-10 block of the oracle's RNG (ipt_oracle_philox)."""
    lib = load()
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib.ipt_oracle_philox.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.ipt_oracle_philox.restype = None
    lib.ipt_oracle_philox(c.ctypes.data, k.ctypes.data, out.ctypes.data)
    return out
