"""ctypes binding of include/ipt_capi.h (libipt_hip.so).

This is the Python-side view of the drop-in boundary: the same entry points a
cgo / JNI / ctypes caller of the reference would bind.
Only plain pointers cross it. The library has no CPU fallback: every rendering
call needs a gfx950 device and fails loudly (IptError) otherwise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "lib" / "libipt_hip.so"

IPT_OK = 0
IPT_E_INVALID = -1
IPT_DDF_COSINE, IPT_DDF_LIGHT, IPT_DDF_MIXTURE, IPT_DDF_COSINE_TABLE = 0, 1, 2, 3
IPT_E_DEVICE = -2
IPT_E_UNSUPPORTED = -3
IPT_E_NOSCENE = -4
IPT_E_OOM = -5

IPT_GEOM_SPHERE_IN_BOX = 0
IPT_GEOM_SPHERES_IN_BOX = 1
IPT_GEOM_FLOOR = 2
IPT_GEOM_CORNER = 3
IPT_GEOM_SPHERES = 4
IPT_GEOM_SMALLPT = 5
IPT_LIGHT_AREA_DIAMOND = 0
IPT_LIGHT_AREA_TRIANGLE = 1
IPT_LIGHT_SPHERE, IPT_LIGHT_POINT, IPT_LIGHT_OUTER_SPHERE = 2, 3, 4
IPT_FLAG_COUNTERS = 1

F3 = C.c_float * 3


class AreaLight(C.Structure):
    _fields_ = [("position", F3), ("x_axis", F3), ("y_axis", F3), ("power", C.c_float),
                ("type", C.c_int32)]


class Camera(C.Structure):
    _fields_ = [("position", F3), ("direction", F3), ("right", F3), ("up", F3)]


class Sphere(C.Structure):
    _fields_ = [("center", F3), ("radius", C.c_float)]


class Scene(C.Structure):
    _fields_ = [("geometry_kind", C.c_int32), ("n_lights", C.c_int32),
                ("lights", C.POINTER(AreaLight)), ("n_spheres", C.c_int32),
                ("spheres", C.POINTER(Sphere)), ("camera", Camera)]


class Params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32),
                ("spp_offset", C.c_int32), ("n_rays", C.c_int32), ("depth_max", C.c_int32),
                ("seed", C.c_uint64), ("tile_rows", C.c_int32), ("n_shards", C.c_int32),
                ("shard_id", C.c_int32), ("flags", C.c_uint32)]


class Image(C.Structure):
    _fields_ = [("pixels", C.c_void_p), ("counters", C.c_void_p), ("sums", C.c_void_p),
                ("pixel_max", C.c_void_p)]


ABI_VERSION = 5  # include/ipt_capi.h IPT_ABI_VERSION
ABI_LAYOUT_COMPATIBLE = (3, 4, 5)  # versions with this binding's struct layouts (IPT_ABI_COMPAT only)

COUNTER_NAMES = ("paths", "traced_rays", "surface_hits", "light_hits", "expanded_nodes",
                 "iterations", "light_samples", "skipped", "sphere_frames", "light_traces",
                 "drifted", "bvh_nodes", "sphere_tests", "light_nodes", "light_tests")


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in COUNTER_NAMES]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in COUNTER_NAMES}


EXPORTED_SYMBOLS = (
    "ipt_abi_version", "ipt_last_error", "ipt_create", "ipt_destroy", "ipt_upload_scene",
    "ipt_render", "ipt_render_device", "ipt_render_device_async", "ipt_render_wait", "ipt_render_values",
    "ipt_get_counters",
    "ipt_reset_counters", "ipt_last_kernel_ms", "ipt_math_host", "ipt_math_device",
    "ipt_shard_plan", "ipt_get_profile", "ipt_math_selfcheck", "ipt_smooth", "ipt_glare", "ipt_ddf_sample", "ipt_ddf_value",
    "ipt_philox", "ipt_transfer_bytes",
)

# path-kernel phases of the IPT_PROF profile (ipt_kernels.hip IPT_PHASE ids)
PROFILE_PHASES = ("step", "pop", "new_path", "iteration", "philox", "frame_worker",
                  "walk_cell", "light_sample", "trace", "geometry", "push", "wg_step")
# step segments of the IPT_STAMP diagnostic build (IPT_STAMP_AT ids)
STAMP_SEGMENTS = ("loop_top", "refill", "pop_early", "pre_prologue", "prologue_philox_frame", "exit_test",
                  "pop", "frame_prefetch", "new_path_direction", "lights", "mixture_geometry", "resolve_push")

_lib = None


class IptError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ipt error {code}: {msg}")
        self.code = code


def load(path: str | os.PathLike | None = None):
    """Load libipt_hip.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("IPT_LIB_PATH", LIB_PATH))
    if not p.exists():
        raise IptError(IPT_E_DEVICE, f"{p} is not built; run __graft_entry__.build()")
    lib = C.CDLL(str(p))
    lib.ipt_abi_version.restype = C.c_int
    # (IPT_ABI_COMPAT=1: A/B tooling loading an older variant library; only
    # the versions whose struct layouts this binding shares are accepted -- ABI
    # 4 added entry points to 3 without touching a layout -- and the entry
    # points an older library lacks are then unavailable)
    v = lib.ipt_abi_version()
    if v != ABI_VERSION:
        if not (os.environ.get("IPT_ABI_COMPAT") and v in ABI_LAYOUT_COMPATIBLE):
            raise IptError(IPT_E_INVALID, f"{p}: ABI {v} != {ABI_VERSION}; rebuild")
        import warnings
        warnings.warn(f"{p}: loading ABI {v} under IPT_ABI_COMPAT (binding is ABI {ABI_VERSION})")
    lib.ipt_last_error.restype = C.c_char_p
    lib.ipt_last_error.argtypes = [C.c_void_p]
    lib.ipt_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    lib.ipt_destroy.argtypes = [C.c_void_p]
    lib.ipt_destroy.restype = None
    lib.ipt_upload_scene.argtypes = [C.c_void_p, C.POINTER(Scene)]
    lib.ipt_render.argtypes = [C.c_void_p, C.POINTER(Params), C.POINTER(Image)]
    lib.ipt_render_device.argtypes = [C.c_void_p, C.POINTER(Params), C.POINTER(Image), C.c_void_p]
    if hasattr(lib, "ipt_render_device_async"):
        lib.ipt_render_device_async.argtypes = [C.c_void_p, C.POINTER(Params), C.POINTER(Image), C.c_void_p]
        lib.ipt_render_wait.argtypes = [C.c_void_p]
    if hasattr(lib, "ipt_transfer_bytes"):
        lib.ipt_transfer_bytes.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    lib.ipt_render_values.argtypes = [C.c_void_p, C.POINTER(Params), C.c_void_p, C.c_void_p]
    lib.ipt_get_counters.argtypes = [C.c_void_p, C.POINTER(Counters)]
    lib.ipt_reset_counters.argtypes = [C.c_void_p]
    lib.ipt_math_selfcheck.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_uint64,
                                       C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
    lib.ipt_ddf_sample.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    lib.ipt_ddf_value.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    lib.ipt_smooth.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                               C.POINTER(C.c_float)]
    lib.ipt_glare.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_float]
    lib.ipt_get_profile.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    lib.ipt_last_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    lib.ipt_math_host.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int64]
    lib.ipt_math_device.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64]
    lib.ipt_shard_plan.argtypes = [C.POINTER(Params), C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)]
    lib.ipt_philox.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int64]
    if path is None:
        _lib = lib
    return lib


def _check(lib, ctx, rc):
    if rc != IPT_OK:
        raise IptError(rc, lib.ipt_last_error(ctx).decode(errors="replace"))


def make_scene(desc: dict) -> tuple[Scene, list]:
    """Build an ipt_scene from the dict produced by ipt_amd.scenes; returns the
    struct and the Python objects that keep its arrays alive."""
    lights = desc.get("lights", [])
    la = (AreaLight * max(len(lights), 1))()
    for i, L in enumerate(lights):
        la[i].position[:] = L["position"]
        la[i].x_axis[:] = L["x_axis"]
        la[i].y_axis[:] = L["y_axis"]
        la[i].power = L["power"]
        la[i].type = L.get("type", IPT_LIGHT_AREA_DIAMOND)
    spheres = desc.get("spheres", [])
    sa = (Sphere * max(len(spheres), 1))()
    for i, (c, r) in enumerate(spheres):
        sa[i].center[:] = c
        sa[i].radius = r
    cam = desc["camera"]
    s = Scene()
    s.geometry_kind = desc["geometry_kind"]
    s.n_lights = len(lights)
    s.lights = C.cast(la, C.POINTER(AreaLight))
    s.n_spheres = len(spheres)
    s.spheres = C.cast(sa, C.POINTER(Sphere))
    s.camera.position[:] = cam["position"]
    s.camera.direction[:] = cam["direction"]
    s.camera.right[:] = cam["right"]
    s.camera.up[:] = cam["up"]
    return s, [la, sa]


def make_params(width, height, spp, spp_offset=0, n_rays=16, depth_max=8, seed=20241223,
                tile_rows=0, n_shards=1, shard_id=0, flags=0) -> Params:
    p = Params()
    p.width, p.height, p.spp, p.spp_offset = width, height, spp, spp_offset
    p.n_rays, p.depth_max, p.seed = n_rays, depth_max, seed
    p.tile_rows, p.n_shards, p.shard_id, p.flags = tile_rows, n_shards, shard_id, flags
    return p


class Context:
    """One ipt_ctx on one HIP device."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        rc = self.lib.ipt_create(device, C.byref(h))
        if rc != IPT_OK:
            raise IptError(rc, self.lib.ipt_last_error(None).decode(errors="replace"))
        self.h = h
        self._keep = None

    def close(self):
        if self.h:
            self.lib.ipt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload_scene(self, desc: dict):
        s, keep = make_scene(desc)
        _check(self.lib, self.h, self.lib.ipt_upload_scene(self.h, C.byref(s)))
        self._keep = keep

    def render_values(self, p: Params):
        n = p.spp * p.width * p.height
        vals = np.zeros(n, np.float32)
        codes = np.zeros(n, np.uint8)
        _check(self.lib, self.h, self.lib.ipt_render_values(
            self.h, C.byref(p), vals.ctypes.data, codes.ctypes.data))
        shape = (p.spp, p.height, p.width)
        return vals.reshape(shape), codes.reshape(shape)

    def render(self, p: Params, img: dict):
        """Host-buffer render into img = {pixels, counters, sums?, pixel_max?} (numpy)."""
        im = Image()
        im.pixels = img["pixels"].ctypes.data
        im.counters = img["counters"].ctypes.data
        im.sums = img["sums"].ctypes.data if img.get("sums") is not None else None
        im.pixel_max = img["pixel_max"].ctypes.data if img.get("pixel_max") is not None else None
        _check(self.lib, self.h, self.lib.ipt_render(self.h, C.byref(p), C.byref(im)))

    def transfer_bytes(self) -> tuple[int, int]:
        """(host -> device, device -> host) bytes of the last render() call."""
        h2d, d2h = C.c_uint64(), C.c_uint64()
        _check(self.lib, self.h, self.lib.ipt_transfer_bytes(self.h, C.byref(h2d), C.byref(d2h)))
        return int(h2d.value), int(d2h.value)

    def render_device(self, p: Params, pixels_ptr, counters_ptr, sums_ptr=None, max_ptr=None,
                      stream=None):
        im = Image()
        im.pixels, im.counters, im.sums, im.pixel_max = pixels_ptr, counters_ptr, sums_ptr, max_ptr
        _check(self.lib, self.h, self.lib.ipt_render_device(self.h, C.byref(p), C.byref(im), stream))

    def render_device_async(self, p: Params, pixels_ptr, counters_ptr, sums_ptr=None, max_ptr=None,
                            stream=None):
        """Queue the render (ipt_render_device_async); complete on `stream`'s
        order or after wait()."""
        im = Image()
        im.pixels, im.counters, im.sums, im.pixel_max = pixels_ptr, counters_ptr, sums_ptr, max_ptr
        _check(self.lib, self.h, self.lib.ipt_render_device_async(self.h, C.byref(p), C.byref(im), stream))

    def wait(self):
        _check(self.lib, self.h, self.lib.ipt_render_wait(self.h))

    @property
    def has_async(self) -> bool:
        return hasattr(self.lib, "ipt_render_device_async")

    def counters(self) -> dict:
        c = Counters()
        _check(self.lib, self.h, self.lib.ipt_get_counters(self.h, C.byref(c)))
        return c.as_dict()

    def reset_counters(self):
        _check(self.lib, self.h, self.lib.ipt_reset_counters(self.h))

    def math_selfcheck(self, fn: int, lo_bits: int = 0, hi_bits: int = 1 << 32):
        """(mismatches, first differing bit pattern) of the device fast path of
        math fn against its exact restatement over [lo_bits, hi_bits)."""
        bad, first = C.c_uint64(), C.c_uint32()
        _check(self.lib, self.h, self.lib.ipt_math_selfcheck(self.h, fn, lo_bits, hi_bits, C.byref(bad),
                                                             C.byref(first)))
        return int(bad.value), int(first.value)

    def ddf_sample(self, kind: int, params, u: np.ndarray) -> np.ndarray:
        """n directions from n x {pick, u1, u2} uniforms (ipt_ddf_sample)."""
        pr = np.ascontiguousarray(np.pad(np.asarray(params, np.float32), (0, 8))[:8])
        uu = np.ascontiguousarray(u, np.float32).reshape(-1, 3)
        out = np.empty((len(uu), 3), np.float32)
        _check(self.lib, self.h, self.lib.ipt_ddf_sample(self.h, kind, pr.ctypes.data, uu.ctypes.data, len(uu),
                                                         out.ctypes.data))
        return out

    def ddf_value(self, kind: int, params, dirs: np.ndarray) -> np.ndarray:
        pr = np.ascontiguousarray(np.pad(np.asarray(params, np.float32), (0, 8))[:8])
        dd = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        out = np.empty(len(dd), np.float32)
        _check(self.lib, self.h, self.lib.ipt_ddf_value(self.h, kind, pr.ctypes.data, dd.ctypes.data, len(dd),
                                                        out.ctypes.data))
        return out

    def smooth(self, pixels: np.ndarray, width: int, height: int, side: int, in_place: bool = True):
        """GridRenderPlane::smooth (in_place) / computeSmoothedMax on the GPU:
        returns (pixels after the call, max_value)."""
        px = np.ascontiguousarray(pixels, dtype=np.float32).copy()
        mx = C.c_float()
        _check(self.lib, self.h, self.lib.ipt_smooth(self.h, px.ctypes.data, width, height, side,
                                                     1 if in_place else 0, C.byref(mx)))
        return px, float(mx.value)

    def glare(self, img: np.ndarray, width: int, height: int, cutoff: float) -> np.ndarray:
        """Gui's glare bloom (gui.cpp:28-52) on the GPU."""
        src = np.ascontiguousarray(img, dtype=np.float32)
        out = np.empty_like(src)
        _check(self.lib, self.h, self.lib.ipt_glare(self.h, src.ctypes.data, out.ctypes.data, width, height,
                                                    C.c_float(cutoff)))
        return out

    def profile(self) -> dict:
        """{phase: (wave executions, active lanes)} from an IPT_PROF build."""
        n = 2 * len(PROFILE_PHASES) + 12
        buf = (C.c_uint64 * n)()
        _check(self.lib, self.h, self.lib.ipt_get_profile(self.h, buf, n))
        out = {ph: (int(buf[2 * i]), int(buf[2 * i + 1])) for i, ph in enumerate(PROFILE_PHASES)}
        base = 2 * len(PROFILE_PHASES)
        out["stamps"] = {sg: int(buf[base + i]) for i, sg in enumerate(STAMP_SEGMENTS)}
        return out

    def last_kernel_ms(self):
        a, b = C.c_float(), C.c_float()
        _check(self.lib, self.h, self.lib.ipt_last_kernel_ms(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def math_device(self, fn: int, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float32)
        out = np.empty_like(x)
        _check(self.lib, self.h, self.lib.ipt_math_device(self.h, fn, x.ctypes.data, out.ctypes.data, x.size))
        return out


def philox(ctr, key, ctx: "Context | None" = None) -> np.ndarray:
    """Philox4x32-10 blocks as the kernels compute them (ipt_philox): ctr
    [n][4] uint32, key (k0, k1); ctx None = the library's host build."""
    lib = load()
    c = np.ascontiguousarray(np.asarray(ctr, np.uint32).reshape(-1, 4))
    out = np.zeros_like(c)
    h = ctx.h if ctx is not None else None
    rc = lib.ipt_philox(h, int(key[0]), int(key[1]), c.ctypes.data, out.ctypes.data, len(c))
    if rc != IPT_OK:
        raise IptError(rc, lib.ipt_last_error(h).decode(errors="replace") if h else "ipt_philox")
    return out


def math_host(fn: int, x: np.ndarray) -> np.ndarray:
    lib = load()
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    rc = lib.ipt_math_host(fn, x.ctypes.data, out.ctypes.data, x.size)
    if rc != IPT_OK:
        raise IptError(rc, "ipt_math_host")
    return out


MATH_FNS = {"acosf": 0, "sinf": 1, "cosf": 2, "acos_f64_f32": 3, "sincosf_sin": 4,
            "sincosf_cos": 5, "sqrtf": 6, "div_pi": 7, "two_pi_times": 8, "div_pairs": 9,
            "div_inrange_pairs": 10, "longer_pairs": 11, "udiv_exact_pairs": 12,
            "sqrt_inrange": 13, "frame_angle_sin": 14, "frame_angle_cos": 15}
SELFCHECK_FRAME_FAST = 16  # ipt_math_selfcheck only: fast vs exact sphere-in-box frame
# ipt_math_selfcheck only: reciprocal with 1 / 2 Newton corrections vs the round-4 three-correction
# sequence; the range-free division vs IEEE over the division pairs / near-all-ones divisors
SELFCHECK_RCP1, SELFCHECK_RCP2, SELFCHECK_DIV_PAIRS, SELFCHECK_DIV_ONES = 17, 18, 19, 20
# ipt_math_selfcheck only: the range-free division over every pair of significands (pattern
# indices up to 2^46) and the reciprocal's exact scaling over the range (all 2^32 floats)
SELFCHECK_DIV_ALL_SIGNIFICANDS, SELFCHECK_RCP_SCALING = 21, 22


def shard_plan(p: Params):
    """(owned_rows bool[H], candidate source rows int[]) of a sharded render."""
    lib = load()
    owned = np.zeros(p.height, np.uint8)
    cand = np.zeros(p.height, np.int32)
    n = C.c_int32()
    rc = lib.ipt_shard_plan(C.byref(p), owned.ctypes.data, cand.ctypes.data, C.byref(n))
    if rc != IPT_OK:
        raise IptError(rc, "ipt_shard_plan")
    return owned.astype(bool), cand[:n.value].copy()
