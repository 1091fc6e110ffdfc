"""Edge cases of the C-ABI render path (include/ipt_capi.h) on the GPU.

* Degenerate frames: 1x1, single rows and columns, two-row frames -- the
  sizes where GridRenderPlane::addRay's float row index (the nominal source
  row H-2-y, row H-1 doubling into row 0, the empty last row;
  GridRenderPlane.cpp:61-75) and the camera's pixel-centre math
  (SimpleCamera, main.cpp:192-211) are at their extremes. The accumulated
  state, sharded and unsharded, must equal the oracle's addRay replay bit for
  bit.
* spp = 0: a valid call that renders nothing and leaves the plane untouched.
* Argument validation (ipt_capi.h error codes): every out-of-range parameter
  is refused with its code before any launch, and the context stays usable.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi, scenes

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (1, 7), (7, 1), (2, 2), (3, 2), (2, 3), (5, 17)]


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _plane(W, H):
    return {k: np.zeros(W * H, dt) for k, dt in (("pixels", np.float32), ("counters", np.uint32),
                                                ("sums", np.float32), ("pixel_max", np.float32))}


def _assert_plane_equal(img, ref):
    for k in ("pixels", "sums", "pixel_max"):
        assert np.array_equal(_bits(img[k]), _bits(ref[k])), k
    assert np.array_equal(img["counters"], ref["counters"])


@pytest.mark.parametrize("W,H", SIZES)
def test_degenerate_frames_bit_exact(gpu_ctx, oracle, W, H):
    desc = scenes.make_scene_box()
    gpu_ctx.upload_scene(desc)
    p = capi.make_params(W, H, 5, spp_offset=11)
    gv, gc = gpu_ctx.render_values(p)
    ov, oc = ob.render_values(desc, p)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov))
    img = _plane(W, H)
    gpu_ctx.render(p, img)
    _assert_plane_equal(img, ob.accumulate(ov, oc))


@pytest.mark.parametrize("W,H,tile,n_shards", [(3, 2, 1, 2), (1, 7, 2, 3), (5, 17, 4, 4), (4, 3, 4, 3)])
def test_degenerate_frames_sharded(gpu_ctx, oracle, W, H, tile, n_shards):
    """Every shard of a plan whose tiles are as small as the frame allows
    (shards with no rows included), each into a plane of its own: a shard
    writes only its owned rows, and the assembled plane == the oracle's whole
    frame."""
    desc = scenes.make_scene_box()
    gpu_ctx.upload_scene(desc)
    img = _plane(W, H)
    for s in range(n_shards):
        p = capi.make_params(W, H, 4, spp_offset=1, tile_rows=tile, n_shards=n_shards, shard_id=s)
        part = _plane(W, H)
        gpu_ctx.render(p, part)
        owned, _ = capi.shard_plan(p)
        mask = np.repeat(owned, W)
        for k in img:
            assert not part[k][~mask].any(), "shard wrote outside its rows"
            img[k][mask] = part[k][mask]
    ov, oc = ob.render_values(desc, capi.make_params(W, H, 4, spp_offset=1))
    _assert_plane_equal(img, ob.accumulate(ov, oc))


def test_zero_spp_is_a_no_op(gpu_ctx):
    gpu_ctx.upload_scene(scenes.make_scene_box())
    W, H = 6, 5
    img = _plane(W, H)
    gpu_ctx.render(capi.make_params(W, H, 3), img)
    before = {k: v.copy() for k, v in img.items()}
    gpu_ctx.render(capi.make_params(W, H, 0, spp_offset=3), img)
    for k in img:
        assert np.array_equal(_bits(img[k]), _bits(before[k])), k


def _with(p, **kw):
    for k, v in kw.items():
        setattr(p, k, v)
    return p


BAD = [
    (dict(width=0), capi.IPT_E_INVALID),
    (dict(height=0), capi.IPT_E_INVALID),
    (dict(width=-3), capi.IPT_E_INVALID),
    (dict(width=65537), capi.IPT_E_INVALID),
    (dict(width=65536, height=65536), capi.IPT_E_INVALID),  # more than 2^31 pixels
    (dict(spp=-1), capi.IPT_E_INVALID),
    (dict(spp_offset=-1), capi.IPT_E_INVALID),
    (dict(depth_max=-1), capi.IPT_E_INVALID),
    (dict(depth_max=65), capi.IPT_E_INVALID),
    (dict(n_rays=-1), capi.IPT_E_UNSUPPORTED),
    (dict(n_rays=65536), capi.IPT_E_UNSUPPORTED),
    (dict(n_rays=512, depth_max=10), capi.IPT_E_UNSUPPORTED),  # 512 >> 9 = 1: 9 suspended levels (> 8)
    (dict(tile_rows=4, n_shards=3, shard_id=3), capi.IPT_E_INVALID),
    (dict(tile_rows=4, n_shards=3, shard_id=-1), capi.IPT_E_INVALID),
]


@pytest.mark.parametrize("bad,code", BAD, ids=[",".join(f"{k}={v}" for k, v in b.items()) for b, _ in BAD])
def test_invalid_params_refused(gpu_ctx, bad, code):
    """Each entry point validates its parameters before it looks at its
    buffers: called with NULL buffers, it must return the parameter's own code
    (a NULL-buffer refusal would mean the parameter got through)."""
    lib = capi.load()
    gpu_ctx.upload_scene(scenes.make_scene_box())
    W, H = 4, 3
    p = _with(capi.make_params(W, H, 2), **bad)
    null_img = capi.Image()
    for call in (lambda: lib.ipt_render(gpu_ctx.h, C.byref(p), C.byref(null_img)),
                 lambda: lib.ipt_render_device(gpu_ctx.h, C.byref(p), C.byref(null_img), None),
                 lambda: lib.ipt_render_values(gpu_ctx.h, C.byref(p), None, None)):
        assert call() == code
        assert b"NULL" not in lib.ipt_last_error(gpu_ctx.h)
    # the context still renders
    img = _plane(W, H)
    gpu_ctx.render(capi.make_params(W, H, 2), img)
    assert img["counters"].sum() > 0


def test_null_image_refused(gpu_ctx):
    lib = capi.load()
    gpu_ctx.upload_scene(scenes.make_scene_box())
    p = capi.make_params(4, 3, 1)
    im = capi.Image()
    assert lib.ipt_render(gpu_ctx.h, C.byref(p), C.byref(im)) == capi.IPT_E_INVALID
    assert b"NULL" in lib.ipt_last_error(gpu_ctx.h)
    assert lib.ipt_render_values(gpu_ctx.h, C.byref(p), None, None) == capi.IPT_E_INVALID
