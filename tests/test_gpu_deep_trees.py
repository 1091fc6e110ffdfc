"""GPU parity of the estimator's deeper and non-power-of-two trees.

The reference takes n_rays from argv (/root/reference/src/main.cpp:239-243),
loops over i < n_rays at every node (main.cpp:149), hands n_rays/2 to each
child (main.cpp:177) and divides the node's sum by its own n
(main.cpp:181, `isfinite(res) ? res/n_rays : 0`). The kernel has two forms
of that division -- `r * 2^-e` for power-of-two n_rays and
`r / (float)(n_rays >> d)` otherwise (ipt_kernels.hip pop_node fin_v/fin_s) --
and two stack depths: MAXSUSP = 4 (every test elsewhere) and MAXSUSP = 8,
selected when a node deeper than 4 is pushed (n_rays >= 32 with depth_max >= 6).
Each case here is bit-exact against the oracle (oracle/ipt_oracle.cpp
ray_power, main.cpp:98-184) on every geometry/light family the kernels
specialise: the box (single axis-aligned light), the C5 light lattice, the
light BVH (random emitters), the C3 sphere grid, the sphere BVH and round
lights. Frames are sized so that the oracle stays within seconds.
"""
import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi, scenes

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _check(ctx, desc, p):
    ctx.upload_scene(desc)
    gv, gc = ctx.render_values(p)
    ov, oc = ob.render_values(desc, p, 0)
    assert np.array_equal(gc, oc)
    assert np.array_equal(_bits(gv), _bits(ov)), (
        f"{int((_bits(gv) != _bits(ov)).sum())} of {gv.size} samples differ; max |d| = {np.abs(gv - ov).max()}")
    return ov


def _round_lights_scene():
    base = scenes.make_scene_box()
    desc = dict(base)
    desc["lights"] = list(base["lights"]) + [
        scenes.sphere_light((0.3, 0.2, 0.4), 0.15, 0.7),
        scenes.point_light((-0.4, 0.3, -0.2), 0.05, 0.5),
        scenes.outer_light(9.0, 0.05),
    ]
    return desc


# (n_rays, depth_max, W, H, spp): MAXSUSP 8 (32, 64, deeper than the tree),
# non-power-of-two divisors at every depth (3 -> 1, 6 -> 3 -> 1, 12, 24, 100),
# wide roots within the 8-bit iteration field (128, 255)
BOX_CASES = [
    (32, 8, 12, 10, 1), (64, 8, 4, 4, 1), (64, 12, 4, 3, 1), (32, 6, 12, 8, 1), (32, 7, 8, 8, 2),
    (3, 8, 32, 24, 2), (6, 8, 32, 24, 2), (12, 8, 24, 16, 1), (24, 8, 16, 12, 1), (24, 5, 16, 12, 2),
    (100, 3, 8, 6, 1), (128, 3, 4, 4, 1), (255, 2, 4, 4, 1), (48, 8, 6, 4, 1),
]


@pytest.mark.parametrize("n_rays,depth_max,W,H,spp", BOX_CASES)
def test_box_deep_and_nonpow2_bit_exact(gpu_ctx, oracle, n_rays, depth_max, W, H, spp):
    p = capi.make_params(W, H, spp, spp_offset=3, n_rays=n_rays, depth_max=depth_max)
    ov = _check(gpu_ctx, scenes.make_scene_box(), p)
    assert (ov > 0).mean() > 0.3


@pytest.mark.parametrize("n_rays,depth_max,W,H", [(32, 8, 8, 8), (12, 8, 16, 12), (24, 8, 16, 12), (64, 7, 4, 4)])
def test_light_lattice_deep_bit_exact(gpu_ctx, oracle, n_rays, depth_max, W, H):
    """C5's 256-emitter lattice (kLightsGridA10; at MAXSUSP 8 the LDS-record
    instance does not fit one CU, so the global-record instance runs)."""
    p = capi.make_params(W, H, 1, n_rays=n_rays, depth_max=depth_max)
    _check(gpu_ctx, scenes.make_scene_box_lights(16), p)


@pytest.mark.parametrize("n_rays,depth_max", [(32, 8), (6, 8)])
def test_light_bvh_deep_bit_exact(gpu_ctx, oracle, n_rays, depth_max):
    """Overlapping random emitters: the resumable light-BVH walk (kLightsGlobal)."""
    p = capi.make_params(8, 6, 1, n_rays=n_rays, depth_max=depth_max)
    _check(gpu_ctx, scenes.make_scene_random_lights(64, seed=7), p)


@pytest.mark.parametrize("n_spheres,n_rays,depth_max,W,H", [
    (10000, 24, 8, 4, 3),   # C3's scene: the wave-spread grid walk, non-power-of-two n
    (10000, 6, 8, 8, 6),
    (3000, 32, 8, 6, 4),    # sphere grid at MAXSUSP 8
    (200, 32, 8, 8, 6),     # <= 256 spheres: the resumable sphere-BVH walk
    (200, 12, 8, 12, 8),
])
def test_sphere_lists_deep_bit_exact(gpu_ctx, oracle, n_spheres, n_rays, depth_max, W, H):
    p = capi.make_params(W, H, 1, n_rays=n_rays, depth_max=depth_max)
    _check(gpu_ctx, scenes.make_scene_spheres(n_spheres, seed=1), p)


@pytest.mark.parametrize("n_rays,depth_max,W,H", [(32, 8, 8, 8), (12, 8, 16, 12), (3, 8, 24, 16)])
def test_round_lights_deep_bit_exact(gpu_ctx, oracle, n_rays, depth_max, W, H):
    """Sphere / point / outer lights beside the area light (kLightsAny)."""
    p = capi.make_params(W, H, 1, n_rays=n_rays, depth_max=depth_max)
    _check(gpu_ctx, _round_lights_scene(), p)


@pytest.mark.parametrize("n_rays,depth_max", [(32, 8), (24, 8)])
def test_fractal_deep_bit_exact(gpu_ctx, oracle, n_rays, depth_max):
    """sample_scenes.cpp:43-55 (FractalSpheres, no walls, SphereLight)."""
    p = capi.make_params(48, 40, 1, n_rays=n_rays, depth_max=depth_max)
    _check(gpu_ctx, scenes.make_scene_fractal(), p)


def test_n_rays_limit(gpu_ctx):
    """What the 16-bit iteration field and the 8-level instances cannot hold is
    refused, not mis-rendered: n_rays above 65535, and trees deeper than 8
    suspended levels (n_rays >= 512 with depth_max >= 11)."""
    gpu_ctx.upload_scene(scenes.make_scene_box())
    for n, d in ((65536, 2), (1000, 11), (512, 11)):
        with pytest.raises(capi.IptError) as e:
            gpu_ctx.render_values(capi.make_params(4, 4, 1, n_rays=n, depth_max=d))
        assert e.value.code == capi.IPT_E_UNSUPPORTED, (n, d)


@pytest.mark.parametrize("scene,n,d", [("box", 256, 2), ("box", 300, 2), ("box", 1000, 2),
                                       ("box", 511, 3), ("spheres300", 260, 2)])
def test_wide_n_rays_bit_exact(gpu_ctx, oracle, scene, n, d):
    """n_rays above 255 (the reference takes any int from argv, main.cpp:239-243):
    the suspended level's iteration count in 16 bits, the node kind (6 + sphere
    index on the sphere-list scene) above it; power-of-two and other n."""
    desc = scenes.make_scene_box() if scene == "box" else scenes.make_scene_spheres(300)
    gpu_ctx.upload_scene(desc)
    p = capi.make_params(4, 3, 1, n_rays=n, depth_max=d)
    vals, codes = gpu_ctx.render_values(p)
    ov, oc = ob.render_values(desc, p)
    assert np.array_equal(vals.view(np.uint32), ov.view(np.uint32))
    assert np.array_equal(codes, oc)


def _duplicated_lattice(k, r, dup_stride):
    """k^3 lattice spheres, each listed twice (the copy dup_stride entries
    later), plus coincident copies of every 7th sphere at the end: equal t on
    distinct indices in every cell, spheres spanning several cells."""
    base = []
    for i in range(k):
        for j in range(k):
            for m in range(k):
                c = [float(np.float32(-0.8 + 1.6 * (q + 0.5) / k)) for q in (i, j, m)]
                base.append((c, float(np.float32(r))))
    sp = []
    for s in range(0, len(base), dup_stride):
        chunk = base[s:s + dup_stride]
        sp += chunk + chunk
    sp += base[::7]
    d = scenes.make_scene_spheres(1, seed=1)
    d["spheres"] = sp
    d["camera"] = scenes.simple_camera((0.05, -2.5, 0.1), (0.0, 1.0, 0.05))
    return d


@pytest.mark.parametrize("k,r,dup_stride", [(8, 0.14, 5), (6, 0.2, 1), (4, 0.05, 3)])
def test_coincident_spheres_tie_bit_exact(gpu_ctx, oracle, k, r, dup_stride):
    """exactly equal t on different sphere indices, within a cell
    and across cells (radius 0.14-0.2 spans several of the grid's cells; k=4
    has <= 256 spheres: the BVH). FractalSpheres.cpp:75-84 keeps the lowest
    index (strict '<'); the wave walk's (t bits, item position) slot key
    must reproduce that."""
    desc = _duplicated_lattice(k, r, dup_stride)
    p = capi.make_params(16, 12, 1, n_rays=8, depth_max=5)
    gpu_ctx.upload_scene(desc)
    gpu_ctx.reset_counters()
    _check(gpu_ctx, desc, p)


def _high_index_spheres(n_low=32800, n_high=200):
    """n_low tiny spheres (r = 1e-4, C3's random centres) listed before n_high
    large ones (r = 0.05-0.09) that fill the view: camera rays hit spheres
    whose kind 6 + index is >= 32768."""
    desc = scenes.make_scene_spheres(n_low + n_high, seed=3)
    sp = []
    for i, (c, r) in enumerate(desc["spheres"]):
        if i < n_low:
            sp.append((c, 1e-4))
        else:
            sp.append(([c[0] * 0.8, c[1] * 0.8, c[2] * 0.8], 0.05 + 0.04 * ((i * 7919) % 101) / 100.0))
    desc["spheres"] = sp
    return desc


def test_wide_n_rays_high_sphere_index_bit_exact(gpu_ctx, oracle):
    """with n_rays > 255 a suspended level's meta word is ti | kind
    << 16, and a sphere node's kind (6 + index) >= 32768 sets bit 31; the
    decode must not sign-extend it (a negative kind reads another lane's frame
    column). Camera rays hit spheres 32800..32999, whose children are pushed,
    so those nodes are suspended and resumed."""
    desc = _high_index_spheres()
    p = capi.make_params(8, 6, 1, n_rays=260, depth_max=2)
    ov = _check(gpu_ctx, desc, p)
    assert (ov != 0).mean() > 0.2
