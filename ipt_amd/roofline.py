"""Algorithmic cost model of the hot path and gfx950 peaks.

The path kernel is bound by instruction issue (no MFMA; its HBM traffic is
the radiance output, the raygen records and the CosineDdf / frame-table
gathers: ~0.6 KB per path at a fraction of 8 TB/s, their latency hidden), so
its roofline is the VALU issue rate. The op count
is ALGORITHMIC: the reference's own arithmetic per event, counted as written
(no credit for work the GPU kernel avoids, e.g. precomputed wall frames), with
each transcendental (acos, sin, cos) at 20 op-eq. Event counts come from the
kernel's own counters (ipt_counters), which tests pin equal to the oracle's.
"""
from __future__ import annotations

# gfx950 (MI355X): 256 CU x 4 SIMD-32, wave64 VALU instruction every 2 cycles
# per SIMD at 2.4 GHz -> 256*4*32*2.4e9 = 78.6e12 lane-ops/s (the 157.3 TFLOP/s
# FP32 spec counts an FMA as 2; the reference's arithmetic has no FMAs and must
# not be contracted). /opt/skills/guides/MI355X_MICROARCH.md "Chip-level".
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
HBM_PEAK_GBPS = 8000.0  # spec; ~6.3 TB/s achievable (guide §HBM)
TRANSC_OP_EQ = 20

# per-event FP op counts
OPS = {
    "camera": 28,            # camera + jitter, per path
    "geom_trace": 130,       # box: 127 miss / 133 hit
    "light_trace": 57,       # area light trace (miss cost; hits +23 are in light_hit)
    "occlusion": 18,         # light-vs-geometry length compare, per light hit
    "rotate_build": 109,     # RotateDdf built by every geometry hit (GeometrySphereInBox.cpp:63-74)
    "mixture_weights": 8,    # unite() weights, per expanded node
    "sphere_normal": 10,     # per sphere-hit frame
    "iter_light_kept": 207,  # light-sampled branch iteration, kept
    "iter_cosine": 118,      # cosine-sampled branch iteration
    "iter_skipped": 56,      # skipped (back-facing light sample)
    "node_finalize": 1,
    "sphere_test": 37,       # intersection_with_sphere + FractalSpheres acceptance
    "bvh_node": 29,          # slab test + entry/prune compares, per BVH node visited
    "light_cell": 30,        # light lattice: plane point, cell coordinates, <= 4 cell reads, per trace
}
TRANSC = {"rotate_build": 3, "iter_cosine": 4}


def light_lattice(c: dict, n_lights: int) -> bool:
    """The many-light scene ran the light lattice lookup (no BVH nodes, and far
    fewer light tests than the reference's scans)."""
    return (n_lights > 16 and c.get("light_nodes", 0) == 0
            and c["light_tests"] < 0.25 * max(c["light_traces"], 1))


def ops_from_counters(c: dict, n_spheres: int = 0, n_lights: int = 1) -> float:
    """Algorithmic op-eq for a set of ipt_counters. The base formula is §8(d)'s
    for sample_scenes[0]; many-light scenes add 57 per AreaLight::traceRay
    beyond the box's two per traced ray, sphere-stress scenes add 37 per
    sphere test (§8(d): "C3 adds N x 37 per trace"). Where a BVH or the light
    lattice replaced a scan, the tests actually run are priced (plus 29 per
    BVH node, 30 per lattice lookup), not the scan."""
    kept_light = c["light_samples"] - c["skipped"]
    cosine = c["iterations"] - c["light_samples"]
    lattice = light_lattice(c, n_lights)
    light_bvh = c.get("light_nodes", 0) > 0 or lattice
    f = (c["paths"] * OPS["camera"]
         + c["traced_rays"] * OPS["geom_trace"]
         + (c["light_tests"] * OPS["light_trace"] + c["light_nodes"] * OPS["bvh_node"]
            + (c["traced_rays"] * OPS["light_cell"] if lattice else 0) if light_bvh
            else c["traced_rays"] * OPS["light_trace"])
         + c["light_hits"] * OPS["occlusion"]
         + c["surface_hits"] * (OPS["rotate_build"] + TRANSC["rotate_build"] * TRANSC_OP_EQ)
         + c["expanded_nodes"] * OPS["mixture_weights"]
         + c["sphere_frames"] * OPS["sphere_normal"]
         + kept_light * OPS["iter_light_kept"]
         + cosine * (OPS["iter_cosine"] + TRANSC["iter_cosine"] * TRANSC_OP_EQ)
         + c["skipped"] * OPS["iter_skipped"]
         + c["expanded_nodes"] * OPS["node_finalize"])
    if not light_bvh:
        f += max(0, c["light_traces"] - 2 * c["traced_rays"]) * OPS["light_trace"]
    if "sphere_tests" in c:
        f += c["sphere_tests"] * OPS["sphere_test"] + c.get("bvh_nodes", 0) * OPS["bvh_node"]
    else:
        f += c["traced_rays"] * n_spheres * OPS["sphere_test"]
    return float(f)


def reference_scan_ops(c: dict, n_spheres: int) -> float:
    """Op-eq of the reference's brute-force sphere and light scans for the
    same rays (work the BVH walks skip)."""
    f = float(c["traced_rays"]) * n_spheres * OPS["sphere_test"]
    f += (c["traced_rays"] + max(0, c["light_traces"] - 2 * c["traced_rays"])) * OPS["light_trace"]
    return f


def accumulate_bytes(n_dest_pixels: int, spp: int, with_sums: bool = True,
                     with_max: bool = True) -> int:
    """Algorithmic HBM bytes of one accumulate launch: the radiance buffer read
    once (4 B per sample) + the GridRenderPlane state read and written."""
    state = 8 + (4 if with_sums else 0) + (4 if with_max else 0)
    return n_dest_pixels * (4 * spp + 2 * state)


def path_bytes(paths: int, cosine_samples: int = 0, frame_builds: int = 0) -> int:
    """HBM bytes of one launch of the path's per-sample work (raygen_kernel +
    path_kernel), as the kernels move them: 4 B radiance + 1 B drift code
    written per path, the 32 B raygen record written by raygen_kernel and read
    back by path_kernel, the 4-byte CosineDdf r entry gathered per
    cosine-sampled iteration (64 MiB table; (cos phi, sin phi) is computed
    in-lane since round 2), and the 8-byte frame-table entry gathered per
    sphere-node frame build (1 GiB table; pushes counted, the ~30 % rebuilds
    after pops are not). Scene data is a few hundred bytes, read once per
    workgroup. The records and gathers are implementation choices (they
    replace VALU work); compulsory_bytes() is the reference's own traffic."""
    return (5 + 2 * 32) * paths + 4 * cosine_samples + 8 * frame_builds


# The per-sample output the GridRenderPlane replay needs: the 4-byte radiance
# and the 1-byte drift code of every path ("compulsory HBM
# traffic is about 8 B per pixel of output, <= 16 B/path").
COMPULSORY_BYTES_PER_PATH = 5


def compulsory_bytes(paths: int) -> int:
    return COMPULSORY_BYTES_PER_PATH * paths
