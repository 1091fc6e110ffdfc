"""Scene descriptions for the C-ABI, built with the reference's constructor
arithmetic (float32, glm operation order) so that the flattened values equal
the fields of the reference objects bit-for-bit.

make_scene_box()       sample_scenes[0] (reference src/sample_scenes.cpp:20-41)
make_scene_box_lights  the [0] light split into k x k co-planar squares
                       (BASELINE.json configs[4])
make_scene_spheres     box planes + N seeded spheres (configs[2])

The C++ mirror (ipt_amd/host/sample_scenes.cpp) builds the same scenes for
C++ callers; tests check the two agree.
"""
from __future__ import annotations

import numpy as np

from .capi import (IPT_GEOM_CORNER, IPT_GEOM_FLOOR, IPT_GEOM_SMALLPT, IPT_GEOM_SPHERE_IN_BOX, IPT_GEOM_SPHERES,
                   IPT_GEOM_SPHERES_IN_BOX, IPT_LIGHT_AREA_DIAMOND, IPT_LIGHT_AREA_TRIANGLE, IPT_LIGHT_OUTER_SPHERE,
                   IPT_LIGHT_POINT, IPT_LIGHT_SPHERE)

f32 = np.float32


def _v(*a):
    return np.array(a, dtype=f32)


def dot(a, b):
    t = (a * b).astype(f32)
    return f32(f32(t[0] + t[1]) + t[2])


def cross(x, y):
    return np.array([f32(x[1] * y[2]) - f32(y[1] * x[2]),
                     f32(x[2] * y[0]) - f32(y[2] * x[0]),
                     f32(x[0] * y[1]) - f32(y[0] * x[1])], dtype=f32)


def normalize(v):
    s = f32(f32(1.0) / np.sqrt(dot(v, v), dtype=f32))
    return (v * s).astype(f32)


def simple_camera(position, direction, up_hint=(0.0, 0.0, 1.0)):
    """SimpleCamera ctor (reference src/SimpleCamera.cpp:8-13)."""
    position = _v(*position)
    direction = _v(*direction)
    right = normalize(cross(direction, _v(*up_hint)))
    up = normalize(cross(right, direction))
    return {"position": position.tolist(), "direction": direction.tolist(),
            "right": right.tolist(), "up": up.tolist()}


def square_light(corner, normal, x_side, power=1.0):
    """CollectionLighting::addSquareLight (CollectionLighting.cpp:42-46)."""
    corner = _v(*corner)
    x_side = _v(*x_side)
    y_side = cross(_v(*normal), x_side)
    return {"position": corner.tolist(), "x_axis": x_side.tolist(), "y_axis": y_side.tolist(),
            "power": float(f32(power)), "type": IPT_LIGHT_AREA_DIAMOND}


def box_camera():
    # sample_scenes.cpp:36-38
    camera_pos = _v(0.0, -3.0, 0.1)
    camera_dir = normalize((_v(0.0, 1.0, -1.0) - camera_pos).astype(f32))
    return simple_camera(camera_pos, camera_dir)


def box_light_corner():
    # vec3{+0.1f, -0.8f-0.1f, -0.15f}: -0.8f-0.1f is a float subtraction
    return (f32(0.1), f32(f32(-0.8) - f32(0.1)), f32(-0.15))


def make_scene_box():
    """sample_scenes[0]: GeometrySphereInBox + one 0.2x0.2 square light."""
    light = square_light(box_light_corner(), (0.0, 0.0, -1.0), (0.0, 0.2, 0.0), 1.0)
    return {"geometry_kind": IPT_GEOM_SPHERE_IN_BOX, "lights": [light], "spheres": [],
            "camera": box_camera()}


def make_scene_square_lit_by_square():
    """sample_scenes.cpp:73-85: GeometryFloor lit by a 0.1 square, camera at
    (0,-5,0) looking at (0,0,-1), direction scaled by 2, up hint +y."""
    light = square_light((-0.05, -0.05, -0.9), (0.0, 0.0, -1.0), (0.0, 0.1, 0.0), 1.0)
    camera_pos = _v(0.0, -5.0, 0.0)
    camera_dir = normalize((_v(0.0, 0.0, -1.0) - camera_pos).astype(f32))
    cam = simple_camera(camera_pos, (camera_dir * f32(2.0)).astype(f32), up_hint=(0.0, 1.0, 0.0))
    return {"geometry_kind": IPT_GEOM_FLOOR, "lights": [light], "spheres": [], "camera": cam}


def make_scene_lit_corner():
    """sample_scenes.cpp:88-108: GeometryCorner lit by a triangle light
    (addTriangleLight(cx, cz-cx, cy-cx)), camera at (4,1,1) looking at 0."""
    out = _v(1.0, 1.0, 1.0)
    half = (f32(0.5) * out).astype(f32)
    cx = (_v(-0.5, -1.0, -1.0) + half).astype(f32)
    cy = (_v(-1.0, -0.5, -1.0) + half).astype(f32)
    cz = (_v(-1.0, -1.0, -0.5) + half).astype(f32)
    light = {"position": cx.tolist(), "x_axis": (cz - cx).astype(f32).tolist(),
             "y_axis": (cy - cx).astype(f32).tolist(), "power": 1.0, "type": IPT_LIGHT_AREA_TRIANGLE}
    camera_pos = _v(4.0, 1.0, 1.0)
    camera_dir = normalize((_v(0.0, 0.0, 0.0) - camera_pos).astype(f32))
    return {"geometry_kind": IPT_GEOM_CORNER, "lights": [light], "spheres": [],
            "camera": simple_camera(camera_pos, camera_dir)}


def sphere_light(position, radius, power=1.0):
    """CollectionLighting::addSphereLight (CollectionLighting.cpp:39-41)."""
    return {"position": _v(*position).tolist(), "x_axis": [float(f32(radius)), 0.0, 0.0],
            "y_axis": [0.0, 0.0, 0.0], "power": float(f32(power)), "type": IPT_LIGHT_SPHERE}


def point_light(position, virtual_radius, power=1.0):
    """CollectionLighting::addPointLight (CollectionLighting.cpp:36-38)."""
    return {"position": _v(*position).tolist(), "x_axis": [float(f32(virtual_radius)), 0.0, 0.0],
            "y_axis": [0.0, 0.0, 0.0], "power": float(f32(power)), "type": IPT_LIGHT_POINT}


def outer_light(radius, power=1.0):
    """CollectionLighting::addOuterLight (CollectionLighting.cpp:52-55)."""
    return {"position": [0.0, 0.0, 0.0], "x_axis": [float(f32(radius)), 0.0, 0.0],
            "y_axis": [0.0, 0.0, 0.0], "power": float(f32(power)), "type": IPT_LIGHT_OUTER_SPHERE}


_libm = None


def _glibc():
    """glibc's float asinf/sinf, as FractalSpheres' generator calls them."""
    global _libm
    if _libm is None:
        import ctypes
        _libm = ctypes.CDLL("libm.so.6")
        for fn in ("asinf", "sinf"):
            getattr(_libm, fn).restype = ctypes.c_float
            getattr(_libm, fn).argtypes = [ctypes.c_float]
    return _libm


def fractal_spheres():
    """FractalSpheres::FractalSpheres (FractalSpheres.cpp:46-67) with
    generate_spheres (FractalSpheres.cpp:16-44), float arithmetic and glibc
    asinf/sinf: a list of (centre, radius)."""
    m = _glibc()
    pi = f32(3.14159265358979323846)  # M_PIf32

    def length(v):
        return np.sqrt(dot(v, v), dtype=f32)

    spheres = []

    def add(r, c):
        if float(r) < 0.001:
            return True
        spheres.append((c.astype(f32).tolist(), float(r)))
        return False

    def gen(r1, c1, r2, c2, left):
        L = f32(f32(length((c1 - c2).astype(f32)) - r1) - r2)
        if float(L) < 0.01:
            return
        sin_alpha = f32(r1 / f32(r1 + L))
        alpha = f32(m.asinf(sin_alpha))
        sin_beta = f32(r2 / f32(r2 + L))
        beta = f32(m.asinf(sin_beta))
        gamma = f32(f32(pi - alpha) - beta)
        A = f32(f32(L * sin_alpha) / f32(m.sinf(gamma)))
        x = f32(f32(A * f32(m.sinf(f32(gamma / f32(2))))) / f32(m.sinf(f32(f32(pi - beta) - f32(gamma / f32(2))))))
        c3 = (c1 + (normalize((c2 - c1).astype(f32)) * f32(x + r1)).astype(f32)).astype(f32)
        r3 = f32(x * sin_beta)
        if add(r3, c3):
            return
        if left:
            gen(r1, c1, r3, c3, not left)
        else:
            gen(r3, c3, r2, c2, not left)

    r1, c1, r2, c2 = f32(0.5), _v(-2.0, 0.0, 0.0), f32(0.5), _v(2.0, 0.0, 0.0)
    add(r1, c1)
    add(r2, c2)
    gen(r1, c1, r2, c2, True)
    return spheres


def make_scene_fractal():
    """sample_scenes.cpp:43-55: FractalSpheres lit by a unit SphereLight at
    (-5.5,0,0), camera at (0,-4,0) looking along +y."""
    cam = simple_camera(_v(0.0, -4.0, 0.0), _v(0.0, 1.0, 0.0))
    return {"geometry_kind": IPT_GEOM_SPHERES, "lights": [sphere_light((-5.5, 0.0, 0.0), 1.0)],
            "spheres": fractal_spheres(), "camera": cam}


def smallpt_spheres():
    """GeometrySmallPt.cpp:24-33: smallpt's room (radius, centre), the centres
    written as double expressions converted to float by glm::vec3."""
    return [
        ([1e3 + 1, 40.8, 81.6], 1e3),   # left
        ([-1e3 + 99, 40.8, 81.6], 1e3),  # right
        ([50, 40.8, 1e3], 1e3),          # back
        ([50, 1e3, 81.6], 1e3),          # bottom
        ([50, -1e3 + 81.6, 81.6], 1e3),  # top
        ([27, 16.5, 47], 16.5),
        ([73, 16.5, 78], 16.5),          # glass
    ]


def make_scene_smallpt():
    """sample_scenes.cpp:57-71: smallpt's room lit by an 8x8 square light,
    camera at (50,52,295.6), direction normalize((0,-0.042612,-1))*2, up +y."""
    spheres = [([float(f32(v)) for v in c], float(f32(r))) for c, r in smallpt_spheres()]
    lc = _v(50, 81.6 - 16.5, 81.6)
    light = square_light((lc - _v(4.0, 0, 4.0)).astype(f32), (0.0, -1.0, 0.0), (8.0, 0.0, 0.0), 1.0)
    camera_pos = _v(50.0, 52.0, 295.6)
    camera_dir = normalize(_v(0.0, -0.042612, -1.0))
    cam = simple_camera(camera_pos, (camera_dir * f32(2.0)).astype(f32), up_hint=(0.0, 1.0, 0.0))
    return {"geometry_kind": IPT_GEOM_SMALLPT, "lights": [light], "spheres": spheres, "camera": cam}


def make_scene_box_lights(k: int = 16):
    """The [0] light split into k*k co-planar squares of power 1/k^2 each, via
    the public addSquareLight. Expected image equals [0]'s."""
    c0 = box_light_corner()
    side = f32(f32(0.2) / f32(k))
    lights = []
    for a in range(k):
        for b in range(k):
            corner = (f32(c0[0] + f32(f32(b) * side)), f32(c0[1] + f32(f32(a) * side)), c0[2])
            lights.append(square_light(corner, (0.0, 0.0, -1.0), (0.0, float(side), 0.0),
                                       float(f32(1.0) / f32(k * k))))
    return {"geometry_kind": IPT_GEOM_SPHERE_IN_BOX, "lights": lights, "spheres": [],
            "camera": box_camera()}


def splitmix64(seed):
    x = np.uint64(seed)
    while True:
        x = np.uint64(x + np.uint64(0x9E3779B97F4A7C15))
        z = x
        z = np.uint64((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9))
        z = np.uint64((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB))
        yield int(z ^ (z >> np.uint64(31)))


def make_scene_random_lights(n: int = 64, seed: int = 7):
    """Box + n overlapping emitters of random position, orientation and shape
    (parallelograms via Light(corner, x, y) and triangles as addTriangleLight,
    CollectionLighting.cpp:47-50), SplitMix64(seed). Rays cross several
    emitters, exercising traceRayToLight's nearest rule and UnionDdf::value's
    index-order sum over many hits."""
    g = splitmix64(seed)

    def u():
        return f32((next(g) >> 40) * (1.0 / (1 << 24)))

    lights = []
    with np.errstate(over="ignore"):
        for i in range(n):
            corner = [float(f32(f32(-0.8) + f32(f32(1.4) * u()))) for _ in range(3)]
            xs = [float(f32(f32(0.6) * u() - f32(0.3))) for _ in range(3)]
            ys = [float(f32(f32(0.6) * u() - f32(0.3))) for _ in range(3)]
            power = float(f32(f32(0.2) + f32(0.8) * u()))
            lights.append({"position": corner, "x_axis": xs, "y_axis": ys, "power": power,
                           "type": IPT_LIGHT_AREA_TRIANGLE if i % 3 == 2 else IPT_LIGHT_AREA_DIAMOND})
    return {"geometry_kind": IPT_GEOM_SPHERE_IN_BOX, "lights": lights, "spheres": [],
            "camera": box_camera()}


def make_scene_spheres(n: int = 10000, seed: int = 1):
    """Box planes + n random spheres (centres uniform in [-0.9,0.9]^3, radius in
    [0.01,0.03], SplitMix64(seed)), same camera and light as [0]."""
    g = splitmix64(seed)

    def u():
        return f32((next(g) >> 40) * (1.0 / (1 << 24)))

    spheres = []
    with np.errstate(over="ignore"):
        for _ in range(n):
            c = [float(f32(f32(-0.9) + f32(f32(1.8) * u()))) for _ in range(3)]
            r = float(f32(f32(0.01) + f32(f32(0.02) * u())))
            spheres.append((c, r))
    light = square_light(box_light_corner(), (0.0, 0.0, -1.0), (0.0, 0.2, 0.0), 1.0)
    return {"geometry_kind": IPT_GEOM_SPHERES_IN_BOX, "lights": [light], "spheres": spheres,
            "camera": box_camera()}
