"""Synthetic benchmark / parity scenes (BASELINE.json ``configs``).

Every random number comes from :class:`SplitMix64` seeded with ``0x5EED0000 + config id``, so
the same scene is rebuilt bit-identically by the bench, the tests and the golden generator.

* ``c1`` — the reference ``main()`` scene (RaytracingEngine.cpp:223-290) minus the OBJ model
  whose ``box.obj`` is absent from the reference repo: a 5-plane open box, 2 point lights,
  1000×1000, focal 500.
* ``c2`` — 1920×1080, 16 spheres + 2 planes (floor, back) + 1 point light.  THE bench config.
* ``c3`` — 3840×2160, 128 spheres + 4 planes + 4 point lights.
* ``c4`` — 7680×4320, 256 spheres + 8 point lights (row-tiled over 8 GPUs).
* ``c5`` — 3840×2160, 64 spheres + 1 build-defined area light, 16 shadow samples.

Feature scenes with no BASELINE counterpart (parity coverage of every TraceRay branch):
``mirror`` (reflection chain), ``glass`` (refraction tree + partial shadow transmittance),
``mesh`` (triangles + a Model).
"""
from __future__ import annotations

import math

from .scene import AreaLight, Camera, Material, SceneData

M64 = (1 << 64) - 1


class SplitMix64:
    """splitmix64 (Steele, Lea, Flood 2014): state += golden gamma, then the mix64 finalizer."""

    def __init__(self, seed: int):
        self.state = seed & M64

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & M64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def uniform(self, lo: float, hi: float) -> float:
        return lo + (hi - lo) * ((self.next_u64() >> 11) * 2.0 ** -53)


CONFIG_IDS = {"c1": 1, "c2": 2, "c3": 3, "c4": 4, "c5": 5, "mirror": 6, "glass": 7, "mesh": 8,
              "bigmesh": 9}

# name -> (width, height, n_spheres, plane list, n_lights)
_PLANE_SPECS = {
    # point, normal (SURVEY §8d order: floor, back, left, right, ceiling)
    "floor": ((0.0, -10.0, 0.0), (0.0, 1.0, 0.0), (0.9, 0.9, 0.9)),
    "back": ((0.0, 0.0, 15.0), (0.0, 0.0, -1.0), (0.7, 0.8, 0.9)),
    "left": ((-15.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.9, 0.3, 0.3)),
    "right": ((15.0, 0.0, 0.0), (-1.0, 0.0, 0.0), (0.3, 0.9, 0.3)),
    "ceiling": ((0.0, 15.0, 0.0), (0.0, -1.0, 0.0), (0.9, 0.9, 0.9)),
}
_PLANE_ORDER = ["floor", "back", "left", "right", "ceiling"]

_SPHERE_CONFIGS = {
    "c2": (1920, 1080, 16, 2, 1),
    "c3": (3840, 2160, 128, 4, 4),
    "c4": (7680, 4320, 256, 0, 8),
    "c5": (3840, 2160, 64, 0, 0),
}


def _random_sphere_scene(name: str, width: int, height: int, n_spheres: int, n_planes: int,
                         n_lights: int, aa: int) -> SceneData:
    rng = SplitMix64(0x5EED0000 + CONFIG_IDS[name])
    cam = Camera((0.0, 0.0, -25.0), width / 2.0, width, height, 0.0, 200.0, aa)
    sc = SceneData(cam, name=name)
    for _ in range(n_spheres):
        cx, cy, cz = rng.uniform(-12, 12), rng.uniform(-8, 8), rng.uniform(0, 14)
        r = rng.uniform(0.8, 2.3)
        col = (rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0))
        sc.add_sphere((cx, cy, cz), r, Material(col))
    for pname in _PLANE_ORDER[:n_planes]:
        p, n, col = _PLANE_SPECS[pname]
        sc.add_plane(p, n, Material(col))
    for _ in range(n_lights):
        x, y, z = rng.uniform(-8, 8), rng.uniform(8, 12), rng.uniform(-20, 0)
        sc.add_light((x, y, z), (1.0, 1.0, 1.0), 300.0 / n_lights)
    return sc


def reference_box(aa: int = 1) -> SceneData:
    """RaytracingEngine.cpp:223-290 without the model of :249-251 (box.obj is missing)."""
    cam = Camera((0.0, 0.0, -25.0), 500.0, 1000, 1000, 0.0, 200.0, aa)
    sc = SceneData(cam, name="c1")
    dirs = [(0, 0, -1), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0)]
    cols = [(1, 1, 1), (0, 1, 0), (0, 0, 1), (1, 1, 1), (1, 1, 1)]
    distance = 15.0
    for d, c in zip(dirs, cols):
        mat = Material(tuple(map(float, c)), shininess=0.128, specular=0.01, transparency=0.0,
                       refractive_index=1.5)
        # Plane(dir * -distance, dir, mat): Vec3 * double
        point = tuple(float(x) * -distance for x in d)
        sc.add_plane(point, tuple(map(float, d)), mat)
    sc.add_light((0.0, 0.0, -5.0), (1.0, 1.0, 1.0), 150.0)
    sc.add_light((-2.0, 2.0, -5.0), (1.0, 1.0, 1.0), 150.0)
    return sc


def mirror_scene(width=1920, height=1080, aa=1) -> SceneData:
    """Reflective spheres in a reflective box: exercises the depth-10 reflection chain."""
    rng = SplitMix64(0x5EED0000 + CONFIG_IDS["mirror"])
    cam = Camera((0.0, 0.0, -25.0), width / 2.0, width, height, 0.0, 200.0, aa)
    sc = SceneData(cam, name="mirror")
    for i in range(12):
        c = (rng.uniform(-10, 10), rng.uniform(-6, 6), rng.uniform(0, 12))
        r = rng.uniform(1.0, 2.5)
        col = (rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0))
        spec = [0.0, 0.3, 0.9][i % 3]
        sc.add_sphere(c, r, Material(col, shininess=rng.uniform(8, 256), specular=spec))
    for pname in _PLANE_ORDER:
        p, n, col = _PLANE_SPECS[pname]
        sc.add_plane(p, n, Material(col, shininess=32.0, specular=0.25))
    sc.add_light((0.0, 12.0, -10.0), (1.0, 1.0, 1.0), 200.0)
    sc.add_light((-6.0, 9.0, -15.0), (1.0, 0.9, 0.8), 120.0)
    return sc


def glass_scene(width=1920, height=1080, aa=1) -> SceneData:
    """Transparent spheres: refraction + Fresnel binary tree, partial shadow transmittance."""
    rng = SplitMix64(0x5EED0000 + CONFIG_IDS["glass"])
    cam = Camera((0.0, 0.0, -25.0), width / 2.0, width, height, 0.0, 200.0, aa)
    sc = SceneData(cam, name="glass")
    for i in range(10):
        c = (rng.uniform(-10, 10), rng.uniform(-6, 6), rng.uniform(0, 12))
        r = rng.uniform(1.0, 2.8)
        col = (rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0))
        tr = [0.0, 0.6, 0.95, 1.0, 0.3][i % 5]
        sc.add_sphere(c, r, Material(col, shininess=64.0, specular=0.2, transparency=tr,
                                     refractive_index=[1.5, 1.33, 2.4, 1.1, 1.5][i % 5]))
    for pname in ("floor", "back", "left"):
        p, n, col = _PLANE_SPECS[pname]
        sc.add_plane(p, n, Material(col, specular=0.1 if pname == "floor" else 0.0))
    sc.add_light((2.0, 11.0, -8.0), (1.0, 1.0, 1.0), 250.0)
    return sc


def _icosahedron(scale: float):
    t = (1.0 + math.sqrt(5.0)) / 2.0
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t),
         (0, 1, -t), (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    v = [tuple(c * scale for c in p) for p in v]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4),
         (11, 10, 2), (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8),
         (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    return [(v[a], v[b], v[c]) for a, b, c in f]


def mesh_scene(width=1920, height=1080, aa=1) -> SceneData:
    """Standalone triangles + two Models (translation-only transforms) + spheres + planes."""
    cam = Camera((0.0, 0.0, -25.0), width / 2.0, width, height, 0.0, 200.0, aa)
    sc = SceneData(cam, name="mesh")
    sc.add_sphere((6.0, -2.0, 6.0), 2.5, Material((0.9, 0.4, 0.2), specular=0.2, shininess=64.0))
    sc.add_sphere((-7.0, 3.0, 9.0), 1.5, Material((0.3, 0.5, 0.9)))
    for pname in ("floor", "back"):
        p, n, col = _PLANE_SPECS[pname]
        sc.add_plane(p, n, Material(col))
    # a quad of two standalone triangles, one with a translation
    sc.add_triangle((-12, -9, 4), (-4, -9, 4), (-4, -1, 8), Material((0.2, 0.8, 0.3)))
    sc.add_triangle((0, 0, 0), (8, 8, 4), (0, 8, 4), Material((0.8, 0.8, 0.2), specular=0.3),
                    translation=(-12.0, -9.0, 4.0))
    sc.add_model(_icosahedron(2.2), (0.0, 1.0, 5.0),
                 Material((0.0, 0.0, 1.0), shininess=128.0, specular=0.5, refractive_index=1.5))
    sc.add_model(_icosahedron(1.2), (-3.0, -6.5, 1.0), Material((0.9, 0.9, 0.9), specular=0.05))
    sc.add_light((0.0, 12.0, -10.0), (1.0, 1.0, 1.0), 250.0)
    sc.add_light((8.0, 6.0, -12.0), (1.0, 0.8, 0.6), 80.0)
    return sc


def _icosphere(radius: float, levels: int):
    """Icosahedron subdivided `levels` times (20·4^levels triangles), vertices on the sphere."""
    tris = _icosahedron(1.0)

    def norm(p):
        n = math.sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2])
        return (p[0] / n, p[1] / n, p[2] / n)

    tris = [tuple(norm(v) for v in t) for t in tris]
    for _ in range(levels):
        out = []
        for a, b, c in tris:
            ab = norm(tuple((x + y) / 2 for x, y in zip(a, b)))
            bc = norm(tuple((x + y) / 2 for x, y in zip(b, c)))
            ca = norm(tuple((x + y) / 2 for x, y in zip(c, a)))
            out += [(a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca)]
        tris = out
    return [tuple(tuple(radius * x for x in v) for v in t) for t in tris]


def _terrain(n: int, size: float, rng: SplitMix64):
    """n×n quads (2n² triangles) of a bumpy height field over [-size, size]²."""
    h = [[rng.uniform(-0.8, 0.8) for _ in range(n + 1)] for _ in range(n + 1)]
    def p(i, j):
        return (-size + 2 * size * i / n, h[i][j], -size + 2 * size * j / n)
    tris = []
    for i in range(n):
        for j in range(n):
            tris.append((p(i, j), p(i + 1, j), p(i + 1, j + 1)))
            tris.append((p(i, j), p(i + 1, j + 1), p(i, j + 1)))
    return tris


def bigmesh_scene(width=1920, height=1080, aa=1) -> SceneData:
    """Models at scale ('Models at scale need a BVH'): a 5120-triangle icosphere
    and a 3200-triangle terrain, plus spheres, a back plane and two lights; opaque, no
    specular, so it renders through the packet kernel with the triangle BVH."""
    rng = SplitMix64(0x5EED0000 + CONFIG_IDS["bigmesh"])
    cam = Camera((0.0, 0.0, -25.0), width / 2.0, width, height, 0.0, 200.0, aa)
    sc = SceneData(cam, name="bigmesh")
    sc.add_sphere((7.0, -3.0, 4.0), 2.0, Material((0.9, 0.4, 0.2)))
    sc.add_sphere((-9.0, 4.0, 8.0), 1.5, Material((0.3, 0.5, 0.9)))
    p, n, col = _PLANE_SPECS["back"]
    sc.add_plane(p, n, Material(col))
    sc.add_model(_icosphere(4.0, 4), (-3.0, 1.0, 6.0), Material((0.8, 0.8, 0.85)))
    sc.add_model(_terrain(40, 14.0, rng), (0.0, -9.0, 6.0), Material((0.4, 0.7, 0.3)))
    sc.add_light((0.0, 12.0, -10.0), (1.0, 1.0, 1.0), 250.0)
    sc.add_light((9.0, 7.0, -8.0), (1.0, 0.8, 0.6), 90.0)
    return sc


def make_config(name: str, width: int | None = None, height: int | None = None,
                aa: int = 1) -> SceneData:
    """Build a named scene at its BASELINE resolution (or at width×height)."""
    if name == "c1":
        sc = reference_box(aa)
    elif name in _SPHERE_CONFIGS:
        w, h, ns, npl, nl = _SPHERE_CONFIGS[name]
        sc = _random_sphere_scene(name, w, h, ns, npl, nl, aa)
        if name == "c5":
            sc.area_light = AreaLight((-3.0, 12.0, -8.0), (6.0, 0.0, 0.0), (0.0, 0.0, 6.0),
                                      (1.0, 1.0, 1.0), 300.0, 16)
    elif name == "mirror":
        sc = mirror_scene(aa=aa)
    elif name == "glass":
        sc = glass_scene(aa=aa)
    elif name == "mesh":
        sc = mesh_scene(aa=aa)
    elif name == "bigmesh":
        sc = bigmesh_scene(aa=aa)
    else:
        raise KeyError(f"unknown config {name!r}; known: {sorted(CONFIG_IDS)}")
    if width is not None:
        sc = sc.resized(width, height if height is not None else width, aa)
        sc.name = f"{name}_{width}x{sc.camera.height}"
    return sc
