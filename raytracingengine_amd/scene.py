"""Scene data shared by the bench, the tests and the C-ABI bindings.

The numpy dtypes below have exactly the byte layout of the C structs in ``include/rt_capi.h``
(``rt_sphere``, ``rt_plane``, ``rt_triangle``, ``rt_light``, ``rt_camera``, ``rt_area_light``), so
one set of host buffers feeds the HIP library, the C oracle and the scene-file writer.

Semantics follow the reference constructors (paths relative to
``/root/reference/RaytracingEngine``):

* ``Material`` defaults (Shape.h:13-19): shininess 128, specular 0, transparency 0, ior 1.
* ``Plane`` normalizes its normal in the constructor (Shape.h:141-142) — :func:`vec_normalize`
  reproduces ``Vec3::normalize`` (Math.h:31-37) bit for bit with IEEE doubles.
* ``Camera(position, focal, width, height, near, far)`` with ``antiAliasingAmount`` (Math.h:85-97).
* ``Model`` (Shape.h:248-307) is flattened into triangles carrying the model material and
  translation, appended after the standalone triangles (IntersectClosest order, Scene.h:243-254).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np

MATERIAL_DTYPE = np.dtype(
    [
        ("color", "<f8", (3,)),
        ("shininess", "<f8"),
        ("specular", "<f8"),
        ("transparency", "<f8"),
        ("refractive_index", "<f8"),
    ]
)
SPHERE_DTYPE = np.dtype([("center", "<f8", (3,)), ("radius", "<f8"), ("material", MATERIAL_DTYPE)])
PLANE_DTYPE = np.dtype([("point", "<f8", (3,)), ("normal", "<f8", (3,)), ("material", MATERIAL_DTYPE)])
TRIANGLE_DTYPE = np.dtype(
    [
        ("v0", "<f8", (3,)),
        ("v1", "<f8", (3,)),
        ("v2", "<f8", (3,)),
        ("translation", "<f8", (3,)),
        ("material", MATERIAL_DTYPE),
    ]
)
LIGHT_DTYPE = np.dtype([("position", "<f8", (3,)), ("color", "<f8", (3,)), ("intensity", "<f8")])
CAMERA_DTYPE = np.dtype(
    [
        ("position", "<f8", (3,)),
        ("focal", "<f8"),
        ("width", "<u4"),
        ("height", "<u4"),
        ("aa_samples", "<i4"),
        ("_pad0", "<i4"),
        ("near_plane", "<f8"),
        ("far_plane", "<f8"),
    ]
)
AREA_LIGHT_DTYPE = np.dtype(
    [
        ("corner", "<f8", (3,)),
        ("edge_u", "<f8", (3,)),
        ("edge_v", "<f8", (3,)),
        ("color", "<f8", (3,)),
        ("intensity", "<f8"),
        ("samples", "<i4"),
        ("_pad0", "<i4"),
    ]
)

assert SPHERE_DTYPE.itemsize == 88 and PLANE_DTYPE.itemsize == 104
assert TRIANGLE_DTYPE.itemsize == 152 and LIGHT_DTYPE.itemsize == 56
assert CAMERA_DTYPE.itemsize == 64 and AREA_LIGHT_DTYPE.itemsize == 112


def vec_normalize(v: Sequence[float]) -> tuple[float, float, float]:
    """``Vec3::normalize`` (Math.h:31-37): 0 if length <= 1e-12, else per-component division."""
    x, y, z = float(v[0]), float(v[1]), float(v[2])
    length = math.sqrt(x * x + y * y + z * z)
    if length <= 1e-12:
        return (0.0, 0.0, 0.0)
    return (x / length, y / length, z / length)


@dataclass
class Material:
    color: tuple[float, float, float] = (0.0, 0.0, 0.0)
    shininess: float = 128.0
    specular: float = 0.0
    transparency: float = 0.0
    refractive_index: float = 1.0

    def as_tuple(self):
        return (tuple(self.color), self.shininess, self.specular, self.transparency, self.refractive_index)


@dataclass
class Camera:
    position: tuple[float, float, float]
    focal: float = 1.0
    width: int = 800
    height: int = 600
    near_plane: float = 1.0
    far_plane: float = 1000.0
    antiAliasingAmount: int = 32  # reference default, Math.h:94

    def to_struct(self) -> np.ndarray:
        a = np.zeros(1, CAMERA_DTYPE)
        a["position"][0] = self.position
        a["focal"] = self.focal
        a["width"] = self.width
        a["height"] = self.height
        a["aa_samples"] = self.antiAliasingAmount
        a["near_plane"] = self.near_plane
        a["far_plane"] = self.far_plane
        return a


@dataclass
class AreaLight:
    """Build-defined parallelogram emitter (BASELINE config 5); no reference semantics."""

    corner: tuple[float, float, float]
    edge_u: tuple[float, float, float]
    edge_v: tuple[float, float, float]
    color: tuple[float, float, float] = (1.0, 1.0, 1.0)
    intensity: float = 300.0
    samples: int = 16

    def to_struct(self) -> np.ndarray:
        k = int(round(math.sqrt(self.samples)))
        if k * k != self.samples:
            raise ValueError("area light samples must be a perfect square")
        a = np.zeros(1, AREA_LIGHT_DTYPE)
        a["corner"][0] = self.corner
        a["edge_u"][0] = self.edge_u
        a["edge_v"][0] = self.edge_v
        a["color"][0] = self.color
        a["intensity"] = self.intensity
        a["samples"] = self.samples
        return a


@dataclass
class SceneData:
    """A flattened scene: the order of each list is the reference's insertion order."""

    camera: Camera
    spheres: list = field(default_factory=list)    # (center, radius, Material)
    planes: list = field(default_factory=list)     # (point, unnormalized normal, Material)
    triangles: list = field(default_factory=list)  # (v0, v1, v2, translation, Material)
    models: list = field(default_factory=list)     # (list[(v0,v1,v2)], translation, Material)
    lights: list = field(default_factory=list)     # (position, color, intensity)
    area_light: AreaLight | None = None
    name: str = "scene"

    # ---------------------------------------------------------------- builders
    def add_sphere(self, center, radius, mat: Material):
        self.spheres.append((tuple(map(float, center)), float(radius), mat))

    def add_plane(self, point, normal, mat: Material):
        self.planes.append((tuple(map(float, point)), tuple(map(float, normal)), mat))

    def add_triangle(self, v0, v1, v2, mat: Material, translation=(0.0, 0.0, 0.0)):
        self.triangles.append((tuple(v0), tuple(v1), tuple(v2), tuple(translation), mat))

    def add_obj(self, path: str, translation=(0.0, 0.0, 0.0), mat: Material | None = None):
        """A Model from a Wavefront OBJ file, as the reference application's LoadObject
        (RaytracingEngine.cpp:15-65) builds it: see load_obj."""
        self.add_model(load_obj(path), translation, mat if mat is not None else Material())

    def add_model(self, tris: Iterable, translation, mat: Material):
        self.models.append(([tuple(map(tuple, t)) for t in tris], tuple(translation), mat))

    def add_light(self, position, color, intensity):
        self.lights.append((tuple(map(float, position)), tuple(map(float, color)), float(intensity)))

    # ---------------------------------------------------------------- flattened arrays
    def sphere_array(self) -> np.ndarray:
        a = np.zeros(len(self.spheres), SPHERE_DTYPE)
        for i, (c, r, m) in enumerate(self.spheres):
            a[i] = (c, r, m.as_tuple())
        return a

    def plane_array(self) -> np.ndarray:
        a = np.zeros(len(self.planes), PLANE_DTYPE)
        for i, (p, n, m) in enumerate(self.planes):
            a[i] = (p, vec_normalize(n), m.as_tuple())
        return a

    def triangle_array(self) -> np.ndarray:
        rows = [(v0, v1, v2, t, m.as_tuple()) for (v0, v1, v2, t, m) in self.triangles]
        for tris, t, m in self.models:
            rows.extend((v0, v1, v2, t, m.as_tuple()) for (v0, v1, v2) in tris)
        a = np.zeros(len(rows), TRIANGLE_DTYPE)
        for i, r in enumerate(rows):
            a[i] = r
        return a

    def light_array(self) -> np.ndarray:
        a = np.zeros(len(self.lights), LIGHT_DTYPE)
        for i, (p, c, s) in enumerate(self.lights):
            a[i] = (p, c, s)
        return a

    def resized(self, width: int, height: int, aa: int | None = None) -> "SceneData":
        """Same geometry, new resolution; focal = width/2 keeps the 90-degree horizontal FOV."""
        cam = Camera(
            self.camera.position,
            width / 2.0 if self.camera.focal == self.camera.width / 2.0 else self.camera.focal,
            width,
            height,
            self.camera.near_plane,
            self.camera.far_plane,
            self.camera.antiAliasingAmount if aa is None else aa,
        )
        return SceneData(cam, list(self.spheres), list(self.planes), list(self.triangles),
                         list(self.models), list(self.lights), self.area_light,
                         f"{self.name}_{width}x{height}")

    # ---------------------------------------------------------------- scene file
    def to_text(self) -> str:
        """Scene-file text read by oracle/_ref (ref_harness.cpp load_scene).  Doubles are
        written with repr() so they round-trip exactly."""

        def f(x):
            return repr(float(x))

        def vec(v):
            return " ".join(f(c) for c in v)

        def mat(m: Material):
            return " ".join(f(x) for x in (*m.color, m.shininess, m.specular, m.transparency,
                                            m.refractive_index))

        c = self.camera
        out = ["rtscene 1",
               f"camera {vec(c.position)} {f(c.focal)} {c.width} {c.height} {f(c.near_plane)} "
               f"{f(c.far_plane)} {c.antiAliasingAmount}"]
        for ctr, r, m in self.spheres:
            out.append(f"sphere {vec(ctr)} {f(r)} {mat(m)}")
        for p, n, m in self.planes:
            out.append(f"plane {vec(p)} {vec(n)} {mat(m)}")
        for v0, v1, v2, t, m in self.triangles:
            out.append(f"triangle {vec(v0)} {vec(v1)} {vec(v2)} {vec(t)} {mat(m)}")
        for tris, t, m in self.models:
            out.append(f"model {len(tris)} {vec(t)} {mat(m)}")
            for v0, v1, v2 in tris:
                out.append(f"v {vec(v0)} {vec(v1)} {vec(v2)}")
        for p, col, s in self.lights:
            out.append(f"light {vec(p)} {vec(col)} {f(s)}")
        out.append("end")
        return "\n".join(out) + "\n"

    def write(self, path) -> None:
        with open(path, "w") as fh:
            fh.write(self.to_text())


def tinyobj_real(s: str, fallback: float) -> float:
    """A real as tinyobjloader v1.0.x reads it — the same restatement as tinyobj_real in
    api/rtamd/obj.cpp (not correctly rounded; ".5" reads as the fallback)."""
    lut = [1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001]
    i, n = 0, len(s)
    if n == 0:
        return fallback
    sign = "+"
    if s[0] in "+-":
        sign = s[0]
        i = 1
    elif not s[0].isdigit():
        return fallback
    mantissa = 0.0
    digits = 0
    while i < n and s[i].isdigit():
        mantissa *= 10
        mantissa += int(s[i])
        i += 1
        digits += 1
    if digits == 0:
        return fallback
    exponent = 0
    if i < n and s[i] == ".":
        i += 1
        k = 1
        while i < n and s[i].isdigit():
            mantissa += int(s[i]) * (lut[k] if k < 8 else math.pow(10.0, -k))
            k += 1
            i += 1
    if i < n and s[i] in "eE":
        i += 1
        esign = "+"
        if i < n and s[i] in "+-":
            esign = s[i]
            i += 1
        elif not (i < n and s[i].isdigit()):
            return fallback
        ed = 0
        while i < n and s[i].isdigit():
            exponent = exponent * 10 + int(s[i])
            i += 1
            ed += 1
        if ed == 0:
            return fallback
        if esign == "-":
            exponent = -exponent
    val = math.ldexp(mantissa * math.pow(5.0, exponent), exponent) if exponent else mantissa
    return val if sign == "+" else -val


def load_obj(path: str) -> list[tuple[tuple[float, float, float], ...]]:
    """Triangles of a Wavefront OBJ file as tinyobjloader v1.0.x (triangulate on) and the
    reference's LoadObject produce them: `v` positions rounded to float32 (tinyobj's real_t) then
    widened, `f` corners `i`, `i/t`, `i//n`, `i/t/n` (1-based; 0 read as 0; negative relative to
    the vertices read so far) fanned from the first corner, faces in file order.  Same rules as
    the C++ rtamd::LoadObject (api/rtamd/obj.cpp)."""
    pos: list[tuple[float, float, float]] = []
    tris = []

    def atoi(tok: str) -> int:
        digits = ""
        for i, ch in enumerate(tok):
            if ch.isdigit() or (i == 0 and ch in "+-"):
                digits += ch
            else:
                break
        try:
            return int(digits)
        except ValueError:
            return 0

    def f32(tok: str) -> float:
        return float(np.float32(tinyobj_real(tok, 0.0)))

    with open(path) as fh:
        for line in fh:
            parts = line.split()
            if not parts:
                continue
            if parts[0] == "v":
                xyz = (parts[1:4] + ["0", "0", "0"])[:3]
                pos.append(tuple(f32(t) for t in xyz))
            elif parts[0] == "f":
                face = []
                for tok in parts[1:]:
                    i = atoi(tok)
                    i = i - 1 if i > 0 else (0 if i == 0 else len(pos) + i)
                    if not 0 <= i < len(pos):
                        raise ValueError(f"OBJ face index out of range in {path}")
                    face.append(i)
                for k in range(2, len(face)):
                    tris.append((pos[face[0]], pos[face[k - 1]], pos[face[k]]))
    return tris
