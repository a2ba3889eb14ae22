"""AddressSanitizer + UndefinedBehaviorSanitizer run of the host code: the triangle
BVH builder (csrc/rt_bvh.cpp), the OBJ importer (api/rtamd/obj.cpp, the reference's LoadObject
RaytracingEngine.cpp:15-65), the scene-file parser (api/rtamd/scenefile.hpp) and the C oracle
(oracle/rt_oracle.c), built with g++/gcc -fsanitize=address,undefined and driven by
tests/sanitize/san_main.cpp on well-formed and malformed inputs.  CPU only (GPU sanitizers are
not available on the test pool; the device code is covered by the parity suite).
"""
import os
import subprocess

import numpy as np
import pytest

from raytracingengine_amd.configs import make_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def san(tmp_path_factory):
    d = tmp_path_factory.mktemp("san")
    inc = [f"-I{ROOT}/raytracingengine_amd/csrc", f"-I{ROOT}/include",
           f"-I{ROOT}/raytracingengine_amd/api", f"-I{ROOT}/oracle", "-I/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__"]
    oracle_o = str(d / "rt_oracle.o")
    subprocess.run(["gcc", "-std=c11", "-ffp-contract=off", "-fopenmp", *SAN,
                    f"-I{ROOT}/oracle", "-c", f"{ROOT}/oracle/rt_oracle.c", "-o", oracle_o],
                   check=True)
    exe = str(d / "san_main")
    subprocess.run(["g++", "-std=c++20", "-ffp-contract=off", "-fopenmp", *SAN, *inc,
                    f"{ROOT}/tests/sanitize/san_main.cpp",
                    f"{ROOT}/raytracingengine_amd/csrc/rt_bvh.cpp",
                    f"{ROOT}/raytracingengine_amd/api/rtamd/obj.cpp", oracle_o, "-o", exe, "-lm"],
                   check=True)
    return exe, d


def _run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, env=ENV,
                       timeout=300)
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def _tri_records(tris):
    """kTriStride records as rt_capi.cpp packs them: a0, e1, e2, unit normal."""
    v0, v1, v2, t = tris[:, 0:3], tris[:, 3:6], tris[:, 6:9], tris[:, 9:12]
    a0 = v0 + t
    n = np.cross(v1 - v0, v2 - v0)
    ln = np.linalg.norm(n, axis=1, keepdims=True)
    n = np.where(ln > 1e-12, n / np.where(ln > 0, ln, 1), 0.0)
    return np.concatenate([a0, (v1 + t) - a0, (v2 + t) - a0, n], axis=1)


@pytest.mark.parametrize("kind", ["random", "degenerate", "coincident", "one", "big"])
def test_bvh_builder(san, kind):
    exe, d = san
    rng = np.random.default_rng(hash(kind) % 2 ** 32)
    n = {"random": 500, "degenerate": 64, "coincident": 100, "one": 1, "big": 20000}[kind]
    tris = rng.uniform(-10, 10, (n, 12))
    if kind == "degenerate":  # collinear and zero-area triangles, zero-extent axes
        tris[:, 6:9] = tris[:, 0:3] + (tris[:, 3:6] - tris[:, 0:3]) * 2.0
        tris[:32, 2] = tris[:32, 5] = tris[:32, 8] = 0.0
    if kind == "coincident":  # every triangle identical (identical centroids)
        tris[:] = tris[0]
    rec = _tri_records(tris)
    path = d / f"tri_{kind}.bin"
    rec.astype(np.float64).tofile(path)
    out = _run(exe, "bvh", path, n)
    assert f"bvh {n} triangles" in out


@pytest.mark.parametrize("kind", ["random", "coincident", "nonfinite", "odd", "big"])
def test_sphere_chunk_builder(san, kind):
    """The packet kernel's spatial sphere chunks (rt_bvh.cpp build_sphere_chunks): a permutation
    and per-chunk bounding spheres that contain their members, under ASan/UBSan."""
    exe, d = san
    rng = np.random.default_rng(abs(hash(kind)) % 2 ** 32)
    n = {"random": 256, "coincident": 130, "nonfinite": 200, "odd": 65, "big": 5000}[kind]
    c = rng.uniform(-20, 20, (n, 3))
    r = rng.uniform(0.1, 3.0, n)
    if kind == "coincident":   # identical centres (ties in every split)
        c[:] = c[0]
    if kind == "nonfinite":    # NaN / inf centres and radii: their chunks are never culled
        c[5, 0] = np.nan
        c[77, 2] = np.inf
        r[150] = np.inf
    rec = np.concatenate([c, (r * r)[:, None]], axis=1).astype(np.float64)
    path = d / f"sph_{kind}.bin"
    rec.tofile(path)
    out = _run(exe, "chunks", path, n)
    assert f"chunks {n} spheres" in out


MALFORMED_OBJ = [
    "v 1 2 3\nv 4 5 6\nv 7 8 9\nf 1 2 3\n",
    "v 1 2 3\nf 1 2 3\n",                         # indices past the vertex list
    "v 1 2 3\nv 1 2\nf -1 -2 -3\nf 0 0 0\n",      # short vertex, relative and zero indices
    "f 1//2 3/4/5 6/7\nv .5 -e3 1e400\nv nan inf -inf\nf 1 2 3 4 5 6 7\n",
    "v " + " ".join(["1"] * 5000) + "\nf" + " 1" * 3000 + "\n",  # long lines, huge fan
    "# comment\r\nv 1 2 3\r\nv 2 3 4\r\nv 5 6 7\r\nf 1 2 3\r\n\t\n\nf\n",
    "",
]


@pytest.mark.parametrize("i", range(len(MALFORMED_OBJ)))
def test_obj_import(san, i):
    exe, d = san
    path = d / f"m{i}.obj"
    path.write_text(MALFORMED_OBJ[i])
    assert "obj" in _run(exe, "obj", path)


def test_obj_fixtures_and_missing_file(san):
    exe, d = san
    for name in ("objtest.obj", "box.obj"):
        assert "triangles" in _run(exe, "obj", os.path.join(ROOT, "tests", "golden", name))
    assert "obj error" in _run(exe, "obj", d / "does_not_exist.obj")


@pytest.mark.parametrize("name", ["c1", "c2", "c5", "glass", "mesh"])
def test_scene_file_parser(san, name):
    exe, d = san
    sc = make_config(name, 32, 18)
    path = d / f"{name}.txt"
    sc.write(str(path))
    out = _run(exe, "scene", path)
    assert f"scene {len(sc.spheres)} spheres {len(sc.planes)} planes" in out


@pytest.mark.parametrize("text", [
    "camera 0 0 -25 500 16 9 0 200 1\nsphere 0 0 0\n",            # truncated record
    "camera x y z\n", "bogus 1 2 3\n", "model 3 0 0 0 1 1 1 128 0 0 1\nv 1 2 3\n", ""])
def test_scene_file_parser_malformed(san, text):
    exe, d = san
    path = d / f"bad_{abs(hash(text))}.txt"
    path.write_text(text)
    assert "scene" in _run(exe, "scene", path)


@pytest.mark.parametrize("name", ["c1", "c3", "c5", "mirror", "glass", "mesh", "bigmesh"])
def test_oracle_under_sanitizers(san, oracle, name):
    """The C oracle's render, tonemaps and per-function entry points; the sanitized build's rows
    are the regular build's (tests/test_oracle_golden.py pins those to the reference)."""
    exe, d = san
    sc = make_config(name, 48, 27)
    sd = d / f"o_{name}"
    sd.mkdir(exist_ok=True)
    for fname, arr in (("spheres", sc.sphere_array()), ("planes", sc.plane_array()),
                       ("triangles", sc.triangle_array()), ("lights", sc.light_array()),
                       ("camera", sc.camera.to_struct())):
        np.ascontiguousarray(arr).tofile(sd / f"{fname}.bin")
    if sc.area_light is not None:
        sc.area_light.to_struct().tofile(sd / "area.bin")
    rows = 9 if name != "bigmesh" else 3
    _run(exe, "oracle", sd, rows)
    got = np.fromfile(sd / "out.f64", np.float64).reshape(rows, 48, 3)
    ref, _, _ = oracle.render(sc, rows=(0, rows))
    assert np.array_equal(got, ref)
