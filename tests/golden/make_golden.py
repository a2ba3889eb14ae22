#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the UNMODIFIED reference renderer.

Runs only where /root/reference exists (it drives oracle/_ref/ref_harness, built by
oracle/Makefile from the reference sources where they lie).  Outputs are data only: inputs
and the reference's outputs for them.  The reference has no tests or fixtures of its own
(SURVEY.md §4), so these are the pins of the oracle.

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz / *.json
    python tests/golden/make_golden.py --full [name ...]  # full-size frames (FULL2_SCENES)
    python tests/golden/make_golden.py --oracle-full      # C5 (no reference semantics): oracle
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as po  # noqa: E402
from raytracingengine_amd.configs import make_config  # noqa: E402

SMALL = (96, 54)
SMALL_SCENES = ["c1", "c2", "c3", "c4", "mirror", "glass", "mesh"]
FULL_SCENES = ["c1", "c2"]  # full BASELINE resolution: sha256 + 1-in-64 subsample
SUBSAMPLE = 64


def scene_hash(sc) -> str:
    return hashlib.sha256(sc.to_text().encode()).hexdigest()


def run(mode, *args):
    subprocess.run([po.REF_HARNESS, mode, *map(str, args)], check=True, capture_output=True)


def kat_inputs(rng: np.random.Generator):
    n = 4096
    # spheres: ray origin, direction (not always unit), centre, radius
    o = rng.uniform(-20, 20, (n, 3))
    c = rng.uniform(-10, 10, (n, 3))
    toward = c - o + rng.normal(0, 3, (n, 3))
    d = toward * rng.choice([1.0, 1.0, 1.0, 0.25, 3.0], (n, 1))
    r = rng.uniform(0.1, 6, (n, 1))
    # special rows: origin inside, tangent-ish, pointing away, zero-length direction
    o[:64] = c[:64] + rng.uniform(-0.5, 0.5, (64, 3))
    r[:64] = 2.0
    d[64:128] = -toward[64:128]
    d[128:136] = 0.0
    sphere = np.concatenate([o, d, c, r], axis=1)

    # planes: ray, point, unnormalised normal (some parallel rays, some t==0 exactly)
    m = 2048
    po_ = rng.uniform(-20, 20, (m, 3))
    pd = rng.normal(0, 1, (m, 3))
    pp = rng.uniform(-10, 10, (m, 3))
    pn = rng.normal(0, 1, (m, 3)) * rng.choice([1.0, 5.0, 0.1], (m, 1))
    pd[:64] = np.cross(pn[:64], rng.normal(0, 1, (64, 3)))  # parallel to the plane
    po_[64:128] = pp[64:128]                                # origin on the plane: t == 0
    pn[128:136] = 0.0                                       # degenerate normal
    plane = np.concatenate([po_, pd, pp, pn], axis=1)

    # triangles: ray, v0, v1, v2, translation
    k = 2048
    tv = rng.uniform(-5, 5, (k, 9))
    tt = rng.uniform(-3, 3, (k, 3))
    centroid = (tv[:, 0:3] + tv[:, 3:6] + tv[:, 6:9]) / 3.0 + tt
    to = rng.uniform(-15, 15, (k, 3))
    td = centroid - to + rng.normal(0, 2.0, (k, 3))
    tv[:32, 6:9] = tv[:32, 0:3] + (tv[:32, 3:6] - tv[:32, 0:3]) * 2.0  # degenerate (collinear)
    tri = np.concatenate([to, td, tv, tt], axis=1)

    # getRay: pos, focal, W, H, x, y
    g = 512
    W = rng.integers(1, 4000, g)
    H = rng.integers(1, 3000, g)
    getray = np.stack([rng.uniform(-30, 30, g), rng.uniform(-30, 30, g), rng.uniform(-30, 30, g),
                       rng.uniform(0.5, 3000, g), W, H, rng.integers(0, W), rng.integers(0, H)],
                      axis=1).astype(np.float64)
    return {"sphere": sphere, "plane": plane, "triangle": tri, "getray": getray}


def tonemap_inputs(rng):
    n = 1024
    px = rng.exponential(1.0, (n, 3)) * rng.choice([0.01, 0.3, 1.0, 5.0, 40.0], (n, 1))
    px[:16] = 0.0                           # black: luminance operators give 0/0 -> NaN -> 0
    px[16:32] = rng.uniform(-1, 0, (16, 3))  # negative radiance
    px[32:48] = rng.uniform(0.99, 1.01, (16, 3))
    px[48:64] = 1e6
    px[64:80, 0] = 0.0                       # partial zeros
    # values that sit exactly on the x*255 truncation boundary
    px[80:336] = (np.arange(256)[:, None] / 255.0) * np.ones((1, 3))
    return px


REFAPP_NAMES = ["simple", "reinhard_simple", "reinhard_extended", "reinhard_extended_luminance",
                "reinhard_jodie", "uncharted2", "aces"]
REFAPP_BLOCK = 20


def ppm_blocks(path, block=REFAPP_BLOCK):
    """Mean of every block×block pixel block of a P6 file written by writePPM."""
    data = open(path, "rb").read()
    header = b"P6\n1000 1000\n255\n"
    assert data.startswith(header)
    img = np.frombuffer(data[len(header):], np.uint8).reshape(1000, 1000, 3).astype(np.float64)
    return img.reshape(1000 // block, block, 1000 // block, block, 3).mean(axis=(1, 3))


def refapp_golden():
    """Run the reference APPLICATION (its own main(), CPU renderer, AA=32) on tests/golden/box.obj
    and keep 20x20 block means of its seven PPMs (the AA jitter is unseeded, so a statistical pin)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "refapp"], check=True)
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_app_cpu")
    with tempfile.TemporaryDirectory() as td:
        import shutil
        shutil.copy(os.path.join(HERE, "box.obj"), td)
        res = subprocess.run([exe], cwd=td, capture_output=True, text=True)
        assert res.stdout.count("Image written") == 7, res.stdout
        blocks = np.stack([ppm_blocks(os.path.join(td, f"{n}.ppm")) for n in REFAPP_NAMES])
    np.savez_compressed(os.path.join(HERE, "refapp_blocks.npz"), blocks=blocks)
    print("refapp blocks", blocks.shape)


def main():
    if not po.ref_available():
        po.build()
    assert po.ref_available(), "oracle/_ref/ref_harness missing (needs /root/reference)"
    rng = np.random.default_rng(20260128)
    meta = {"generator": "tests/golden/make_golden.py", "reference": "Sorax5/RaytracingEngine",
            "reference_build": "oracle/Makefile (g++ -std=c++20 -O2 -fopenmp)", "scenes": {}}

    with tempfile.TemporaryDirectory() as td:
        # ---- whole-image renders at 96x54, AA=1 (deterministic in the reference)
        arrays = {}
        for name in SMALL_SCENES:
            sc = make_config(name, *SMALL)
            img, _, _ = po.ref_render(sc)
            arrays[name] = img
            meta["scenes"][f"{name}_small"] = {"scene_sha256": scene_hash(sc),
                                               "width": SMALL[0], "height": SMALL[1]}
        np.savez_compressed(os.path.join(HERE, "renders_small.npz"), **arrays)

        # ---- full-resolution renders: sha256 of the float64 image + a subsample
        full = {}
        for name in FULL_SCENES:
            sc = make_config(name)
            img, ms, thr = po.ref_render(sc)
            flat = img.reshape(-1, 3)
            full[name] = flat[::SUBSAMPLE]
            meta["scenes"][f"{name}_full"] = {
                "scene_sha256": scene_hash(sc), "width": sc.camera.width,
                "height": sc.camera.height, "image_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
                "subsample_stride": SUBSAMPLE}
        np.savez_compressed(os.path.join(HERE, "renders_full_subsample.npz"), **full)

        # ---- per-function known answers
        kats = kat_inputs(rng)
        kat_out = {}
        for kind, arr in kats.items():
            inp = os.path.join(td, f"{kind}.f64")
            out = os.path.join(td, f"{kind}.out")
            np.ascontiguousarray(arr, np.float64).tofile(inp)
            run("kat", kind, inp, len(arr), out)
            width = {"sphere": 2, "plane": 5, "triangle": 5, "getray": 6}[kind]
            kat_out[f"{kind}_in"] = arr
            kat_out[f"{kind}_out"] = np.fromfile(out, np.float64).reshape(len(arr), width)

        # IntersectClosest on the mesh scene (spheres, planes, triangles, models)
        sc = make_config("mesh", *SMALL)
        scene_path = os.path.join(td, "mesh.txt")
        sc.write(scene_path)
        nr = 1024
        ro = rng.uniform(-15, 15, (nr, 3))
        ro[:, 2] = rng.uniform(-25, -5, nr)
        rd = rng.uniform(-1, 1, (nr, 3))
        rd[:, 2] = np.abs(rd[:, 2]) + 0.2
        rays = np.concatenate([ro, rd], axis=1)
        rays.tofile(os.path.join(td, "rays.f64"))
        run("closest", scene_path, os.path.join(td, "rays.f64"), nr, os.path.join(td, "cl.out"))
        kat_out["closest_rays"] = rays
        kat_out["closest_out"] = np.fromfile(os.path.join(td, "cl.out"), np.float64).reshape(nr, 9)
        meta["closest_scene_sha256"] = scene_hash(sc)

        # tonemap operators: curves (pre-quantisation) and toColor bytes; tonemapAll + tonemap()
        px = tonemap_inputs(rng)
        px.tofile(os.path.join(td, "px.f64"))
        run("tonemap", os.path.join(td, "px.f64"), len(px), os.path.join(td, "tm.u8"))
        run("curves", os.path.join(td, "px.f64"), len(px), os.path.join(td, "cv.f64"))
        kat_out["tonemap_in"] = px
        kat_out["tonemap_bytes"] = np.fromfile(os.path.join(td, "tm.u8"), np.uint8).reshape(8, len(px), 3)
        kat_out["tonemap_curves"] = np.fromfile(os.path.join(td, "cv.f64"), np.float64).reshape(7, len(px), 3)

        # writePPM bytes of a 7x5 image
        raw = rng.integers(0, 256, (5, 7, 3), dtype=np.uint8)
        raw.tofile(os.path.join(td, "img.u8"))
        run("ppm", os.path.join(td, "img.u8"), 7, 5, os.path.join(td, "img.ppm"))
        kat_out["ppm_in"] = raw
        kat_out["ppm_bytes"] = np.frombuffer(open(os.path.join(td, "img.ppm"), "rb").read(), np.uint8)
        np.savez_compressed(os.path.join(HERE, "kats.npz"), **kat_out)

    with open(os.path.join(HERE, "golden_meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
    sizes = {f: os.path.getsize(os.path.join(HERE, f)) for f in os.listdir(HERE)
             if f.endswith((".npz", ".json"))}
    print(json.dumps(sizes))


# Full-size frames added in round 2 (``--full``): the BASELINE configs the bench and the scaling
# runs render, at their own resolution.  HDR: sha256 of the float64 image + a sparse subsample
# (diagnostics on a mismatch; configs whose shading calls libm pow are compared on the subsample
# within the pow tolerance).  LDR: sha256 of the bytes of tonemapAll() (7 operators) and
# tonemap() (ACES) of the reference, RaytracingEngine.cpp:113-135,165-214.
# Round 3 adds c1 (the reference main() scene: BASELINE config 1 is "ACES tonemap ->
# output.ppm", so its bytes are pinned for every operator too).
FULL2_SCENES = {"c1": 64, "c2": 64, "c3": 1024, "c4": 4096, "mirror": 256, "glass": 256,
                "mesh": 256}
LDR_NAMES = REFAPP_NAMES + ["tonemap_aces"]


def full_golden(names=None):
    """``--full [name ...]``: (re)generate the full-size reference frames of `names` (default:
    every FULL2_SCENES entry)."""
    if not po.ref_available():
        po.build()
    meta_path = os.path.join(HERE, "golden_meta.json")
    with open(meta_path) as fh:
        meta = json.load(fh)
    sub_path = os.path.join(HERE, "renders_full_subsample.npz")
    full = dict(np.load(sub_path))
    with tempfile.TemporaryDirectory() as td:
        for name, stride in FULL2_SCENES.items():
            if names and name not in names:
                continue
            sc = make_config(name)
            img, ms, thr = po.ref_render(sc)
            flat = np.ascontiguousarray(img.reshape(-1, 3))
            key = f"{name}_full"
            if name not in full or stride != SUBSAMPLE:
                full[name if stride == SUBSAMPLE else f"{name}_s{stride}"] = flat[::stride]
            entry = meta["scenes"].get(key, {})
            entry.update({"scene_sha256": scene_hash(sc), "width": sc.camera.width,
                          "height": sc.camera.height,
                          "image_sha256": hashlib.sha256(flat.tobytes()).hexdigest(),
                          "subsample_stride": stride})
            inp, out = os.path.join(td, "px.f64"), os.path.join(td, "px.u8")
            flat.tofile(inp)
            run("tonemap", inp, len(flat), out)
            ldr = np.fromfile(out, np.uint8).reshape(8, len(flat), 3)
            entry["ldr_sha256"] = {n: hashlib.sha256(ldr[i].tobytes()).hexdigest()
                                   for i, n in enumerate(LDR_NAMES)}
            meta["scenes"][key] = entry
            print(name, f"{ms[0]:.0f} ms on {thr} threads", entry["image_sha256"][:16], flush=True)
    np.savez_compressed(sub_path, **full)
    with open(meta_path, "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)


# BASELINE config 5 (the build-defined area light) has no reference semantics: its
# full frame is pinned by the ORACLE (itself pinned bit for bit to the reference on every other
# scene by tests/test_oracle_golden.py), and recorded as such ("source": "oracle").
ORACLE_FULL_SCENES = ["c5"]


def oracle_full_golden():
    meta_path = os.path.join(HERE, "golden_meta.json")
    with open(meta_path) as fh:
        meta = json.load(fh)
    for name in ORACLE_FULL_SCENES:
        sc = make_config(name)
        img, nt, ns = po.render(sc)
        flat = np.ascontiguousarray(img.reshape(-1, 3))
        meta["scenes"][f"{name}_full"] = {
            "source": "oracle", "scene_sha256": scene_hash(sc), "width": sc.camera.width,
            "height": sc.camera.height, "image_sha256": hashlib.sha256(flat.tobytes()).hexdigest(),
            "trace_rays": nt, "shadow_rays": ns,
            "ldr_sha256": {n: hashlib.sha256(po.tonemap(flat, i).tobytes()).hexdigest()
                           for i, n in enumerate(REFAPP_NAMES)}}
        print(name, "oracle", meta["scenes"][f"{name}_full"]["image_sha256"][:16], flush=True)
    with open(meta_path, "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)


def obj_golden():
    """The reference application's LoadObject (tinyobjloader) on the OBJ fixtures: triangles as
    9 doubles each (oracle/_ref/ref_harness obj)."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name in ("objtest", "box"):
            dst = os.path.join(td, name + ".f64")
            run("obj", os.path.join(HERE, name + ".obj"), dst)
            out[name] = np.fromfile(dst, np.float64).reshape(-1, 9)
    np.savez_compressed(os.path.join(HERE, "obj_tris.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    if "--refapp" in sys.argv:
        refapp_golden()
    elif "--obj" in sys.argv:
        obj_golden()
    elif "--full" in sys.argv:
        full_golden([a for a in sys.argv[1:] if not a.startswith("--")])
    elif "--oracle-full" in sys.argv:
        oracle_full_golden()
    else:
        main()
