"""GPU parity: the HIP path (through the C-ABI) against the oracle and the reference goldens.

Bars (north star: per-channel |Δ| < 1e-4 before tonemap, byte-identical PPM where that holds):
  * scenes whose shading calls no libm pow/log (C2–C5 synthetic configs) — bit-exact;
  * scenes with Blinn-Phong / Fresnel pow (C1 box, mirror, glass, mesh) — |Δ| ≤ 1e-12 here
    (device pow is ≤ 1 ulp from glibc), far inside the 1e-4 north-star tolerance;
  * LDR bytes — identical wherever the HDR is identical;
  * full BASELINE sizes — size-independent properties: SHA-256 of the reference C2 frame,
    row-tile == full-frame bytes, determinism, exact ray counts, oracle spot rows.
"""
import hashlib

import numpy as np
import pytest

from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
from raytracingengine_amd.scene import Camera, Material, SceneData

pytestmark = pytest.mark.gpu

SMALL = (96, 54)
POW_TOL = 1e-12
NORTH_STAR_TOL = 1e-4
EXACT = {"c2", "c3", "c4", "c5"}


def _render(ctx, sc, **kw):
    ds = ctx.scene(sc)
    try:
        return ds.render(**kw)
    finally:
        ds.close()


def test_device_libm(ctx):
    """Division and sqrt are correctly rounded on gfx950 (the basis of bit-exactness);
    pow/log are within 1 ulp of glibc."""
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(1e-6, 1e3, 20000), rng.uniform(0, 1, 5000)])
    y = np.concatenate([rng.uniform(0.05, 300, 20000), rng.uniform(0.01, 5, 5000)])
    out = ctx.debug_f64_ops(x, y)
    assert np.array_equal(out[:, 0], x / y)
    assert np.array_equal(out[:, 1], np.sqrt(x))
    p = np.power(x, y)
    ok = np.isfinite(p) & (p > 0)
    assert np.all(np.abs(out[ok, 2] - p[ok]) <= np.spacing(p[ok]))
    lg = np.log(x)
    assert np.all(np.abs(out[:, 3] - lg) <= np.spacing(np.abs(lg)))


def test_blinn_phong_pow_accuracy(ctx):
    """pow_bp (rt_device.hpp), the Blinn-Phong pow(N·H, shininess) of every trace kernel: within
    2.5e-16 absolute of libm pow on (0, 1] x [0, 4096] (results in [0, 1]), and the libm value
    itself outside its fast domain."""
    rng = np.random.default_rng(5)
    n = 200000
    x = np.concatenate([rng.uniform(0, 1, n), np.exp2(rng.uniform(-1074, 0, n)),
                        1.0 - rng.uniform(0, 1e-6, n), [1.0, 1.0 + 2 ** -52, 5e-324, 0.5]])
    y = np.concatenate([rng.uniform(0, 300, n), rng.uniform(0, 4096, n), rng.uniform(0, 1, n),
                        [0.128, 128.0, 0.5, 0.0]])
    y[::7] = 0.128  # the reference scene's shininess
    out = ctx.debug_f64_ops(x, y)
    with np.errstate(all="ignore"):
        ref = np.power(x, y)
    assert np.all(np.abs(out[:, 4] - ref) <= 2.5e-16), np.abs(out[:, 4] - ref).max()
    odd_x = np.array([2.0, 0.0, -0.5, np.inf, np.nan, 0.3, 0.3, 0.3])
    odd_y = np.array([3.0, 2.0, 2.0, 1.0, 1.0, np.nan, np.inf, -1e300])
    odd = ctx.debug_f64_ops(odd_x, odd_y)
    assert _same_bits(odd[:, 4], odd[:, 2])  # out of its domain: the libm pow


def _same_bits(a, b):
    """Bitwise equality (signed zeros distinguished), any NaN equal to any NaN."""
    nan = np.isnan(a) & np.isnan(b)
    return np.array_equal(a.view(np.int64)[~nan], b.view(np.int64)[~nan]) and \
        np.array_equal(np.isnan(a), np.isnan(b))


def _edge_inputs():
    rng = np.random.default_rng(11)
    n = 60000
    # log-uniform magnitudes over the whole binary64 range (denormals included), random signs
    mag = lambda k: np.exp2(rng.uniform(-1074, 1023, k)) * rng.choice([-1.0, 1.0], k)
    x, y = mag(n), mag(n)
    # realistic operands: what the trace divides and takes roots of
    x = np.concatenate([x, rng.uniform(-1e4, 1e4, n), rng.uniform(0, 1e6, n)])
    y = np.concatenate([y, rng.uniform(-1e4, 1e4, n), rng.uniform(1e-6, 1e3, n)])
    # near 1 (normalising unit vectors)
    k = np.concatenate([np.arange(0, 5000), rng.integers(0, 1 << 26, 20000),
                        (1 << 22) + np.arange(-64, 64)]).astype(np.int64)
    one = np.float64(1.0).view(np.int64)
    near = np.concatenate([(one + k).view(np.float64), (one - k).view(np.float64)])
    x = np.concatenate([x, near])
    y = np.concatenate([y, rng.uniform(0.5, 2.0, near.size)])
    # scaling thresholds of the division/sqrt sequences and IEEE specials
    edges = np.array([2.0 ** e * f for e in (-1074, -1023, -1022, -767, -700, -301, -300, -299,
                                             299, 300, 301, 700, 1023)
                      for f in (1.0, 1.0 - 2 ** -53, 1.0 + 2 ** -52, 1.5)])
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 5e-324, -5e-324,
                        np.finfo(np.float64).max, np.finfo(np.float64).tiny])
    ex = np.concatenate([edges, -edges, special])
    gx, gy = np.meshgrid(ex, ex)
    x = np.concatenate([x, gx.ravel()])
    y = np.concatenate([y, gy.ravel()])
    return x, y


def test_device_div_sqrt_edge_cases(ctx):
    """Device double division and sqrt give IEEE correctly rounded bits (numpy's) over the whole
    binary64 range: zeros of both signs, denormals, infinities, NaN, near-1 operands."""
    x, y = _edge_inputs()
    with np.errstate(all="ignore"):
        out = ctx.debug_f64_ops(x, y)
        assert _same_bits(out[:, 0], x / y)
        assert _same_bits(out[:, 1], np.sqrt(x))


def _vec_inputs():
    rng = np.random.default_rng(23)
    n = 40000
    mag = lambda k: np.exp2(rng.uniform(-1074, 1023, k)) * rng.choice([-1.0, 1.0], k)
    vs = [mag(3 * n).reshape(-1, 3),                                   # every binary64 range
          rng.uniform(-50, 50, (n, 3)),                                # scene-scale vectors
          rng.uniform(-1, 1, (n, 3)) * np.exp2(rng.uniform(-45, 65, (n, 1))),  # around the gates
          rng.normal(size=(n, 3))]
    u = rng.normal(size=(n, 3))
    vs.append(u / np.sqrt((u * u).sum(1, keepdims=True)))             # unit: the 2nd normalize
    # components at the numerator gate (2^-900) and zero / negative zero components
    g = rng.uniform(-1, 1, (n, 3))
    g[:, 0] = np.exp2(rng.uniform(-905, -895, n)) * rng.choice([-1.0, 1.0], n)
    g[: n // 4, 1] = 0.0
    g[n // 4: n // 2, 2] = -0.0
    vs.append(g)
    # length^2 exactly at the gates 2^-78 and 2^120, and axis-aligned unit vectors
    vs.append(np.array([[2.0 ** -39, 0.0, 0.0], [2.0 ** 60, 0.0, 0.0],
                        [2.0 ** -39.5, 2.0 ** -39.5, 1e-300], [1.0, 0.0, 0.0], [0.0, -1.0, 0.0],
                        [0.6, 0.8, 0.0], [3.0, 4.0, 12.0], [0.0, 0.0, 0.0],
                        [np.inf, 1.0, 1.0], [np.nan, 1.0, 1.0], [1e-12, 0.0, 0.0],
                        [1e-12 * (1 + 2 ** -52), 0.0, 0.0], [5e-324, 0.0, 0.0]]))
    return np.concatenate(vs)


def test_fast_exact_cores(ctx):
    """The sqrt / division cores (rt_device.hpp: unit(), light_dir()) return the same bits as the
    compiler's correctly rounded lowering for every input (the cores run only inside their
    ranges, the exact lowering outside), and both equal numpy's IEEE results."""
    v = _vec_inputs()
    with np.errstate(all="ignore"):
        out = ctx.debug_vec_ops(v)
        assert _same_bits(out[:, 0:3], out[:, 3:6])        # unit == unit_exact
        ok = out[:, 6] > 0                                  # light_dir vs exact where dist > 0
        assert _same_bits(out[:, 6], out[:, 11])
        assert _same_bits(out[ok, 7:11], out[ok, 12:16])
        # numpy: Vec3::length / normalize (Math.h:27-37)
        dist = np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2])
        assert _same_bits(out[:, 6], dist)
        assert _same_bits(out[ok, 7:10], v[ok] / dist[ok, None])
        assert _same_bits(out[ok, 10], 1.0 / (dist[ok] * dist[ok]))
        ref = np.where((dist <= 1e-12)[:, None], 0.0,
                       np.where((dist == 1.0)[:, None], v, v / dist[:, None]))
        assert _same_bits(out[:, 0:3], ref)


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4", "mirror", "glass", "mesh"])
def test_small_scenes_vs_reference_golden(ctx, golden, name):
    sc = make_config(name, *SMALL)
    out = _render(ctx, sc, hdr64=True, tonemap=1)
    ref = golden["small"][name]
    d = np.abs(out["hdr64"] - ref).max()
    if name in EXACT:
        assert np.array_equal(out["hdr64"], ref), d
    assert d <= POW_TOL, d
    assert d < NORTH_STAR_TOL


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4", "c5", "mirror", "glass", "mesh"])
def test_small_scenes_vs_oracle_counts_and_ldr(ctx, oracle, name):
    sc = make_config(name, *SMALL)
    out = _render(ctx, sc, hdr64=True, hdr32=True, tonemap=1, stats=True)
    ref, nt, ns = oracle.render(sc)
    assert out["trace_rays"] == nt and out["shadow_rays"] == ns
    assert np.abs(out["hdr64"] - ref).max() <= POW_TOL
    assert np.array_equal(out["hdr32"], out["hdr64"].astype(np.float32))
    same = np.all(out["hdr64"] == ref, axis=-1)
    ldr_ref = oracle.tonemap(ref, 1).reshape(out["ldr"].shape)
    assert np.array_equal(out["ldr"][same], ldr_ref[same])


def test_full_c2_sha256_matches_reference(ctx, golden):
    """The whole 1920×1080 C2 frame is bit-identical to the unmodified reference."""
    sc = make_config("c2")
    out = _render(ctx, sc, hdr64=True, stats=True)
    info = golden["meta"]["scenes"]["c2_full"]
    assert hashlib.sha256(out["hdr64"].tobytes()).hexdigest() == info["image_sha256"]
    assert out["trace_rays"] == 1920 * 1080


@pytest.mark.parametrize("name", ["c2", "mirror"])
def test_row_tiles_equal_full_frame(ctx, name):
    """Row tiles (the multi-GPU split) reassemble to the full frame byte for byte."""
    sc = make_config(name, 320, 200)
    ds = ctx.scene(sc)
    try:
        full = ds.render(hdr64=True, tonemap=6)
        cuts = [0, 37, 64, 150, 199, 200]
        tiles = [ds.render(hdr64=True, tonemap=6, row_begin=a, row_end=b)
                 for a, b in zip(cuts[:-1], cuts[1:])]
    finally:
        ds.close()
    assert np.array_equal(np.concatenate([t["hdr64"] for t in tiles]), full["hdr64"])
    assert np.array_equal(np.concatenate([t["ldr"] for t in tiles]), full["ldr"])


@pytest.mark.parametrize("name,world,block", [("c2", 3, 16), ("c3", 8, 16), ("glass", 4, 5),
                                              ("mirror", 2, 7), ("mesh", 8, 1)])
def test_block_cyclic_rows_equal_full_frame(ctx, name, world, block):
    """Block-cyclic row sets (row_block / row_cycle, the balanced multi-GPU split): each rank's
    single launch returns exactly its rows of the full frame, on every kernel path (packet,
    chain, wavefront tree)."""
    from raytracingengine_amd.distributed import plan_rows, render_opts_for, row_ranges
    sc = make_config(name, 200, 123)
    H = sc.camera.height
    ds = ctx.scene(sc)
    try:
        full = ds.render(hdr64=True, tonemap=6)
        frame = np.full_like(full["hdr64"], np.nan)
        for r in range(world):
            ranges = row_ranges(r, world, H, block)
            out = ds.render(hdr64=True, tonemap=6,
                            opts=render_opts_for(ranges, r, world, H, block, tonemap=6))
            assert out["hdr64"].shape[0] == plan_rows(ranges)
            k = 0
            for a, b in ranges:
                frame[a:b] = out["hdr64"][k:k + b - a]
                assert np.array_equal(out["ldr"][k:k + b - a], full["ldr"][a:b])
                k += b - a
    finally:
        ds.close()
    assert np.array_equal(frame, full["hdr64"])


def test_deterministic(ctx):
    sc = make_config("c3", 640, 360)
    a = _render(ctx, sc, hdr64=True)
    b = _render(ctx, sc, hdr64=True)
    assert np.array_equal(a["hdr64"], b["hdr64"])


@pytest.mark.parametrize("name,aa", [("c2", 4), ("mirror", 3), ("glass", 2), ("c1", 4)])
def test_antialiasing_vs_oracle(ctx, oracle, name, aa):
    """AA>1 uses the build-defined counter RNG (the reference's is unseeded); same RNG on
    both sides gives identical jitter."""
    sc = make_config(name, *SMALL, aa=aa)
    out = _render(ctx, sc, hdr64=True, seed=1234)
    ref, _, _ = oracle.render(sc, seed=1234)
    assert np.abs(out["hdr64"] - ref).max() <= POW_TOL


def test_area_light_c5_vs_oracle(ctx, oracle):
    sc = make_config("c5", 160, 90)
    out = _render(ctx, sc, hdr64=True, stats=True, seed=99)
    ref, nt, ns = oracle.render(sc, seed=99)
    assert np.array_equal(out["hdr64"], ref)
    assert out["shadow_rays"] == ns


def test_tonemap_kernel_vs_reference_bytes(ctx, golden):
    k = golden["kats"]
    allops = ctx.tonemap(k["tonemap_in"], capi.TONEMAP_ALL)
    for op in range(7):
        single = ctx.tonemap(k["tonemap_in"], op)
        assert np.array_equal(single, allops[op])
        if op == 4:  # Reinhard-Jodie uses log/pow: allow rare 1-ulp truncation flips
            assert (single != k["tonemap_bytes"][op]).sum() <= 3
        else:
            assert np.array_equal(single, k["tonemap_bytes"][op]), capi.TONEMAPS[op]


def test_reinhard_truncation_boundaries(ctx, oracle):
    """Reinhard-simple bytes at the truncation boundaries: inputs on and within a few ulps /
    1e-9..3e-3 of every c = k/(255-k) (where RN(c/(c+1))*255 crosses an integer), plus zeros,
    NaN/inf, negatives, tiny and huge values, give the reference's bytes (the bench's LDR).
    The kernel decides most bytes from an FP32 estimate (rt_device.hpp reinhard_byte, the packet
    kernel's fused path too) and falls back to FP64 within 5e-4 of a byte boundary."""
    rng = np.random.default_rng(11)
    k = np.arange(256, dtype=np.float64)
    with np.errstate(divide="ignore"):
        base = k / (255.0 - k)
    base = base[np.isfinite(base)]
    vals = [base, np.nextafter(base, 0), np.nextafter(base, np.inf),
            base * (1 + 1e-9), base * (1 - 1e-9)]
    for rel in (1e-7, 1e-6, 1e-5, 1e-4, 3e-4, 1e-3, 3e-3):  # FP32 decision margin ~2e-6 rel
        vals.append((base * (1 + rng.uniform(-rel, rel, (64, base.size)))).ravel())
    vals += [np.array([0.0, -0.0, np.nan, np.inf, -np.inf, -1.0, -0.5, 1e-300, 5e-324, 1e-8,
                       1e6, 1e6 + 1, 1e7, 1e300, 2.0 ** 53, 0.5, 1.0, 2.0 ** 20,
                       np.nextafter(2.0 ** 20, 0), np.nextafter(2.0 ** 20, np.inf)]),
             10.0 ** rng.uniform(-12, 8, 50000), rng.uniform(0, 4, 50000)]
    c = np.concatenate([np.ravel(v) for v in vals])
    c = c[: c.size - c.size % 3].reshape(-1, 3)
    got = ctx.tonemap(c, 1)
    assert np.array_equal(got, oracle.tonemap(c, 1))


def _scene(width, height, aa=1, focal=None):
    f = width / 2.0 if focal is None else focal
    return SceneData(Camera((0.0, 0.0, -25.0), f, width, height, 0.0, 200.0, aa))


def test_edge_empty_scene_is_sky(ctx, oracle):
    sc = _scene(67, 13)
    out = _render(ctx, sc, hdr64=True, stats=True)
    ref, _, _ = oracle.render(sc)
    assert np.array_equal(out["hdr64"], ref)
    assert out["shadow_rays"] == 0


def test_edge_no_lights_and_one_pixel(ctx, oracle):
    sc = _scene(1, 1, focal=100.0)  # the pixel-corner ray of a 1x1 image hits the sphere
    sc.add_sphere((0, 0, 5), 2.0, Material((1, 0, 0)))
    out = _render(ctx, sc, hdr64=True)
    assert np.array_equal(out["hdr64"], oracle.render(sc)[0])
    assert np.array_equal(out["hdr64"], np.zeros((1, 1, 3)))


def test_edge_aa_zero_is_black(ctx):
    sc = make_config("c2", 64, 8, aa=0)
    out = _render(ctx, sc, hdr64=True)
    assert not out["hdr64"].any()


@pytest.mark.parametrize("max_rec", [0, 1, 2, 16])
def test_edge_max_recursion(ctx, oracle, max_rec):
    sc = make_config("mirror", 48, 32)
    out = _render(ctx, sc, hdr64=True, max_recursion=max_rec)
    ref, _, _ = oracle.render(sc, max_recursion=max_rec)
    assert np.abs(out["hdr64"] - ref).max() <= POW_TOL


def test_edge_large_scene_bypasses_lds(ctx, oracle):
    """Scenes whose records exceed the LDS budget are read from HBM instead."""
    sc = _scene(64, 36)
    rng = np.random.default_rng(3)
    for _ in range(1500):
        sc.add_sphere(rng.uniform(-12, 12, 3) + (0, 0, 10), rng.uniform(0.1, 0.4),
                      Material(tuple(rng.uniform(0.2, 1, 3))))
    sc.add_light((0, 10, -5), (1, 1, 1), 200)
    out = _render(ctx, sc, hdr64=True)
    assert np.array_equal(out["hdr64"], oracle.render(sc)[0])


@pytest.mark.parametrize("scale", [1e150, 1e-100, 1e-160])
def test_edge_out_of_core_range_vectors(ctx, oracle, scale):
    """Lights and spheres at magnitudes where v·v leaves [2^-78, 2^120] (light vectors, hit
    normals) mixed with ordinary ones in the same waves: the exact lowering takes those lanes
    (rt_device.hpp), and the image is still bit-identical."""
    sc = _scene(96, 54)
    sc.add_sphere((0, 0, 5), 3.0, Material((0.8, 0.3, 0.3)))
    sc.add_sphere((-6, 2, 8), 2.0, Material((0.3, 0.8, 0.3)))
    sc.add_sphere((5 * scale, 3 * scale, 40 * scale), 4 * scale, Material((0.3, 0.3, 0.9)))
    sc.add_plane((0, -4, 0), (0, 1, 0), Material((0.7, 0.7, 0.7)))
    sc.add_light((0, 10, -5), (1, 1, 1), 150)
    sc.add_light((0.0, 3.0 + 2 * scale, 5.0), (1, 0.5, 0.5), 20)   # zero x: exact zero components
    sc.add_light((2 * scale, 2 * scale, -3 * scale), (0.5, 0.5, 1), 80 * scale * scale)
    out = _render(ctx, sc, hdr64=True, stats=True)
    ref, nt, ns = oracle.render(sc)
    assert np.array_equal(out["hdr64"], ref)
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


@pytest.mark.parametrize("offset", [0.0, 1e-300, -1e-200, 1e-13])
def test_edge_camera_on_or_near_a_plane(ctx, oracle, offset):
    """Planes through (or within a denormal distance of) the camera give camera-ray numerators
    outside the plane core's range: those planes take the exact division (rt_packet.hip
    plane_t); tilted normals give zero / tiny components."""
    sc = _scene(80, 40)
    sc.add_plane((0, offset, -25), (0, 1, 0), Material((0.6, 0.6, 0.6)))  # camera at y = 0
    sc.add_plane((0, -5, 0), (0.0, 1.0, 1e-310), Material((0.5, 0.7, 0.5)))
    sc.add_plane((0, 0, 30), (0.3, -0.2, -1.0), Material((0.4, 0.4, 0.8)))
    sc.add_sphere((1, 1, 6), 2.5, Material((0.9, 0.4, 0.2)))
    sc.add_light((0, 8, 0), (1, 1, 1), 200)
    out = _render(ctx, sc, hdr64=True)
    assert np.array_equal(out["hdr64"], oracle.render(sc)[0])


def _grazing_shadow_scene(gap):
    """1×1 image (all 64 lanes of the wave trace the same pixel, so the shadow packet's origin
    ball has radius 0) of a floor point lit by a light 0.14 away; a sphere of radius 0.01 sits
    `gap` beyond the segment [so, light] on the side the traced shadow ray deviates to.  The
    ray starts at so = P + n·bias but aims along (light − P), so near the light end it runs
    ~6e-4 off that segment (rt_packet.hip cull_capsule): with gap = 4e-4 it still passes 2e-4
    inside the sphere, and the reference shades the pixel black."""
    cam = np.array([0.0, 5.0, 0.0])
    f = 5.0
    d = np.array([-0.5, 0.5, cam[2] + f]) - cam    # the 1×1 image's ray (Math.h:99-121)
    d /= np.linalg.norm(d)
    P = cam + d * (cam[1] / -d[1])                  # on the floor y = 0
    so = P + np.array([0.0, 1e-3, 0.0])             # + n·bias
    light = P + np.array([0.1, 0.1, 0.0])
    u = (light - so) / np.linalg.norm(light - so)
    w = np.array([0.0, 1.0, 0.0]) - u[1] * u
    w /= np.linalg.norm(w)
    r = 0.01
    sc = SceneData(Camera(tuple(cam), f, 1, 1, 0.0, 200.0, 1))
    sc.add_plane((0, 0, 0), (0, 1, 0), Material((0.8, 0.8, 0.8)))
    sc.add_sphere(tuple(so + 0.12 * u + (r + gap) * w), r, Material((0.9, 0.2, 0.2)))
    sc.add_light(tuple(light), (1, 1, 1), 1.0)
    return sc


@pytest.mark.parametrize("gap", [4e-4, 5e-2])
def test_edge_shadow_ray_grazing_near_the_light(ctx, oracle, gap):
    """The shadow packet's cull covers the traced ray, not only the segment it aims at."""
    sc = _grazing_shadow_scene(gap)
    ref, nt, ns = oracle.render(sc)
    assert (ref == 0).all() == (gap < 1e-3)          # blocked only by the grazed sphere
    out = _render(ctx, sc, hdr64=True, stats=True)
    assert np.array_equal(out["hdr64"], ref)
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


@pytest.mark.parametrize("gap", [0.0, 5e-4, 2e-3, -3e-4])
def test_edge_plane_cull_light_near_a_plane(ctx, oracle, gap):
    """Scenes with ≥ 3 planes cull planes per shadow packet (rt_packet.hip cull_capsule,
    kFeatPlanes): lights on, just in front of and just behind a wall (within the bias of the
    shadow rays), tilted planes, and origins on the walls themselves — bit-identical images."""
    sc = _scene(96, 54)
    sc.add_plane((0, -6, 0), (0, 1, 0), Material((0.8, 0.8, 0.8)))
    sc.add_plane((0, 0, 14), (0, 0, -1), Material((0.7, 0.8, 0.9)))
    sc.add_plane((-12, 0, 0), (1, 0.05, 0), Material((0.9, 0.3, 0.3)))
    sc.add_plane((12, 0, 0), (-1, 0, 0.02), Material((0.3, 0.9, 0.3)))
    sc.add_sphere((0, -3, 6), 2.5, Material((0.9, 0.6, 0.2)))
    sc.add_sphere((-6, 1, 10), 1.5, Material((0.2, 0.6, 0.9)))
    sc.add_light((2, 4, 14 - gap), (1, 1, 1), 120)     # at / in front of / behind the back wall
    sc.add_light((-12 + gap, 2, 0), (1, 0.8, 0.6), 80)  # at the left wall
    sc.add_light((0, 8, -5), (1, 1, 1), 150)
    out = _render(ctx, sc, hdr64=True, stats=True)
    ref, nt, ns = oracle.render(sc)
    assert np.array_equal(out["hdr64"], ref)
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


def _walls_scene(aa=1, extra_spheres=0, specular=0.0, area=False, gap=5e-4):
    """test_edge_plane_cull_light_near_a_plane's walls, in the other packet variants that cull
    planes per shadow packet: AA > 1 (the multi-sample variant), > 64 spheres (MAXC = 4: also the
    split of wide shadow packets and the exact march's own capsule), specular materials (the
    general variant, kFeatAll) and an area light among the walls (per-cell masks ANDed with
    the shared plane mask)."""
    from raytracingengine_amd.scene import AreaLight
    sc = _scene(96, 54, aa=aa)
    mat = lambda c: Material(c, shininess=24.0, specular=specular)  # noqa: E731
    sc.add_plane((0, -6, 0), (0, 1, 0), mat((0.8, 0.8, 0.8)))
    sc.add_plane((0, 0, 14), (0, 0, -1), mat((0.7, 0.8, 0.9)))
    sc.add_plane((-12, 0, 0), (1, 0.05, 0), mat((0.9, 0.3, 0.3)))
    sc.add_plane((12, 0, 0), (-1, 0, 0.02), mat((0.3, 0.9, 0.3)))
    sc.add_sphere((0, -3, 6), 2.5, mat((0.9, 0.6, 0.2)))
    sc.add_sphere((-6, 1, 10), 1.5, mat((0.2, 0.6, 0.9)))
    for i in range(extra_spheres):   # a grid of small spheres, some touching the floor / walls
        sc.add_sphere((-11 + 22 * (i % 10) / 9, -5.6 + 1.3 * (i // 10), 4 + (i * 7 % 10)),
                      0.45 + 0.1 * (i % 3), mat((0.5, 0.5 + 0.05 * (i % 5), 0.4)))
    sc.add_light((2, 4, 14 - gap), (1, 1, 1), 120)
    sc.add_light((-12 + gap, 2, 0), (1, 0.8, 0.6), 80)
    sc.add_light((0, 8, -5), (1, 1, 1), 150)
    if area:
        sc.area_light = AreaLight((-3.0, 5.9, 2.0), (6.0, 0.0, 0.0), (0.0, 0.0, 6.0),
                                  intensity=200.0, samples=4)
    return sc


@pytest.mark.parametrize("kind", ["aa2", "many_spheres", "many_spheres_aa2", "specular",
                                  "area_specular"])
def test_edge_plane_cull_variants(ctx, oracle, kind):
    sc = _walls_scene(aa=2 if "aa2" in kind else 1,
                      extra_spheres=70 if "many" in kind else 0,
                      specular=0.3 if "specular" in kind else 0.0, area="area" in kind)
    out = _render(ctx, sc, hdr64=True, stats=True, seed=7)
    ref, nt, ns = oracle.render(sc, seed=7)
    if "specular" in kind:   # Blinn-Phong pow: device pow_bp vs libm, the 1e-12 bar
        assert np.allclose(out["hdr64"], ref, rtol=0, atol=1e-12)
    else:
        assert np.array_equal(out["hdr64"], ref)
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


@pytest.mark.parametrize("n_spheres,aa", [(100, 1), (300, 1), (130, 2)])
def test_sphere_chunks_keep_scene_order_ties(ctx, oracle, n_spheres, aa):
    """Scenes with > 64 spheres run the packet kernel on spheres in spatial-chunk order
    (rt_bvh.cpp build_sphere_chunks): coincident duplicate spheres with different materials —
    some in one chunk, some split across chunks — must still resolve to the lower scene index,
    as the reference's in-order loop with strict '<' does (Scene.h:218-257, Shape.h:36)."""
    from raytracingengine_amd.configs import SplitMix64
    rng = SplitMix64(0xC0FFEE + n_spheres)
    sc = _scene(160, 90, aa=aa)
    sc.add_plane((0, -9, 0), (0, 1, 0), Material((0.8, 0.8, 0.8)))
    placed = []
    for i in range(n_spheres):
        if i % 9 == 8 and placed:           # a duplicate of an earlier sphere, new colour
            c, r = placed[int(rng.uniform(0, len(placed)))]
        else:
            c = (rng.uniform(-12, 12), rng.uniform(-7, 7), rng.uniform(0, 16))
            r = rng.uniform(0.4, 1.6)
            placed.append((c, r))
        sc.add_sphere(c, r, Material((rng.uniform(0.1, 1), rng.uniform(0.1, 1), rng.uniform(0.1, 1))))
    sc.add_light((3, 11, -6), (1, 1, 1), 200)
    sc.add_light((-7, 8, -12), (1, 0.9, 0.8), 120)
    out = _render(ctx, sc, hdr64=True, stats=True, seed=11)
    ref, nt, ns = oracle.render(sc, seed=11)
    assert np.array_equal(out["hdr64"], ref)
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


def test_invalid_arguments_raise(ctx):
    sc = make_config("c2", 32, 16)
    ds = ctx.scene(sc)
    try:
        with pytest.raises(capi.RtError) as e:
            ds.render(hdr64=True, row_begin=10, row_end=40)
        assert e.value.status == capi.RT_ERR_INVALID_ARG
        with pytest.raises(capi.RtError):
            ds.render(hdr64=True, row_begin=8, row_end=8)
        with pytest.raises(capi.RtError) as e:
            ds.render(hdr64=True, tonemap=9)
        assert e.value.status == capi.RT_ERR_INVALID_ARG
        with pytest.raises(capi.RtError) as e:  # block-cyclic rows need a block height
            ds.render(hdr64=True, row_cycle=2, row_block=0)
        assert e.value.status == capi.RT_ERR_INVALID_ARG
        # a cycle of 1 is the contiguous range; blocks past row_end are clipped
        one = ds.render(hdr64=True, row_cycle=1, row_block=4)
        full = ds.render(hdr64=True)
        assert np.array_equal(one["hdr64"], full["hdr64"])
        tail = ds.render(hdr64=True, row_begin=12, row_cycle=3, row_block=5)
        assert np.array_equal(tail["hdr64"], full["hdr64"][12:16])
    finally:
        ds.close()
    mirror = make_config("mirror", 16, 16)
    with pytest.raises(capi.RtError) as e:
        _render(ctx, mirror, hdr64=True, max_recursion=17)
    assert e.value.status == capi.RT_ERR_UNSUPPORTED


def _with_camera(sc, k):
    import copy
    out = copy.copy(sc)
    out.camera = Camera((0.7 * k - 6.0, 0.4 * k - 2.0, -25.0 - 0.5 * k), sc.camera.width / 2.0,
                        sc.camera.width, sc.camera.height, 0.0, 200.0, 1)
    return out


def test_packet_image_per_camera(ctx, oracle):
    """The packet kernel's LDS image is formed once per (scene, camera position) on the second
    render from that camera and then copied by every workgroup (rt_capi.cpp packet_image): 20
    camera positions on one uploaded scene, each rendered twice (the first render forms the
    image in LDS, the second creates the cached one; past 16 cameras every render forms it in
    LDS), then earlier cameras again (cache hits); every frame equals the oracle's."""
    base = make_config("c3", 64, 36)
    ds = ctx.scene(base)
    try:
        frames = []
        for k in range(20):
            sc = _with_camera(base, k)
            ds.camera = sc.camera.to_struct()
            first = ds.render(hdr64=True)["hdr64"]
            frames.append(ds.render(hdr64=True)["hdr64"])
            assert np.array_equal(first, frames[-1])
            if k in (0, 7, 15, 16, 19):
                assert np.array_equal(frames[-1], oracle.render(sc)[0])
        for k in (0, 3, 18):
            ds.camera = _with_camera(base, k).camera.to_struct()
            assert np.array_equal(ds.render(hdr64=True)["hdr64"], frames[k])
    finally:
        ds.close()


def test_packet_image_shared_across_streams(ctx):
    """A camera's image created on one stream (its second render there) and used at once on
    another: the other stream waits for the setup event (or finds it complete) — every frame
    equals a synchronous one."""
    import torch
    base = make_config("c2", 256, 128)
    ds = ctx.scene(base)
    try:
        ds.camera = _with_camera(base, 5).camera.to_struct()
        bufs = [torch.empty(128 * 256 * 3, dtype=torch.float64, device="cuda") for _ in range(3)]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for buf, s in zip(bufs, (streams[0], streams[0], streams[1])):
            ctx.set_stream(s.cuda_stream)
            ds.render_device(buf.data_ptr(), None, None, capi.default_opts())
        for s in streams:
            s.synchronize()
        ctx.set_stream(None)
        ref = ds.render(hdr64=True)["hdr64"].reshape(-1)
        for buf in bufs:
            assert np.array_equal(buf.cpu().numpy(), ref)
    finally:
        ds.close()


def test_render_device_into_torch_buffers(ctx):
    import torch
    sc = make_config("c2", 256, 128)
    ds = ctx.scene(sc)
    try:
        ref = ds.render(hdr64=True, hdr32=True, tonemap=1)
        h32 = torch.empty(128 * 256 * 3, dtype=torch.float32, device="cuda")
        ldr = torch.empty(128 * 256 * 3, dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        ctx.set_stream(s.cuda_stream)
        ds.render_device(None, h32.data_ptr(), ldr.data_ptr(), capi.default_opts(tonemap=1))
        s.synchronize()
        ctx.set_stream(None)
    finally:
        ds.close()
    assert np.array_equal(h32.cpu().numpy().reshape(128, 256, 3), ref["hdr32"])
    assert np.array_equal(ldr.cpu().numpy().reshape(128, 256, 3), ref["ldr"])


# ------------------------------------------------------------------ breadth-first TraceRay
@pytest.mark.parametrize("name,aa,max_rec", [("glass", 1, 10), ("mirror", 1, 10), ("c1", 1, 10),
                                             ("glass", 3, 6), ("mesh", 1, 10), ("glass", 1, 16)])
def test_wavefront_equals_per_pixel_kernel(ctx, monkeypatch, name, aa, max_rec):
    """Scenes with secondary rays render level by level (rt_wavefront.hip); the image must be
    bit-identical to the per-pixel DFS kernel (RT_FLAG_GENERIC_KERNEL) for the tree (glass)
    shape — same rays, same fold order — with AA and deep recursion.  Reflection chains (mirror,
    c1, mesh) are folded back to front breadth-first but accumulated front to back per pixel
    (rt_trace_common.hpp trace_chain): the same sums in another rounding order, within 1e-12."""
    sc = make_config(name, 160, 90, aa=aa)
    monkeypatch.setenv("RTAMD_WF_CHAIN", "1")  # chains are per-pixel by default
    ds = ctx.scene(sc)
    try:
        a = ds.render(hdr64=True, tonemap=1, max_recursion=max_rec)
        b = ds.render(hdr64=True, tonemap=1, max_recursion=max_rec,
                      flags=capi.RT_FLAG_GENERIC_KERNEL)
    finally:
        ds.close()
    if name == "glass":
        assert np.array_equal(a["hdr64"], b["hdr64"], equal_nan=True)
        assert np.array_equal(a["ldr"], b["ldr"])
    else:
        assert np.abs(a["hdr64"] - b["hdr64"]).max() <= POW_TOL
        same = np.all(a["hdr64"] == b["hdr64"], axis=-1)
        assert np.array_equal(a["ldr"][same], b["ldr"][same])


@pytest.mark.parametrize("mb", ["1", "2"])
def test_wavefront_arena_overflow_falls_back_per_pixel(ctx, oracle, monkeypatch, mb):
    """A tiny arena (RTAMD_WF_MB) overflows: the flagged samples are re-rendered by the
    per-pixel kernel in the same stream, so the image is still the reference's."""
    sc = make_config("glass", 320, 180)
    monkeypatch.setenv("RTAMD_WF_MB", mb)
    out = _render(ctx, sc, hdr64=True)
    monkeypatch.delenv("RTAMD_WF_MB")
    ref = _render(ctx, sc, hdr64=True, flags=capi.RT_FLAG_GENERIC_KERNEL)
    assert np.array_equal(out["hdr64"], ref["hdr64"], equal_nan=True)
    want, _, _ = oracle.render(sc, rows=(0, 20))
    assert np.abs(out["hdr64"][:20] - want).max() <= POW_TOL


# ------------------------------------------------------------------ triangle BVH
def test_bvh_scene_vs_oracle(ctx, oracle):
    """8320 triangles (icosphere + terrain models) through the BVH: bit-identical to the C
    restatement's brute-force IntersectClosest, exact ray counts."""
    sc = make_config("bigmesh", 96, 54)
    out = _render(ctx, sc, hdr64=True, tonemap=1, stats=True)
    ref, nt, ns = oracle.render(sc)
    assert np.array_equal(out["hdr64"], ref)
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


@pytest.mark.parametrize("name,flags", [("bigmesh", 0), ("bigmesh", capi.RT_FLAG_GENERIC_KERNEL),
                                        ("mesh", 0), ("mesh", capi.RT_FLAG_GENERIC_KERNEL)])
def test_bvh_equals_every_triangle(ctx, name, flags):
    """The BVH changes which triangles are tested, never which hit wins (ties go to the lowest
    index, as in the reference's ordered loop): images equal the all-triangles test."""
    sc = make_config(name, 320, 180)
    ds = ctx.scene(sc)
    try:
        a = ds.render(hdr64=True, tonemap=1, flags=flags)
        b = ds.render(hdr64=True, tonemap=1, flags=flags | capi.RT_FLAG_NO_BVH)
    finally:
        ds.close()
    assert np.array_equal(a["hdr64"], b["hdr64"])
    assert np.array_equal(a["ldr"], b["ldr"])


def test_bvh_ties_go_to_lowest_index(ctx):
    """Coincident duplicate triangles (same geometry, different materials) in a BVH-sized mesh:
    the first one wins every tie, as in the reference's strict-< loop, so the image equals the
    scene without the duplicates."""
    from raytracingengine_amd.configs import SplitMix64, _terrain

    tris = _terrain(8, 10.0, SplitMix64(5))

    def scene(dup):
        sc = SceneData(Camera((0.0, 0.0, -25.0), 80.0, 160, 90, 1.0, 1000.0, 1), name="ties")
        sc.add_model(tris, (0.0, -2.0, 4.0), Material((1.0, 0.0, 0.0)))
        if dup:
            sc.add_model(tris, (0.0, -2.0, 4.0), Material((0.0, 1.0, 0.0)))
        sc.add_light((0.0, 10.0, -10.0), (1.0, 1.0, 1.0), 200.0)
        return sc

    a = _render(ctx, scene(True), hdr64=True)
    b = _render(ctx, scene(False), hdr64=True)
    assert len(scene(True).triangle_array()) >= 256
    assert np.array_equal(a["hdr64"], b["hdr64"])


# ------------------------------------------------------------------ one frame, several contexts
@pytest.mark.parametrize("name,n,block", [("c2", 3, 16), ("glass", 2, 0), ("c3", 4, 7)])
def test_render_multi_equals_single(name, n, block):
    """rt_render_multi (Scene::SetDevices): n contexts — here all on GPU 0 — render their
    block-cyclic rows concurrently and the host assembles one frame equal to the single-context
    render, ray counts summed."""
    sc = make_config(name, 240, 136)
    ctxs = [capi.Context(0) for _ in range(n)]
    try:
        scenes = [c.scene(sc) for c in ctxs]
        multi = capi.render_multi(scenes, hdr64=True, tonemap=1, stats=True, row_block=block)
        single = scenes[0].render(hdr64=True, tonemap=1, stats=True)
        for ds in scenes:
            ds.close()
    finally:
        for c in ctxs:
            c.close()
    assert np.array_equal(multi["hdr64"], single["hdr64"])
    assert np.array_equal(multi["ldr"], single["ldr"])
    assert (multi["trace_rays"], multi["shadow_rays"]) == (single["trace_rays"],
                                                            single["shadow_rays"])


# ------------------------------------------------------------------ planes: edge rays
def _axis_box_scene():
    """Axis-aligned planes with signed-zero normal components, a plane through the origin, one
    far beyond the scene (3e303) and one tilted plane."""
    sc = _scene(64, 48)
    sc.add_plane((0, -3, 0), (0.0, 1.0, 0.0), Material((0.8, 0.8, 0.8)))
    sc.add_plane((0, 0, 10), (-0.0, -0.0, -1.0), Material((0.7, 0.8, 0.9)))
    sc.add_plane((4, 0, 0), (-1.0, 0.0, -0.0), Material((0.9, 0.3, 0.3)))
    sc.add_plane((0, 0, 0), (0.0, 0.0, 1.0), Material((0.2, 0.9, 0.2)))       # through o = 0
    sc.add_plane((3e303, 5.0, 0), (0.0, -1.0, 0.0), Material((0.5, 0.5, 0.5)))  # bound: literal
    sc.add_plane((0, 6, 0), (0.3, -1.0, 0.2), Material((0.4, 0.4, 0.8)))      # general
    sc.add_sphere((1, 0, 4), 1.5, Material((0.9, 0.4, 0.2)))
    sc.add_light((0, 2.5, -2), (1, 1, 1), 40)
    return sc


def test_edge_axis_planes_batch_rays_vs_oracle(ctx, oracle):
    """IntersectClosest (rt_intersect_rays, the generic closest()) on crafted rays against axis
    planes: origins exactly on a plane (t = ±0 accepted, Shape.h:155), directions parallel to a
    plane or with ±0 components, huge / non-finite origins and directions, against the
    oracle's literal arithmetic (including the sign of a zero distance)."""
    sc = _axis_box_scene()
    rng = np.random.default_rng(11)
    n = 2048
    o = rng.uniform(-2.5, 3.5, (n, 3))
    d = rng.normal(0, 1, (n, 3))
    o[:64, 1] = -3.0                        # on the floor (c == 0 for the floor)
    o[64:128, 2] = 0.0                      # on the z = 0 plane, both signs of zero
    o[96:128, 2] = -0.0
    o[128:192, 0] = 4.0                     # on the right wall
    d[192:256, 1] = 0.0                     # parallel to the floor / ceiling
    d[256:320, 2] = -0.0
    d[320:336, 0] = 1e-7                    # |d_k| ≤ 1e-6 after normalisation below
    d[336:352] = [np.inf, 0.3, 0.1]          # non-finite directions
    d[352:368] = [np.nan, 0.3, 0.1]
    o[368:384] = [2.0 ** 1021, 0.0, 0.0]     # huge origin
    d[384:400] *= 2.0 ** 101                 # huge direction
    o[400:416] = [np.inf, 0.0, 1.0]
    with np.errstate(invalid="ignore"):
        nrm = np.linalg.norm(d[:336], axis=1, keepdims=True)
        d[:336] = d[:336] / nrm
    d[320:336, 0] = 1e-7
    rays = np.concatenate([o, d], axis=1)
    ds = ctx.scene(sc)
    try:
        got = ds.intersect_rays(rays)
    finally:
        ds.close()
    for i, ray in enumerate(rays):
        typ, idx, vals = oracle.closest(sc, ray)
        assert int(got[i, 0]) == typ, i
        if typ:
            assert int(got[i, 1]) == idx, i
            assert np.array_equal(got[i, 2:], vals, equal_nan=True), (i, got[i, 2:], vals)
            # the sign of a zero distance is the reference's too (NaN signs are not IEEE
            # values: x86 and gfx950 produce differently signed default NaNs)
            if got[i, 2] == 0.0:
                assert np.signbit(got[i, 2]) == np.signbit(vals[0]), i


@pytest.mark.parametrize("flags", [0, capi.RT_FLAG_GENERIC_KERNEL])
def test_edge_axis_planes_scene_vs_oracle(ctx, oracle, flags):
    """The same box rendered whole (packet kernel and the generic kernel): shadow rays starting
    on and next to the walls — bit-identical to the oracle."""
    sc = _axis_box_scene()
    out = _render(ctx, sc, hdr64=True, stats=True, flags=flags)
    ref, nt, ns = oracle.render(sc)
    assert np.array_equal(out["hdr64"], ref)
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


# ------------------------------------------------------------------ costliest-first tile order
@pytest.mark.parametrize("name,w,h", [("c2", 1920, 1080), ("c3", 1920, 1080), ("c5", 960, 540),
                                      ("c4", 1000, 600)])
def test_tile_order_is_a_permutation_and_keeps_the_image(ctx, name, w, h):
    """rt_capi.cpp tile_order: the render that creates a camera's packet image records every
    wave's duration, the next one builds the dispatch order (rt_packet.hip packet_order_kernel)
    and renders by it.  The order is a permutation of the tiles (every tile rendered exactly
    once) and the image is bit-identical to the unordered renders."""
    sc = make_config(name, w, h)
    ds = ctx.scene(sc)
    try:
        first = ds.render(hdr64=True)                       # publish slot, default order
        assert ds.debug_tile_order()[0] == 0
        second = ds.render(hdr64=True)                      # image created, durations recorded
        st, order, cost = ds.debug_tile_order()
        assert st == 1 and order is None and (cost > 0).all()
        third = ds.render(hdr64=True)                       # order built and used
        st, order, cost = ds.debug_tile_order()
        assert st == 2
        assert np.array_equal(np.sort(order), np.arange(order.size, dtype=np.uint32))
        tile = cost.max(axis=1).astype(np.float64)
        print(f"TILECOST {name} {w}x{h}: tiles {tile.size} median {np.median(tile):.0f} "
              f"p99 {np.percentile(tile, 99):.0f} max {tile.max():.0f} (10 ns ticks); "
              f"order default {bool(np.array_equal(order[:8], _default_order(order.size, w)[:8]))}")
        unordered = ds.render(hdr64=True, flags=capi.RT_FLAG_NO_TILE_ORDER)
    finally:
        ds.close()
    for img in (second, third, unordered):
        assert np.array_equal(img["hdr64"], first["hdr64"])


def _default_order(tiles, w):
    gx = (w + 15) // 16
    gy = tiles // gx
    lin = np.arange(tiles)
    return (gy - 1 - lin // gx) * gx + lin % gx


# ------------------------------------------------------------------ planes-only chain kernel
def _room_scene(kind):
    """Planes-only reflection-chain scenes for the planes-only chain kernel (rt_box.hip)."""
    mir = dict(specular=0.3, shininess=16.0)
    if kind == "c1":          # the reference main()'s box at a reduced size
        return make_config("c1", 120, 100)
    if kind == "room":        # axis walls with signed-zero normals, one tilted wall, a plane far
        sc = _scene(72, 56)   # away and two coincident walls of different colour (ties)
        sc.add_plane((0, -3, 0), (0.0, 1.0, 0.0), Material((0.8, 0.8, 0.8), **mir))
        sc.add_plane((0, 0, 10), (-0.0, -0.0, -1.0), Material((0.7, 0.8, 0.9), **mir))
        sc.add_plane((4, 0, 0), (-1.0, 0.0, -0.0), Material((0.9, 0.3, 0.3), specular=0.5))
        sc.add_plane((4, 0, 0), (-1.0, 0.0, 0.0), Material((0.1, 0.9, 0.3), specular=0.5))
        sc.add_plane((-4, 0, 0), (1.0, 0.0, 0.0), Material((0.3, 0.3, 0.9), **mir))
        sc.add_plane((3e303, 5.0, 0), (0.0, -1.0, 0.0), Material((0.5, 0.5, 0.5), **mir))
        sc.add_plane((0, 6, 0), (0.3, -1.0, 0.2), Material((0.4, 0.4, 0.8), **mir))
        sc.add_light((0, 2.5, -2), (1, 1, 1), 40)
        sc.add_light((-2, -2.5, 8), (1, 0.5, 0.2), 25)
        return sc
    if kind == "on_floor":    # the camera exactly on the floor plane (camera rays start on it)
        sc = SceneData(Camera((0.0, -3.0, -25.0), 32.0, 64, 48, 0.0, 200.0, 1))
        sc.add_plane((0, -3, 0), (0.0, 1.0, 0.0), Material((0.8, 0.8, 0.8), **mir))
        sc.add_plane((0, 0, 12), (0.0, 0.0, -1.0), Material((0.6, 0.7, 0.8), **mir))
        sc.add_plane((0, 9, 0), (0.0, -1.0, 0.0), Material((0.9, 0.9, 0.5), **mir))
        sc.add_light((1, 4, -3), (1, 1, 1), 60)
        return sc
    if kind == "huge":        # coordinates beyond the shortcut's bounds: the literal path
        sc = SceneData(Camera((2.0 ** 1001, 0.0, -25.0), 32.0, 48, 32, 0.0, 200.0, 1))
        sc.add_plane((0, -3, 0), (0.0, 1.0, 0.0), Material((0.8, 0.8, 0.8), **mir))
        sc.add_plane((2.0 ** 1002, 0, 0), (-1.0, 0.0, 0.0), Material((0.9, 0.3, 0.3), **mir))
        sc.add_light((0, 2.5, -2), (1, 1, 1), 40)
        return sc
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["c1", "room", "on_floor", "huge"])
@pytest.mark.parametrize("aa,max_rec", [(1, 10), (1, 1), (1, 16), (3, 4)])
def test_box_chain_equals_generic_chain(ctx, kind, aa, max_rec):
    """rt_box.hip (planes in axis groups read through the scalar cache, t = (p_k − o_k)/d_k,
    shadow classification from the same A, B) renders every pixel bit-identical to the generic
    chain kernel (RT_FLAG_GENERIC_KERNEL), with the same ray counts — including coincident
    walls (closest-hit ties: lowest scene index), camera rays starting on a plane (t = ±0),
    a tilted plane and coordinates outside the shortcut's bounds."""
    sc = _room_scene(kind)
    if aa != 1:
        sc = sc.resized(sc.camera.width, sc.camera.height, aa)
    out = _render(ctx, sc, hdr64=True, tonemap=6, stats=True,
                  max_recursion=max_rec)
    ref = _render(ctx, sc, hdr64=True, tonemap=6, stats=True,
                  max_recursion=max_rec, flags=capi.RT_FLAG_GENERIC_KERNEL)
    assert np.array_equal(out["hdr64"], ref["hdr64"], equal_nan=True)
    assert np.array_equal(out["ldr"], ref["ldr"])
    assert (out["trace_rays"], out["shadow_rays"]) == (ref["trace_rays"], ref["shadow_rays"])


@pytest.mark.parametrize("kind", ["room", "on_floor"])
def test_box_chain_vs_oracle(ctx, oracle, kind):
    """The planes-only chain kernel against the C restatement (chains: ≤ 1e-12, Blinn-Phong pow)."""
    sc = _room_scene(kind)
    out = _render(ctx, sc, hdr64=True, stats=True)
    ref, nt, ns = oracle.render(sc)
    assert np.max(np.abs(out["hdr64"] - ref)) <= POW_TOL
    assert (out["trace_rays"], out["shadow_rays"]) == (nt, ns)


@pytest.mark.parametrize("aa", [2, 3, 7, 32, 128, 129])
def test_box_sample_parallel_equals_per_thread_loop(ctx, aa):
    """Multi-sample planes-only chains run one thread per sample (rt_box.hip box_aa_kernel: 256 /
    aa pixels per workgroup, the colours summed in sample order from LDS); the image, the ACES
    bytes and the ray counts equal the per-thread sample loop (RT_FLAG_NO_SAMPLE_PARALLEL) and
    the generic chain kernel bit for bit — sample counts that do not divide 256 (idle threads,
    pixels straddling no workgroup), the largest sample-parallel count and the first above it
    (per-thread loop either way), and a block-cyclic row set (the multi-GPU split)."""
    from raytracingengine_amd.distributed import render_opts_for, row_ranges
    sc = make_config("c1", 37 if aa >= 32 else 61, 23 if aa >= 32 else 45, aa=aa)
    ds = ctx.scene(sc)
    try:
        out = ds.render(hdr64=True, tonemap=6, stats=True)
        loop = ds.render(hdr64=True, tonemap=6, stats=True, flags=capi.RT_FLAG_NO_SAMPLE_PARALLEL)
        gen = ds.render(hdr64=True, tonemap=6, stats=True, flags=capi.RT_FLAG_GENERIC_KERNEL)
        H = sc.camera.height
        ranges = row_ranges(1, 3, H, 4)
        part = ds.render(hdr64=True, tonemap=6, opts=render_opts_for(ranges, 1, 3, H, 4, tonemap=6))
    finally:
        ds.close()
    for ref in (loop, gen):
        assert np.array_equal(out["hdr64"], ref["hdr64"])
        assert np.array_equal(out["ldr"], ref["ldr"])
        assert (out["trace_rays"], out["shadow_rays"]) == (ref["trace_rays"], ref["shadow_rays"])
    rows = np.concatenate([out["hdr64"][a:b] for a, b in ranges])
    assert np.array_equal(part["hdr64"], rows)


@pytest.mark.parametrize("name,flags", [("mirror", 0), ("mirror", capi.RT_FLAG_GENERIC_KERNEL),
                                        ("mesh", 0),
                                        ("c1", capi.RT_FLAG_GENERIC_KERNEL),
                                        ("c2", capi.RT_FLAG_GENERIC_KERNEL),
                                        ("c5", capi.RT_FLAG_GENERIC_KERNEL)])
@pytest.mark.parametrize("aa", [3, 32])
def test_generic_sample_parallel_equals_per_thread_loop(ctx, name, flags, aa):
    """Multi-sample frames of the generic direct and chain kernels (rt_trace.hip SPAR: one
    thread per sample, the colours summed in sample order from LDS): image, ACES bytes and ray
    counts equal the per-thread sample loop (RT_FLAG_NO_SAMPLE_PARALLEL) bit for bit — chains
    with spheres (mirror), triangles (mesh), planes only (c1 through the generic kernel), and
    the direct path with point lights (c2) and the area light (c5)."""
    sc = make_config(name, 53, 29, aa=aa)
    ds = ctx.scene(sc)
    try:
        out = ds.render(hdr64=True, tonemap=6, stats=True, flags=flags)
        ref = ds.render(hdr64=True, tonemap=6, stats=True,
                        flags=flags | capi.RT_FLAG_NO_SAMPLE_PARALLEL)
    finally:
        ds.close()
    assert np.array_equal(out["hdr64"], ref["hdr64"])
    assert np.array_equal(out["ldr"], ref["ldr"])
    assert (out["trace_rays"], out["shadow_rays"]) == (ref["trace_rays"], ref["shadow_rays"])


@pytest.mark.parametrize("variant,aa,max_rec", [("glass", 1, 10), ("glass", 3, 6), ("glass", 1, 1),
                                                ("glass", 1, 2), ("glass", 1, 16),
                                                ("glass_area_tris", 1, 10)])
def test_wavefront_deferred_direct_equals_in_level(ctx, monkeypatch, variant, aa, max_rec):
    """The shadow stage (RTAMD_WF_DEFER=1, opt-in): the level kernels queue every hit with
    transparency < 1 and wf_direct_kernel shades them after the last level (the light loop and
    its computeTransmittance marches, plus the fold with the sky children at the last shading
    level).  Bit-identical to the level kernels shading in place (RTAMD_WF_DEFER=0) and to the
    per-pixel DFS kernel, for AA, depth 1 (every root a leaf), 2, 10 and 16, and for the full
    build's level kernels (a transparent scene with triangles and the area light)."""
    sc = make_config("glass", 160, 90, aa=aa)
    if variant == "glass_area_tris":
        from raytracingengine_amd.scene import AreaLight, Material
        sc.add_triangle((-4.0, -3.0, 6.0), (4.0, -3.0, 6.0), (0.0, 4.0, 7.0),
                        Material((0.8, 0.7, 0.6), specular=0.2, transparency=0.5,
                                 refractive_index=1.3))
        sc.area_light = AreaLight((-3.0, 12.0, -8.0), (6.0, 0.0, 0.0), (0.0, 0.0, 6.0),
                                  (1.0, 1.0, 1.0), 150.0, 4)
    ds = ctx.scene(sc)
    try:
        outs = {}
        for defer in ("1", "0"):
            monkeypatch.setenv("RTAMD_WF_DEFER", defer)
            outs[defer] = ds.render(hdr64=True, tonemap=1, max_recursion=max_rec)
        ref = ds.render(hdr64=True, tonemap=1, max_recursion=max_rec,
                        flags=capi.RT_FLAG_GENERIC_KERNEL)
    finally:
        ds.close()
    for k in ("1", "0"):
        assert np.array_equal(outs[k]["hdr64"], ref["hdr64"], equal_nan=True), k
        assert np.array_equal(outs[k]["ldr"], ref["ldr"]), k


def _sphere_room(kind):
    """Scenes for the sphere instantiations of rt_box.hip: the mirror scene (12 spheres in a
    mirrored box), its spheres without the walls, and the mirror spheres around the camera (one
    sphere containing the camera: camera rays start inside it)."""
    import copy
    sc = make_config("mirror", 160, 90)
    if kind == "no_planes":
        sc = copy.deepcopy(sc)
        sc.planes = []
    elif kind == "camera_inside":
        from raytracingengine_amd.scene import Material
        sc = copy.deepcopy(sc)
        sc.add_sphere((0.0, 0.0, -25.0), 3.0, Material((0.5, 0.6, 0.7), shininess=16.0,
                                                       specular=0.5))
    return sc


@pytest.mark.parametrize("kind,aa,max_rec", [("mirror", 1, 10), ("mirror", 3, 4), ("mirror", 1, 1),
                                             ("mirror", 1, 16), ("no_planes", 1, 10),
                                             ("camera_inside", 1, 10), ("mirror", 32, 10)])
def test_box_spheres_equal_generic_chain(ctx, kind, aa, max_rec):
    """Reflection chains with spheres through rt_box.hip (spheres and axis-grouped planes read
    through the scalar cache, every sphere tested first in scene order with the literal
    Sphere::Intersect, then the planes' shortcut): every pixel, the ACES bytes and the ray counts
    bit-identical to the generic chain kernel — depth 1 to 16, AA (sample-parallel and the
    per-thread loop), a scene without planes and a camera inside a sphere."""
    sc = _sphere_room(kind)
    if aa != 1:
        sc = sc.resized(sc.camera.width, sc.camera.height, aa)
    out = _render(ctx, sc, hdr64=True, tonemap=6, stats=True, max_recursion=max_rec)
    ref = _render(ctx, sc, hdr64=True, tonemap=6, stats=True, max_recursion=max_rec,
                  flags=capi.RT_FLAG_GENERIC_KERNEL)
    assert np.array_equal(out["hdr64"], ref["hdr64"], equal_nan=True)
    assert np.array_equal(out["ldr"], ref["ldr"])
    assert (out["trace_rays"], out["shadow_rays"]) == (ref["trace_rays"], ref["shadow_rays"])
    if aa > 1:
        loop = _render(ctx, sc, hdr64=True, tonemap=6, max_recursion=max_rec,
                       flags=capi.RT_FLAG_NO_SAMPLE_PARALLEL)
        assert np.array_equal(out["hdr64"], loop["hdr64"], equal_nan=True)


def test_loaded_library_is_built_from_this_tree(ctx):
    """The librtamd.so this GPU run loaded was compiled from exactly the sources in this tree
    (rt_build_info's source_sha256 against build.source_digest), so the parity results above
    belong to these sources, not to a stale binary."""
    info = capi.build_info()
    assert info["arch"] == "gfx950"
    assert info["matches_tree"], info
