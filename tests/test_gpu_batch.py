"""Frame batches (rt_render_batch, rt_render_gather_batch, rt_render_gather_all_batch): several
frames of one scene — one camera position each — in one packet-kernel launch (one grid plane per
frame), each frame the frame rt_render gives for its camera (RE/Scene.h:311-328), and the
multi-rank batch layouts (padded send rows, per-frame gathers, per-frame assembly) end to end."""
import dataclasses
import hashlib

import numpy as np
import pytest
import torch

from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _positions(ds, n, seed=7):
    """n camera positions around the scene's own: the base position (cached image after its
    second sighting) mixed with moves seen once (hand-off slot / per-workgroup image)."""
    base = ds.camera["position"][0].copy()
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        out.append(base if i % 3 == 0 else base + rng.uniform(-0.5, 0.5, 3))
    return np.array(out)


def _single(ds, pos, opts, rows, w):
    """The frame of one camera position through rt_render_device (synchronous copy)."""
    saved = ds.camera["position"][0].copy()
    ds.camera["position"][0] = pos
    try:
        h = torch.empty(rows * w * 3, dtype=torch.float64, device="cuda")
        l = torch.empty(rows * w * 3, dtype=torch.uint8, device="cuda")
        ds.render_device(h.data_ptr(), None, l.data_ptr(), opts)
        ds.ctx.synchronize()
        return h.cpu().numpy(), l.cpu().numpy()
    finally:
        ds.camera["position"][0] = saved


@pytest.mark.parametrize("name,w,h,n", [("c2", 480, 270, 1), ("c2", 480, 270, 5),
                                        ("c2", 480, 270, 16), ("c2", 320, 180, 21), ("c2", 160, 90, 35),
                                        ("c3", 480, 270, 6), ("c5", 320, 180, 4),
                                        ("c4", 400, 240, 3), ("mesh", 320, 180, 3),
                                        ("bigmesh", 320, 180, 3), ("mirror", 240, 160, 3),
                                        ("glass", 160, 120, 2)])
def test_batch_frames_equal_single_renders(ctx, name, w, h, n):
    """Every frame of a batch equals rt_render_device of its camera, bit for bit (HDR and
    Reinhard bytes): packet scenes in one launch per 32 frames (C2-C5, triangles), chain and
    tree scenes one launch per frame.  Repeated, cached and first-seen cameras mixed."""
    sc = make_config(name, w, h)
    ds = ctx.scene(sc)
    try:
        pos = _positions(ds, n)
        opts = capi.default_opts(tonemap=1)
        refs = [_single(ds, p, opts, h, w) for p in pos]
        for rnd in range(2):  # the second round sees every camera again (cached images)
            H64 = torch.full((n * h * w * 3,), -1.0, dtype=torch.float64, device="cuda")
            L8 = torch.zeros(n * h * w * 3, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            ds.render_batch(ds.cameras(pos), H64.data_ptr(), None, L8.data_ptr(), opts)
            ctx.synchronize()
            a64 = H64.cpu().numpy().reshape(n, -1)
            a8 = L8.cpu().numpy().reshape(n, -1)
            for f in range(n):
                assert np.array_equal(a64[f], refs[f][0]), (rnd, f)
                assert np.array_equal(a8[f], refs[f][1]), (rnd, f)
    finally:
        ds.close()


def test_batch_moved_camera_vs_oracle(ctx, oracle):
    """A batch frame from a moved camera against the C oracle rendering that camera."""
    sc = make_config("c2", 192, 108)
    ds = ctx.scene(sc)
    try:
        base = np.array(sc.camera.position)
        pos = np.array([base, base + (0.3, -0.2, 0.5), base + (-0.7, 0.1, 1.0)])
        H64 = torch.empty(3 * 108 * 192 * 3, dtype=torch.float64, device="cuda")
        ds.render_batch(ds.cameras(pos), H64.data_ptr(), None, None, capi.default_opts(tonemap=-1))
        ctx.synchronize()
        got = H64.cpu().numpy().reshape(3, 108, 192, 3)
    finally:
        ds.close()
    for f in range(3):
        scf = dataclasses.replace(sc, camera=dataclasses.replace(sc.camera,
                                                                 position=tuple(pos[f])))
        ref, _, _ = oracle.render(scf)
        assert np.array_equal(got[f], ref), f


def test_batch_full_c2_static_camera_is_the_reference(ctx, golden):
    """The bench's batch: four 1920x1080 C2 frames of the static camera in one launch — each
    frame's HDR and Reinhard bytes have the reference's SHA-256."""
    info = golden["meta"]["scenes"]["c2_full"]
    sc = make_config("c2")
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    try:
        cams = ds.cameras(np.repeat(ds.camera["position"], 4, axis=0))
        H64 = torch.empty(4 * H * W * 3, dtype=torch.float64, device="cuda")
        L8 = torch.empty(4 * H * W * 3, dtype=torch.uint8, device="cuda")
        for _ in range(3):  # fresh camera, cache-creating and cached launches
            H64.zero_()
            L8.zero_()
            torch.cuda.synchronize()
            ds.render_batch(cams, H64.data_ptr(), None, L8.data_ptr(), capi.default_opts(tonemap=1))
            ctx.synchronize()
            a64 = H64.cpu().numpy().reshape(4, -1)
            a8 = L8.cpu().numpy().reshape(4, -1)
            for f in range(4):
                assert _sha(a64[f]) == info["image_sha256"], f
                assert _sha(a8[f]) == info["ldr_sha256"]["reinhard_simple"], f
    finally:
        ds.close()


def test_batch_row_sets_equal_single_row_renders(ctx):
    """A rank's block-cyclic rows of every frame of a batch = its single-frame row renders."""
    sc = make_config("c3", 480, 270)
    ds = ctx.scene(sc)
    try:
        pos = _positions(ds, 4, seed=3)
        o = capi.default_opts(tonemap=1, row_begin=32, row_end=270, row_block=16, row_cycle=3)
        rows = capi.rendered_rows(o, 270)
        refs = [_single(ds, p, o, rows, 480) for p in pos]
        H64 = torch.empty(4 * rows * 480 * 3, dtype=torch.float64, device="cuda")
        L8 = torch.empty(4 * rows * 480 * 3, dtype=torch.uint8, device="cuda")
        ds.render_batch(ds.cameras(pos), H64.data_ptr(), None, L8.data_ptr(), o)
        ctx.synchronize()
        a64 = H64.cpu().numpy().reshape(4, -1)
        a8 = L8.cpu().numpy().reshape(4, -1)
        for f in range(4):
            assert np.array_equal(a64[f], refs[f][0]), f
            assert np.array_equal(a8[f], refs[f][1]), f
    finally:
        ds.close()


def test_batch_ray_counts_are_the_sum_of_frames(ctx):
    """RT_FLAG_COUNT_RAYS over a batch counts every frame's rays (the counting launch is a
    batch too)."""
    sc = make_config("c2", 320, 180)
    ds = ctx.scene(sc)
    try:
        pos = _positions(ds, 3, seed=11)
        total = 0
        for p in pos:
            ds.camera["position"][0] = p
            out = ds.render(hdr64=True, stats=True)
            total += out["trace_rays"] + out["shadow_rays"]
        ds.camera["position"][0] = pos[0]
        H64 = torch.empty(3 * 180 * 320 * 3, dtype=torch.float64, device="cuda")
        ctx.reset_stats()
        ds.render_batch(ds.cameras(pos), H64.data_ptr(), None, None,
                        capi.default_opts(tonemap=-1, flags=capi.RT_FLAG_COUNT_RAYS))
        st = ctx.stats()
        assert st.trace_rays + st.shadow_rays == total
    finally:
        ds.close()


def test_batch_rejects_mismatched_cameras(ctx):
    sc = make_config("c2", 64, 32)
    ds = ctx.scene(sc)
    try:
        cams = ds.cameras(np.repeat(ds.camera["position"], 2, axis=0))
        cams["width"][1] = 65
        buf = torch.empty(2 * 65 * 32 * 3, dtype=torch.float64, device="cuda")
        with pytest.raises(capi.RtError) as e:
            ds.render_batch(cams, buf.data_ptr(), None, None, capi.default_opts(tonemap=-1))
        assert e.value.status == capi.RT_ERR_INVALID_ARG
        with pytest.raises(capi.RtError) as e:
            ds.render_batch(cams[:0], buf.data_ptr(), None, None, capi.default_opts(tonemap=-1))
        assert e.value.status == capi.RT_ERR_INVALID_ARG
    finally:
        ds.close()


# ------------------------------------------------------------------ gathered batches
@pytest.fixture(scope="module")
def comm1(ctx):
    c = capi.Comm(ctx, 1, 0, capi.comm_unique_id())
    yield c
    c.close()


@pytest.mark.parametrize("pipeline", [False, True])
def test_gather_batch_one_rank_ldr_gathered_hdr_local(ctx, comm1, pipeline):
    """The bench's step at N = 1: rt_render_gather_batch with the Reinhard bytes gathered
    (here: rendered straight into the frame) and the f64 HDR kept rank-local; three batches in
    a row through the pipelined slots.  Every frame = its single render."""
    sc = make_config("c2", 480, 270)
    W, H, n = 480, 270, 4
    ds = ctx.scene(sc)
    try:
        pos = _positions(ds, n, seed=5)
        opts = capi.default_opts(tonemap=1, flags=capi.RT_FLAG_PIPELINE if pipeline else 0)
        refs = [_single(ds, p, capi.default_opts(tonemap=1), H, W) for p in pos]
        outs = []
        for b in range(3):
            L8 = torch.zeros(n * H * W * 3, dtype=torch.uint8, device="cuda")
            R64 = torch.zeros(n * H * W * 3, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            comm1.render_gather_batch(ds, ds.cameras(pos), opts, capi.RT_OUT_LDR,
                                      d_ldr=L8.data_ptr(), rank_hdr64=R64.data_ptr())
            outs.append((L8, R64))
        comm1.synchronize()
        ctx.synchronize()
        for b, (L8, R64) in enumerate(outs):
            a8 = L8.cpu().numpy().reshape(n, -1)
            a64 = R64.cpu().numpy().reshape(n, -1)
            for f in range(n):
                assert np.array_equal(a8[f], refs[f][1]), (b, f)
                assert np.array_equal(a64[f], refs[f][0]), (b, f)
    finally:
        ds.close()


def test_gather_batch_rejects_gathered_and_local_output(ctx, comm1):
    sc = make_config("c2", 64, 32)
    ds = ctx.scene(sc)
    try:
        buf = torch.empty(64 * 32 * 3, dtype=torch.float64, device="cuda")
        with pytest.raises(capi.RtError) as e:
            comm1.render_gather_batch(ds, ds.cameras(ds.camera["position"]),
                                      capi.default_opts(tonemap=-1), capi.RT_OUT_HDR64,
                                      d_hdr64=buf.data_ptr(), rank_hdr64=buf.data_ptr())
        assert e.value.status == capi.RT_ERR_INVALID_ARG
    finally:
        ds.close()


@pytest.mark.parametrize("name,w,h,ranks,block,nf", [("c2", 480, 270, 8, 16, 4),
                                                     ("c2", 160, 90, 3, 16, 34),  # 32 + 2 frames per launch
                                                     ("c2", 480, 270, 3, 16, 5),
                                                     ("c3", 320, 180, 4, 8, 3),
                                                     ("c2", 200, 40, 4, 16, 2)])
def test_gather_all_batch_local_ranks_is_the_frames(name, w, h, ranks, block, nf):
    """The multi-rank batch on one GPU through local communicators: every rank renders its
    block-cyclic rows of every frame in one launch into a padded send buffer (frame f at
    f·max_rows), the whole batch moves in one copy per rank (ONE ncclGather on RCCL
    communicators), rank 0 receives [n][frames][max_rows] rows and assembles all frames in one
    launch.  Ranks with fewer rows (200x40 over 4 ranks of 16-row blocks:
    one rank has none) included.  Every frame = the single-rank frame."""
    ctxs = [capi.Context(0) for _ in range(ranks)]
    try:
        comms = capi.Comm.create_local(ctxs)
        sc = make_config(name, w, h)
        scenes = [c.scene(sc) for c in ctxs]
        pos = _positions(scenes[0], nf, seed=13)
        refs = [_single(scenes[0], p, capi.default_opts(tonemap=1), h, w) for p in pos]
        for pipeline in (False, True):
            opts = capi.default_opts(tonemap=1, row_block=block,
                                     flags=capi.RT_FLAG_PIPELINE if pipeline else 0)
            L8 = torch.zeros(nf * h * w * 3, dtype=torch.uint8, device="cuda")
            H64 = torch.zeros(nf * h * w * 3, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            capi.render_gather_all_batch(comms, scenes, scenes[0].cameras(pos), opts,
                                         capi.RT_OUT_LDR | capi.RT_OUT_HDR64,
                                         d_hdr64=H64.data_ptr(), d_ldr=L8.data_ptr())
            for c in comms:
                c.synchronize()
            a8 = L8.cpu().numpy().reshape(nf, -1)
            a64 = H64.cpu().numpy().reshape(nf, -1)
            for f in range(nf):
                assert np.array_equal(a8[f], refs[f][1]), (pipeline, f)
                assert np.array_equal(a64[f], refs[f][0]), (pipeline, f)
        for s in scenes:
            s.close()
        for c in comms:
            c.close()
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("name,w,h,ranks,block,nf,weight", [
    ("c2", 480, 270, 8, 16, 4, 3), ("c2", 480, 270, 2, 16, 3, 2), ("c3", 320, 180, 4, 8, 3, 4),
    ("c2", 200, 40, 4, 16, 2, 2),   # some row sets empty
    ("c2", 160, 90, 3, 16, 34, 2),  # 32 + 2 frames per row set
    ("glass", 160, 120, 3, 16, 2, 2)])
def test_gather_all_batch_weighted_root_is_the_frames(name, w, h, ranks, block, nf, weight):
    """The weighted split (rt_comm_set_root_weight): the blocks dealt over weight + n − 1 row
    sets, rank 0 renders `weight` of them straight into its receive buffer, every other rank
    one, moved into place by the gather (device copies here; P2P sends on RCCL communicators),
    then the same assembly.  Every frame = the single-rank frame, pipelined or not, and the
    communicators switch back to weight 1 between frames."""
    ctxs = [capi.Context(0) for _ in range(ranks)]
    try:
        comms = capi.Comm.create_local(ctxs)
        sc = make_config(name, w, h)
        scenes = [c.scene(sc) for c in ctxs]
        pos = _positions(scenes[0], nf, seed=17)
        refs = [_single(scenes[0], p, capi.default_opts(tonemap=1), h, w) for p in pos]
        for wt, pipeline in ((weight, False), (weight, True), (1, True)):
            for c in comms:
                c.set_root_weight(wt)
            opts = capi.default_opts(tonemap=1, row_block=block,
                                     flags=capi.RT_FLAG_PIPELINE if pipeline else 0)
            L8 = torch.zeros(nf * h * w * 3, dtype=torch.uint8, device="cuda")
            H64 = torch.zeros(nf * h * w * 3, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            capi.render_gather_all_batch(comms, scenes, scenes[0].cameras(pos), opts,
                                         capi.RT_OUT_LDR | capi.RT_OUT_HDR64,
                                         d_hdr64=H64.data_ptr(), d_ldr=L8.data_ptr())
            for c in comms:
                c.synchronize()
            a8 = L8.cpu().numpy().reshape(nf, -1)
            a64 = H64.cpu().numpy().reshape(nf, -1)
            for f in range(nf):
                assert np.array_equal(a8[f], refs[f][1]), (wt, pipeline, f)
                assert np.array_equal(a64[f], refs[f][0]), (wt, pipeline, f)
        with pytest.raises(capi.RtError) as e:
            comms[0].set_root_weight(0)
        assert e.value.status == capi.RT_ERR_INVALID_ARG
        for s in scenes:
            s.close()
        for c in comms:
            c.close()
    finally:
        for c in ctxs:
            c.close()


def test_moving_batches_on_two_streams_reuse_the_image_ring(ctx):
    """Batches of first-seen cameras (a camera that moves every frame) get every frame's packet
    image formed by one small launch into a ring entry (rt_capi.cpp enqueue_frames, 4 entries)
    that the batch launch reads like cached images.  Seven batches alternating between two
    streams, enqueued without waiting, wrap the ring twice: every frame equals its single
    render."""
    sc = make_config("c2", 320, 180)
    W, H, n = 320, 180, 4
    ds = ctx.scene(sc)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    base = ds.camera["position"][0].copy()
    try:
        batches = [[base + (0.01 * (b * n + f + 1), -0.005 * f, 0.02 * b) for f in range(n)]
                   for b in range(7)]
        opts = capi.default_opts(tonemap=1)
        outs = []
        for b, pos in enumerate(batches):
            ctx.set_stream(streams[b % 2].cuda_stream)
            h = torch.empty(n * H * W * 3, dtype=torch.float64, device="cuda")
            l = torch.empty(n * H * W * 3, dtype=torch.uint8, device="cuda")
            ds.render_batch(ds.cameras(np.array(pos)), h.data_ptr(), None, l.data_ptr(), opts)
            outs.append((h, l))
        torch.cuda.synchronize()
        ctx.set_stream(None)
        for b, pos in enumerate(batches):
            h, l = outs[b]
            a64 = h.cpu().numpy().reshape(n, -1)
            a8 = l.cpu().numpy().reshape(n, -1)
            for f, p in enumerate(pos):
                r64, r8 = _single(ds, p, capi.default_opts(tonemap=1), H, W)
                assert np.array_equal(a64[f], r64), (b, f)
                assert np.array_equal(a8[f], r8), (b, f)
    finally:
        ctx.set_stream(None)
        ds.camera["position"][0] = base
        ds.close()


# ------------------------------------------------------------------ the bench's launch shapes
@pytest.mark.parametrize("nf", [32, 20])
def test_batch_full_c2_bench_launch_shape_is_the_reference(ctx, golden, nf):
    """The bench's own launch at full size: ONE 1920x1080 C2 launch of 32 static-camera frames
    (the default batch) and of 20 (the driver's `--steps 20` timed region): every frame's HDR and
    Reinhard bytes have the reference's SHA-256, on the fresh-camera, cache-creating and cached
    launches (RE/Scene.h:311-328)."""
    info = golden["meta"]["scenes"]["c2_full"]
    sc = make_config("c2")
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    try:
        cams = ds.cameras(np.repeat(ds.camera["position"], nf, axis=0))
        H64 = torch.empty(nf * H * W * 3, dtype=torch.float64, device="cuda")
        L8 = torch.empty(nf * H * W * 3, dtype=torch.uint8, device="cuda")
        for rnd in range(3):
            H64.fill_(-1.0)
            L8.zero_()
            torch.cuda.synchronize()
            ds.render_batch(cams, H64.data_ptr(), None, L8.data_ptr(), capi.default_opts(tonemap=1))
            ctx.synchronize()
            a64 = H64.cpu().numpy().reshape(nf, -1)
            a8 = L8.cpu().numpy().reshape(nf, -1)
            for f in range(nf):
                assert _sha(a64[f]) == info["image_sha256"], (rnd, f)
                assert _sha(a8[f]) == info["ldr_sha256"]["reinhard_simple"], (rnd, f)
    finally:
        ds.close()


def test_batch_full_c2_moving_camera_revisits_vs_oracle(ctx, oracle):
    """A 1920x1080 C2 batch of 32 frames whose camera moves every frame and revisits 5 positions
    an earlier batch rendered (second sightings: their images become cache entries inside the
    batch's one image launch, no launch of their own), plus a frame repeated inside the batch.
    Every frame equals the C oracle rendering its camera, bit for bit (HDR), and the Reinhard
    bytes equal the oracle's tonemap; a second pass (every image cached now) gives the same."""
    sc = make_config("c2")
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    base = np.array(sc.camera.position)
    try:
        early = [base + (0.013 * (i + 1), -0.007 * i, 0.011 * i) for i in range(5)]
        warm = torch.empty(5 * H * W * 3, dtype=torch.uint8, device="cuda")
        ds.render_batch(ds.cameras(np.array(early)), None, None, warm.data_ptr(),
                        capi.default_opts(tonemap=1))
        ctx.synchronize()
        fresh = [base + (-0.02 * (i + 1), 0.004 * i, -0.009 * i) for i in range(26)]
        pos = np.array(early + fresh[:13] + [fresh[3]] + fresh[13:])  # frame 18 repeats 8
        assert len(pos) == 32
        H64 = torch.empty(32 * H * W * 3, dtype=torch.float64, device="cuda")
        L8 = torch.empty(32 * H * W * 3, dtype=torch.uint8, device="cuda")
        got = []
        for rnd in range(2):
            H64.fill_(-1.0)
            L8.zero_()
            torch.cuda.synchronize()
            ds.render_batch(ds.cameras(pos), H64.data_ptr(), None, L8.data_ptr(),
                            capi.default_opts(tonemap=1))
            ctx.synchronize()
            got.append((H64.cpu().numpy().reshape(32, H, W, 3), L8.cpu().numpy().reshape(32, -1)))
    finally:
        ds.close()
    for f in range(32):
        scf = dataclasses.replace(sc, camera=dataclasses.replace(sc.camera,
                                                                 position=tuple(pos[f])))
        ref, _, _ = oracle.render(scf)
        ref8 = oracle.tonemap(ref, 1).reshape(-1)
        for rnd in range(2):
            assert np.array_equal(got[rnd][0][f], ref), (rnd, f)
            assert np.array_equal(got[rnd][1][f], ref8), (rnd, f)


def test_gather_all_batch_rejects_unequal_root_weights():
    """Every rank must plan the same split: a weight set on rank 0 only (or on the peers only)
    is an invalid argument, never a copy past a peer's send buffer."""
    ctxs = [capi.Context(0) for _ in range(3)]
    try:
        comms = capi.Comm.create_local(ctxs)
        sc = make_config("c2", 160, 90)
        scenes = [c.scene(sc) for c in ctxs]
        L8 = torch.zeros(90 * 160 * 3, dtype=torch.uint8, device="cuda")
        opts = capi.default_opts(tonemap=1, row_block=16)
        for who in ([0], [1, 2]):
            for i in who:
                comms[i].set_root_weight(3)
            with pytest.raises(capi.RtError) as e:
                capi.render_gather_all_batch(comms, scenes, scenes[0].cameras(
                    scenes[0].camera["position"]), opts, capi.RT_OUT_LDR, d_ldr=L8.data_ptr())
            assert e.value.status == capi.RT_ERR_INVALID_ARG
            assert "root weight" in str(e.value)
            for c in comms:
                c.set_root_weight(1)
        capi.render_gather_all_batch(comms, scenes, scenes[0].cameras(
            scenes[0].camera["position"]), opts, capi.RT_OUT_LDR, d_ldr=L8.data_ptr())
        for c in comms:
            c.synchronize()
        ref = scenes[0].render(tonemap=1)["ldr"]
        assert np.array_equal(L8.cpu().numpy().reshape(90, 160, 3), ref)
        for s in scenes:
            s.close()
        for c in comms:
            c.close()
    finally:
        for c in ctxs:
            c.close()


# ------------------------------------------------------------------ the fix-up variant (C2)
@pytest.mark.parametrize("name,w,h,n", [("c2", 1920, 1080, 8), ("c2", 1920, 1080, 32),
                                        ("c2", 480, 270, 9), ("c2", 97, 61, 12),
                                        ("c2", 480, 270, 4)])
def test_fixup_variant_equals_marching_variant(ctx, monkeypatch, name, w, h, n):
    """The fix-up variant of the packet kernel (C2's shape: single sample, <= 64 spheres, no
    other feature) does not march undecided shadow rays; their pixels are queued and re-rendered
    by packet_fixup_kernel with the exact per-pixel path (batches of >= 32 M pixels, or any batch
    with RTAMD_PK_FIX=1 as here).  Every
    frame (HDR, float3 and Reinhard bytes) equals the marching variant's (RTAMD_PK_FIX=0): moving
    and repeated cameras, a row set of the multi-GPU split, an odd-sized frame (lanes past the
    edge)."""
    sc = make_config(name, w, h)
    ds = ctx.scene(sc)
    try:
        pos = _positions(ds, n, seed=23)
        for opts in (capi.default_opts(tonemap=1),
                     capi.default_opts(tonemap=1, row_begin=16, row_end=h, row_block=16,
                                       row_cycle=3)):
            rows = capi.rendered_rows(opts, h)
            outs = {}
            for fix in ("1", "0"):
                monkeypatch.setenv("RTAMD_PK_FIX", fix)
                H64 = torch.full((n * rows * w * 3,), -1.0, dtype=torch.float64, device="cuda")
                H32 = torch.full((n * rows * w * 3,), -1.0, dtype=torch.float32, device="cuda")
                L8 = torch.zeros(n * rows * w * 3, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                ds.render_batch(ds.cameras(pos), H64.data_ptr(), H32.data_ptr(), L8.data_ptr(),
                                opts)
                ctx.synchronize()
                outs[fix] = (H64.cpu().numpy(), H32.cpu().numpy(), L8.cpu().numpy())
            for a, b in zip(outs["1"], outs["0"]):
                assert np.array_equal(a, b)
    finally:
        ds.close()


def test_fixup_variant_vs_oracle_on_undecided_shadows(ctx, oracle, monkeypatch):
    """A scene built to leave many shadow rays undecided (spheres resting on the floor and
    touching each other, the light just above them): the fix-up variant's frame equals the C
    oracle bit for bit."""
    monkeypatch.setenv("RTAMD_PK_FIX", "1")  # the fix-up variant at this small size
    from raytracingengine_amd.scene import Camera, Material, SceneData
    sc = SceneData(Camera((0.0, 0.0, -25.0), 160.0, 320, 180, 0.0, 200.0, 1), name="touching")
    for i in range(8):
        sc.add_sphere((-7.0 + 2.0 * i, -9.0, 3.0), 1.0, Material((0.8, 0.3 + 0.05 * i, 0.4)))
        sc.add_sphere((-7.0 + 2.0 * i, -7.0, 3.0), 1.0, Material((0.3, 0.7, 0.2 + 0.05 * i)))
    sc.add_plane((0.0, -10.0, 0.0), (0.0, 1.0, 0.0), Material((0.9, 0.9, 0.9)))
    sc.add_plane((0.0, 0.0, 15.0), (0.0, 0.0, -1.0), Material((0.7, 0.8, 0.9)))
    sc.add_light((0.3, -5.9, 3.0), (1.0, 1.0, 1.0), 40.0)
    ds = ctx.scene(sc)
    n = 8  # a batch
    try:
        H64 = torch.empty(n * 180 * 320 * 3, dtype=torch.float64, device="cuda")
        L8 = torch.empty(n * 180 * 320 * 3, dtype=torch.uint8, device="cuda")
        ds.render_batch(ds.cameras(np.repeat(ds.camera["position"], n, axis=0)), H64.data_ptr(),
                        None, L8.data_ptr(), capi.default_opts(tonemap=1))
        ctx.synchronize()
        got64 = H64.cpu().numpy().reshape(n, 180, 320, 3)
        got8 = L8.cpu().numpy().reshape(n, -1)
    finally:
        ds.close()
    ref, _, _ = oracle.render(sc)
    ref8 = oracle.tonemap(ref, 1).reshape(-1)
    for f in range(n):
        assert np.array_equal(got64[f], ref), f
        assert np.array_equal(got8[f], ref8), f


@pytest.mark.parametrize("pipeline,block", [(True, 16), (False, 16), (True, 8)])
def test_c4_own_shape_8_local_ranks_is_the_reference(ctx, golden, pipeline, block):
    """BASELINE config 4 in its own shape: 7680x4320, 256 spheres, 8 point lights, split over 8
    ranks in block-cyclic 16-row blocks, and in the bench's default 8-row blocks (each 16x16-px
    workgroup of the 256-thread variant then spans two blocks), through 8 local communicators on this one GPU (rt_comm_create_local: the gather as
    device copies, the same plan, padded send rows and assembly launch as the RCCL path).  Three
    calls of 2 static-camera frames — first sighting (publish slots), cache-creating and cached
    camera — and every assembled frame's HDR and Reinhard bytes have the reference's SHA-256
    (RE/Scene.h:311-328; golden_meta.json c4_full)."""
    info = golden["meta"]["scenes"]["c4_full"]
    n, nf = 8, 2  # (8-row blocks: the bench's default; each 16-row workgroup spans two)
    ctxs = [capi.Context(0) for _ in range(n)]
    try:
        comms = capi.Comm.create_local(ctxs)
        sc = make_config("c4")
        W, H = sc.camera.width, sc.camera.height
        assert (W, H) == (info["width"], info["height"])
        scenes = [c.scene(sc) for c in ctxs]
        cams = scenes[0].cameras(np.repeat(scenes[0].camera["position"], nf, axis=0))
        opts = capi.default_opts(tonemap=1, row_block=block,
                                 flags=capi.RT_FLAG_PIPELINE if pipeline else 0)
        H64 = torch.empty(nf * H * W * 3, dtype=torch.float64, device="cuda")
        L8 = torch.empty(nf * H * W * 3, dtype=torch.uint8, device="cuda")
        first = None
        for rnd in range(3):
            H64.fill_(-1.0)
            L8.zero_()
            torch.cuda.synchronize()
            capi.render_gather_all_batch(comms, scenes, cams, opts,
                                         capi.RT_OUT_LDR | capi.RT_OUT_HDR64,
                                         d_hdr64=H64.data_ptr(), d_ldr=L8.data_ptr())
            for c in comms:
                c.synchronize()
            torch.cuda.synchronize()
            h = H64.view(nf, -1)
            l8 = L8.view(nf, -1)
            if first is None:
                # the SHA of the first frame on the host, every other frame equal to it on the GPU
                assert _sha(h[0].cpu().numpy()) == info["image_sha256"]
                assert _sha(l8[0].cpu().numpy()) == info["ldr_sha256"]["reinhard_simple"]
                first = (h[0].clone(), l8[0].clone())
            for f in range(nf):
                assert torch.equal(h[f], first[0]), (rnd, f)
                assert torch.equal(l8[f], first[1]), (rnd, f)
        del H64, L8, first
        for s in scenes:
            s.close()
        for c in comms:
            c.close()
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("fix", ["1", "0"])
def test_zero_step_shadow_origins_vs_oracle(ctx, oracle, monkeypatch, fix):
    """Shadow origins lying exactly on a plane: in C2 the ~1 600 floor hits of row 780, where the
    floor meets the back wall (z = 15), start their shadow ray on the back wall, whose t = ±0 is
    the march's first closest hit (Scene.h:51-55: origin += direction·bias, traveled = bias) —
    every undecided lane of a C2 frame is one of them (the packet classifier leaves them to the
    exact march, or in the fix-up variant to packet_fixup_kernel).  With C2's own light and two
    lights placed just above two such pixels — one closer than 2·bias (traveled = bias >=
    maxDist ends the march: clear) and one a little farther — the rows around the corner equal
    the C oracle bit for bit, through the fix-up variant (a batch) and the marching variant."""
    monkeypatch.setenv("RTAMD_PK_FIX", fix)
    sc = make_config("c2")
    # floor / back-wall corner pixels of row 780 (P = (x − 960)/24, −10, 15) for x = 874, 1614
    sc.add_light((-3.5833333333333335, -10.0 + 1.5e-3, 15.0 - 2e-4), (1.0, 1.0, 1.0), 0.5)
    sc.add_light((27.25, -10.0 + 3e-3, 15.0 - 1e-3), (1.0, 0.5, 0.25), 0.5)
    W, r0, r1 = sc.camera.width, 776, 784
    rows = r1 - r0
    ds = ctx.scene(sc)
    n = 2 if fix == "1" else 1
    try:
        opts = capi.default_opts(tonemap=1, row_begin=r0, row_end=r1)
        H64 = torch.full((n * rows * W * 3,), -1.0, dtype=torch.float64, device="cuda")
        L8 = torch.zeros(n * rows * W * 3, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        if n > 1:
            ds.render_batch(ds.cameras(np.repeat(ds.camera["position"], n, axis=0)),
                            H64.data_ptr(), None, L8.data_ptr(), opts)
        else:
            ds.render_device(H64.data_ptr(), None, L8.data_ptr(), opts)
        ctx.synchronize()
        got64 = H64.cpu().numpy().reshape(n, rows, W, 3)
        got8 = L8.cpu().numpy().reshape(n, -1)
    finally:
        ds.close()
    ref, _, _ = oracle.render(sc, rows=(r0, r1))
    ref8 = oracle.tonemap(ref, 1).reshape(-1)
    for f in range(n):
        assert np.array_equal(got64[f], ref), f
        assert np.array_equal(got8[f], ref8), f
