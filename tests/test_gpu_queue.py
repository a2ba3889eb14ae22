"""The serving frame queue (rt_queue, include/rt_capi.h): frames with several in flight on
separate HIP streams are the frames rt_render gives — the reference's, at full size — including
the per-camera packet image created by one stream's frame and read by another's."""
import hashlib

import numpy as np
import pytest
import torch

from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_queue_frames_equal_synchronous_renders(ctx, depth):
    """Alternating camera positions, frames in flight on `depth` streams, each into its own
    framebuffers: every frame equals the synchronous render of its camera (HDR bits, bytes)."""
    sc = make_config("c3", 480, 270)
    ds = ctx.scene(sc)
    q = capi.Queue(ctx, depth)
    W, H = sc.camera.width, sc.camera.height
    base = ds.camera["position"][0].copy()
    cams = [base, base + (0.5, -0.25, 1.0)]
    try:
        ref = []
        for c in cams:
            ds.camera["position"][0] = c
            ref.append(ds.render(hdr64=True, tonemap=1))
        n = 8
        bufs = [(torch.empty(H * W * 3, dtype=torch.float64, device="cuda"),
                 torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")) for _ in range(n)]
        opts = capi.default_opts(tonemap=1)
        tickets = []
        for i in range(n):
            ds.camera["position"][0] = cams[i % 2]
            h, l = bufs[i]
            tickets.append(q.submit(ds, opts, h.data_ptr(), None, l.data_ptr()))
        assert tickets == list(range(n))
        for i in range(n):
            q.wait(tickets[i])
            h, l = bufs[i]
            r = ref[i % 2]
            assert np.array_equal(h.cpu().numpy().reshape(H, W, 3), r["hdr64"]), i
            assert np.array_equal(l.cpu().numpy().reshape(H, W, 3), r["ldr"]), i
        q.synchronize()
    finally:
        ds.camera["position"][0] = base
        q.close()
        ds.close()


def test_queue_full_c2_matches_reference(ctx, golden):
    """The bench's frame (C2 1920x1080, f64 HDR + fused Reinhard) through a depth-2 queue, four
    frames on two framebuffer sets: each the reference's frame (SHA-256 of HDR and bytes)."""
    info = golden["meta"]["scenes"]["c2_full"]
    sc = make_config("c2")
    ds = ctx.scene(sc)
    q = capi.Queue(ctx, 2)
    W, H = sc.camera.width, sc.camera.height
    bufs = [(torch.empty(H * W * 3, dtype=torch.float64, device="cuda"),
             torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")) for _ in range(2)]
    opts = capi.default_opts(tonemap=1)
    try:
        for rnd in range(2):
            ts = [q.submit(ds, opts, h.data_ptr(), None, l.data_ptr()) for h, l in bufs]
            for t, (h, l) in zip(ts, bufs):
                q.wait(t)
                assert _sha(h.cpu().numpy()) == info["image_sha256"], (rnd, t)
                assert _sha(l.cpu().numpy()) == info["ldr_sha256"]["reinhard_simple"], (rnd, t)
    finally:
        q.close()
        ds.close()


def test_queue_alternating_launch_shapes_keep_their_tile_orders(ctx):
    """One camera, launches of different shapes in flight together on three streams: whole
    frames at two resolutions, a block-cyclic row set and a contiguous row range.  Each shape
    records, builds and then dispatches by its own costliest-first tile order (rt_capi.cpp
    tile_order: one entry per shape, never rewritten while a launch of another shape may read
    it).  Every frame equals the synchronous render of its shape."""
    sc = make_config("c3", 640, 360)
    ds = ctx.scene(sc)
    q = capi.Queue(ctx, 3)
    W, H = sc.camera.width, sc.camera.height
    shapes = [((W, H), capi.default_opts(tonemap=1)),
              ((W // 2, H // 2), capi.default_opts(tonemap=1)),
              ((W, H), capi.default_opts(tonemap=1, row_begin=16, row_end=H, row_block=16,
                                         row_cycle=3)),
              ((W, H), capi.default_opts(tonemap=1, row_begin=40, row_end=200))]
    try:
        refs = []
        for (w, h), o in shapes:
            ds.camera["width"], ds.camera["height"] = w, h
            rows = capi.rendered_rows(o, h)
            hd = torch.empty(rows * w * 3, dtype=torch.float64, device="cuda")
            ld = torch.empty(rows * w * 3, dtype=torch.uint8, device="cuda")
            ds.render_device(hd.data_ptr(), None, ld.data_ptr(), o)
            ctx.synchronize()
            refs.append((hd.cpu().numpy(), ld.cpu().numpy()))
        n = 24   # every shape: cache creation, recording, order build, ordered launches
        bufs = []
        for i in range(n):
            k = i % len(shapes)
            (w, h), o = shapes[k]
            ds.camera["width"], ds.camera["height"] = w, h
            rows = capi.rendered_rows(o, h)
            hd = torch.empty(rows * w * 3, dtype=torch.float64, device="cuda")
            ld = torch.empty(rows * w * 3, dtype=torch.uint8, device="cuda")
            q.submit(ds, o, hd.data_ptr(), None, ld.data_ptr())
            bufs.append((k, hd, ld))
        q.synchronize()
        for i, (k, hd, ld) in enumerate(bufs):
            assert np.array_equal(hd.cpu().numpy(), refs[k][0]), (i, k)
            assert np.array_equal(ld.cpu().numpy(), refs[k][1]), (i, k)
    finally:
        ds.camera["width"], ds.camera["height"] = W, H
        q.close()
        ds.close()


def test_queue_rejects_bad_arguments(ctx):
    with pytest.raises(capi.RtError) as e:
        capi.Queue(ctx, 0)
    assert e.value.status == capi.RT_ERR_INVALID_ARG
    q = capi.Queue(ctx, 2)
    try:
        with pytest.raises(capi.RtError) as e:
            q.wait(0)                       # nothing submitted yet
        assert e.value.status == capi.RT_ERR_INVALID_ARG
    finally:
        q.close()


@pytest.mark.parametrize("depth", [2, 3])
def test_queue_refraction_tree_frames_share_the_arena_safely(ctx, depth):
    """Glass (refraction trees) renders breadth-first through ONE arena per context: queued frames
    of such scenes are serialised behind each other on any stream (rt_queue.cpp), interleaved
    with packet frames (C2) that are not.  Every frame equals its synchronous render, including
    a camera move between glass frames (different trees, different arena fill)."""
    glass = ctx.scene(make_config("glass", 320, 180))
    c2 = ctx.scene(make_config("c2", 320, 180))
    q = capi.Queue(ctx, depth)
    W, H = 320, 180
    base = glass.camera["position"][0].copy()
    cams = [base, base + (0.75, 0.5, 2.0)]
    try:
        ref_g = []
        for c in cams:
            glass.camera["position"][0] = c
            ref_g.append(glass.render(hdr64=True, tonemap=1))
        ref_c2 = c2.render(hdr64=True, tonemap=1)
        n = 9
        bufs = [(torch.empty(H * W * 3, dtype=torch.float64, device="cuda"),
                 torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")) for _ in range(n)]
        opts = capi.default_opts(tonemap=1)
        kinds = []
        for i in range(n):
            h, l = bufs[i]
            if i % 3 == 2:
                kinds.append(None)
                q.submit(c2, opts, h.data_ptr(), None, l.data_ptr())
            else:
                glass.camera["position"][0] = cams[i % 2]
                kinds.append(i % 2)
                q.submit(glass, opts, h.data_ptr(), None, l.data_ptr())
        q.synchronize()
        for i, (h, l) in enumerate(bufs):
            r = ref_c2 if kinds[i] is None else ref_g[kinds[i]]
            assert np.array_equal(h.cpu().numpy().reshape(H, W, 3), r["hdr64"]), i
            assert np.array_equal(l.cpu().numpy().reshape(H, W, 3), r["ldr"]), i
    finally:
        glass.camera["position"][0] = base
        q.close()
        glass.close()
        c2.close()


def test_arena_shared_by_queue_and_context_stream(ctx):
    """The breadth-first arena is one per context: a refraction-tree render on the context's own
    stream (rt_render_device) between queued ones on other streams is ordered behind them and
    they behind it (rt_capi.cpp scratch_wait / scratch_done), whatever API enqueued each render.
    Every frame equals its synchronous render."""
    glass = ctx.scene(make_config("glass", 240, 135))
    q = capi.Queue(ctx, 2)
    W, H = 240, 135
    base = glass.camera["position"][0].copy()
    cams = [base, base + (0.5, 0.25, 1.5), base + (-0.5, 0.0, 0.75)]
    try:
        ref = []
        for c in cams:
            glass.camera["position"][0] = c
            ref.append(glass.render(hdr64=True, tonemap=1))
        opts = capi.default_opts(tonemap=1)
        bufs, kinds = [], []
        for i in range(9):
            k = i % 3
            glass.camera["position"][0] = cams[k]
            h = torch.empty(H * W * 3, dtype=torch.float64, device="cuda")
            l = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
            if k == 2:
                glass.render_device(h.data_ptr(), None, l.data_ptr(), opts)  # context stream
            else:
                q.submit(glass, opts, h.data_ptr(), None, l.data_ptr())
            bufs.append((h, l))
            kinds.append(k)
        q.synchronize()
        ctx.synchronize()
        for i, (h, l) in enumerate(bufs):
            assert np.array_equal(h.cpu().numpy().reshape(H, W, 3), ref[kinds[i]]["hdr64"]), i
            assert np.array_equal(l.cpu().numpy().reshape(H, W, 3), ref[kinds[i]]["ldr"]), i
    finally:
        glass.camera["position"][0] = base
        q.close()
        glass.close()
