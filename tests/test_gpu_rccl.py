"""The RCCL multi-GPU frame path behind the C-ABI (rt_multi.cpp; SURVEY.md §8e, RE/Scene.h:318-325).

The test box has ONE MI355X and RCCL allows one rank per GPU, so the collective itself runs here
with n = 1 (rank 0 gathers from itself over the same code path: render into the send buffer,
ncclGather, assembly into image order); the row plans of n > 1 ranks are pinned through the
assembly hook (rt_debug_assemble_rows) against the Python row planner, and the multi-rank
gather end-to-end runs on CPU with gloo (tests/test_distributed_cpu.py).
"""
import hashlib

import numpy as np
import pytest
import torch

from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
from raytracingengine_amd.distributed import plan_rows, row_ranges

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def comm1(ctx):
    c = capi.Comm(ctx, 1, 0, capi.comm_unique_id())
    yield c
    c.close()


@pytest.mark.parametrize("name,w,h", [("c2", 1920, 1080), ("c3", 640, 360), ("c5", 320, 180),
                                      ("mirror", 320, 180), ("glass", 200, 120)])
def test_render_gather_one_rank_equals_render(ctx, comm1, name, w, h):
    """rt_render_gather on a 1-rank communicator (ncclCommInitRank) = rt_render, every output."""
    sc = make_config(name, w, h)
    ds = ctx.scene(sc)
    try:
        ref = ds.render(hdr64=True, hdr32=True, tonemap=1)
        d64 = torch.empty(h * w * 3, dtype=torch.float64, device="cuda")
        d32 = torch.empty(h * w * 3, dtype=torch.float32, device="cuda")
        d8 = torch.empty(h * w * 3, dtype=torch.uint8, device="cuda")
        outs = capi.RT_OUT_HDR64 | capi.RT_OUT_HDR32 | capi.RT_OUT_LDR
        for k in range(2):
            for t in (d64, d32, d8):
                t.zero_()
            comm1.render_gather(ds, capi.default_opts(tonemap=1, flags=capi.RT_FLAG_TIME_KERNEL),
                                outs, d64.data_ptr(), d32.data_ptr(), d8.data_ptr())
            ctx.synchronize()
            assert np.array_equal(d64.cpu().numpy().reshape(h, w, 3), ref["hdr64"]), k
            assert np.array_equal(d32.cpu().numpy().reshape(h, w, 3), ref["hdr32"]), k
            assert np.array_equal(d8.cpu().numpy().reshape(h, w, 3), ref["ldr"]), k
    finally:
        ds.close()
    t = comm1.timing(reset=True)
    assert t.frames == 2 and t.rows == h and t.max_rows == h
    assert t.render_ms > 0 and t.gather_ms >= 0 and t.assemble_ms > 0


def test_render_gather_ldr_only_full_c4(ctx, comm1, golden):
    """The bench's tiled frame (C4 7680x4320, fused Reinhard bytes only) through the gather:
    the reference's bytes."""
    sc = make_config("c4")
    W, H = sc.camera.width, sc.camera.height
    ds = ctx.scene(sc)
    try:
        d8 = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
        comm1.render_gather(ds, capi.default_opts(tonemap=1), capi.RT_OUT_LDR, None, None,
                            d8.data_ptr())
        ctx.synchronize()
    finally:
        ds.close()
    assert _sha(d8.cpu().numpy()) == golden["meta"]["scenes"]["c4_full"]["ldr_sha256"][
        "reinhard_simple"]


def test_render_gather_rejects_bad_arguments(ctx, comm1):
    sc = make_config("c2", 64, 32)
    ds = ctx.scene(sc)
    try:
        buf = torch.empty(64 * 32 * 3, dtype=torch.uint8, device="cuda")
        with pytest.raises(capi.RtError):  # no outputs
            comm1.render_gather(ds, capi.default_opts(tonemap=1), 0)
        with pytest.raises(capi.RtError):  # rank 0 without its framebuffer
            comm1.render_gather(ds, capi.default_opts(tonemap=1), capi.RT_OUT_LDR)
        with pytest.raises(capi.RtError):  # LDR without an operator
            comm1.render_gather(ds, capi.default_opts(tonemap=-1), capi.RT_OUT_LDR, None, None,
                                buf.data_ptr())
        with pytest.raises(capi.RtError):  # the row split is the communicator's
            comm1.render_gather(ds, capi.default_opts(tonemap=1, row_begin=8), capi.RT_OUT_LDR,
                                None, None, buf.data_ptr())
    finally:
        ds.close()
    with pytest.raises(capi.RtError):
        capi.Comm(ctx, 2, 2, capi.comm_unique_id())


def test_comm_create_all_one_device_and_render_multi(ctx):
    """rt_comm_create_all (ncclCommInitAll) over the box's device, rt_render_gather_all, and the
    drop-in rt_render_multi over distinct devices (here: the one) — all equal rt_render."""
    sc = make_config("c3", 480, 270)
    W, H = 480, 270
    c0 = capi.Context(0)
    try:
        comms = capi.Comm.create_all([c0])
        ds = c0.scene(sc)
        ref = ds.render(hdr64=True, tonemap=6, stats=True)
        d64 = torch.empty(H * W * 3, dtype=torch.float64, device="cuda")
        capi.render_gather_all(comms, [ds], capi.default_opts(tonemap=6), capi.RT_OUT_HDR64,
                               d64.data_ptr())
        c0.synchronize()
        assert np.array_equal(d64.cpu().numpy().reshape(H, W, 3), ref["hdr64"])
        multi = capi.render_multi([ds], hdr64=True, tonemap=6, stats=True)
        assert np.array_equal(multi["hdr64"], ref["hdr64"])
        assert np.array_equal(multi["ldr"], ref["ldr"])
        assert (multi["trace_rays"], multi["shadow_rays"]) == (ref["trace_rays"],
                                                                ref["shadow_rays"])
        again = capi.render_multi([ds], hdr64=True, tonemap=6)  # cached communicators
        assert np.array_equal(again["hdr64"], ref["hdr64"])
        ds.close()
        for c in comms:
            c.close()
        with pytest.raises(capi.RtError):  # RCCL: one rank per GPU
            capi.Comm.create_all([c0, ctx])
    finally:
        c0.close()


@pytest.mark.parametrize("n,block,H,row_bytes", [
    (2, 16, 1080, 5760), (8, 16, 4320, 23040), (8, 16, 100, 48), (3, 7, 136, 720),
    (4, 16, 37, 13), (8, 54, 4320, 64), (5, 1, 23, 24), (16, 16, 64, 16)])
def test_assemble_rows_matches_row_planner(ctx, n, block, H, row_bytes):
    """Rank 0's assembly for n ranks (block-cyclic plans of distributed.row_ranges, ranks with
    no rows included): image row y comes from the rank and packed row the planner assigns."""
    rng = np.random.default_rng(n * 1000 + block)
    image = rng.integers(0, 256, (H, row_bytes), dtype=np.uint8)
    plans = [row_ranges(r, n, H, block) for r in range(n)]
    plans = [[(a, b) for a, b in p if a < H] for p in plans]
    max_rows = max(plan_rows(p) for p in plans)
    gathered = rng.integers(0, 256, (n, max_rows, row_bytes), dtype=np.uint8)  # padding: noise
    for r, p in enumerate(plans):
        k = 0
        for a, b in p:
            gathered[r, k:k + b - a] = image[a:b]
            k += b - a
    out = ctx.debug_assemble_rows(gathered, H, block, n, max_rows)
    assert np.array_equal(out, image)


def test_render_gather_pipelined_frames(ctx, comm1):
    """RT_FLAG_PIPELINE: frame k's gather + assembly run on the communicator's stream while frame
    k+1 renders (two slots).  Five frames from five cameras into five framebuffers, enqueued back
    to back, each equal to its own rt_render; then a serial frame after them."""
    sc = make_config("c3", 640, 360)
    W, H = 640, 360
    ds = ctx.scene(sc)
    try:
        base = ds.camera["position"][0].copy()
        cams = [base + (0.5 * k, -0.25 * k, 0.0) for k in range(5)]
        refs = []
        for cpos in cams:
            ds.camera["position"][0] = cpos
            refs.append(ds.render(hdr64=False, tonemap=1)["ldr"])
        outs = [torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda") for _ in cams]
        flags = capi.RT_FLAG_PIPELINE | capi.RT_FLAG_TIME_KERNEL
        for cpos, o in zip(cams, outs):
            ds.camera["position"][0] = cpos
            comm1.render_gather(ds, capi.default_opts(tonemap=1, flags=flags), capi.RT_OUT_LDR,
                                None, None, o.data_ptr())
        serial = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
        comm1.render_gather(ds, capi.default_opts(tonemap=1), capi.RT_OUT_LDR, None, None,
                            serial.data_ptr())
        comm1.synchronize()
        for k, (o, ref) in enumerate(zip(outs, refs)):
            assert np.array_equal(o.cpu().numpy().reshape(H, W, 3), ref), k
        assert np.array_equal(serial.cpu().numpy().reshape(H, W, 3), refs[-1])
        ds.camera["position"][0] = base
    finally:
        ds.close()
    t = comm1.timing(reset=True)
    assert t.frames == 5 and t.render_ms > 0 and t.assemble_ms > 0
