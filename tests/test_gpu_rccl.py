"""The RCCL multi-GPU frame path behind the C-ABI (rt_multi.cpp; SURVEY.md §8e, RE/Scene.h:318-325).

The test box has ONE MI355X and RCCL allows one rank per GPU ("Duplicate GPU detected"), so
ncclGather itself only runs here with n = 1 (where the rank now renders straight into the frame).
The n > 1 frame runs end to end on the one GPU through LOCAL communicators
(rt_comm_create_local): n contexts, each on its own stream, render their block-cyclic rows into
padded send buffers; the gather is a device copy of every rank's buffer into rank 0's receive
buffer at rank r's offset (what ncclGather delivers); rank 0 assembles — every line of
rt_multi.cpp's multi-rank frame except the ncclGather call.  The row plans are also pinned through
the assembly hook (rt_debug_assemble_rows) against the Python row planner, and the multi-rank
gather of the Python driver runs on CPU with gloo (tests/test_distributed_cpu.py).
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
            torch.cuda.synchronize()  # the fills run on torch's stream, the render on ctx's
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
    # one rank renders straight into the framebuffers: nothing to gather or assemble
    assert t.render_ms > 0 and t.gather_ms >= 0 and t.assemble_ms >= 0


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
        torch.cuda.synchronize()  # the fills run on torch's stream, the renders on ctx's
        flags = capi.RT_FLAG_PIPELINE | capi.RT_FLAG_TIME_KERNEL
        for cpos, o in zip(cams, outs):
            ds.camera["position"][0] = cpos
            comm1.render_gather(ds, capi.default_opts(tonemap=1, flags=flags), capi.RT_OUT_LDR,
                                None, None, o.data_ptr())
        serial = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
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
    assert t.frames == 5 and t.render_ms > 0 and t.assemble_ms >= 0


@pytest.fixture(scope="module")
def local_ctxs():
    cs = [capi.Context(0) for _ in range(8)]
    yield cs
    for c in cs:
        c.close()


def _local_frame(ctxs, sc, n, outputs, flags=0, row_block=0, frames=1, cams=None):
    """n local ranks render `frames` frames of `sc` (one camera per frame) through
    rt_render_gather_all; returns the host copies of rank 0's framebuffers per frame."""
    W, H = sc.camera.width, sc.camera.height
    comms = capi.Comm.create_local(ctxs[:n])
    scenes = [c.scene(sc) for c in ctxs[:n]]
    try:
        outs = []
        for k in range(frames):
            if cams is not None:
                for ds in scenes:
                    ds.camera["position"][0] = cams[k]
            bufs = {"hdr64": torch.zeros(H * W * 3, dtype=torch.float64, device="cuda"),
                    "hdr32": torch.zeros(H * W * 3, dtype=torch.float32, device="cuda"),
                    "ldr": torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")}
            ptr = {k2: (v.data_ptr() if outputs & bit else None) for (k2, v), bit in
                   zip(bufs.items(), (capi.RT_OUT_HDR64, capi.RT_OUT_HDR32, capi.RT_OUT_LDR))}
            torch.cuda.synchronize()  # the zero fills run on torch's stream, the ranks on theirs
            capi.render_gather_all(comms, scenes,
                                   capi.default_opts(tonemap=1, flags=flags, row_block=row_block),
                                   outputs, ptr["hdr64"], ptr["hdr32"], ptr["ldr"])
            outs.append(bufs)
        for c in comms:
            c.synchronize()
        timing = [c.timing(reset=True) for c in comms]
        host = [{k2: v.cpu().numpy().reshape(H, W, 3) for k2, v in b.items()} for b in outs]
        return host, timing
    finally:
        for c in comms:
            c.close()
        for ds in scenes:
            ds.close()


@pytest.mark.parametrize("name,w,h,n,block", [
    ("c2", 640, 360, 2, 0), ("c2", 640, 360, 8, 0), ("c3", 640, 360, 3, 7),
    ("c5", 320, 180, 4, 16), ("glass", 200, 120, 2, 5), ("mirror", 320, 180, 5, 0),
    ("c2", 96, 40, 8, 16)])  # the last: ranks 3..7 have no rows (padding only)
def test_local_ranks_frame_equals_render(ctx, local_ctxs, name, w, h, n, block):
    """n > 1 ranks of the multi-rank frame on one GPU (local communicators): every output equals
    rt_render, with the row plan's padding, empty ranks and per-rank timings."""
    sc = make_config(name, w, h)
    ds = ctx.scene(sc)
    try:
        ref = ds.render(hdr64=True, hdr32=True, tonemap=1)
    finally:
        ds.close()
    outs = capi.RT_OUT_HDR64 | capi.RT_OUT_HDR32 | capi.RT_OUT_LDR
    host, timing = _local_frame(local_ctxs, sc, n, outs, flags=capi.RT_FLAG_TIME_KERNEL,
                                row_block=block)
    assert np.array_equal(host[0]["hdr64"], ref["hdr64"])
    assert np.array_equal(host[0]["hdr32"], ref["hdr32"])
    assert np.array_equal(host[0]["ldr"], ref["ldr"])
    b = block or 16
    plans = [[(a, min(c, h)) for a, c in row_ranges(r, n, h, b) if a < h] for r in range(n)]
    rows = [plan_rows(p) for p in plans]
    assert [t.rows for t in timing] == rows
    assert all(t.max_rows == max(rows) and t.frames == 1 for t in timing)
    assert timing[0].assemble_ms > 0


def test_local_ranks_pipelined_frames(local_ctxs):
    """RT_FLAG_PIPELINE with 4 local ranks: five frames from five cameras enqueued back to back
    (frame k's gather + assembly overlap frame k+1's render, two send/receive slots per rank),
    each equal to rt_render of its camera."""
    sc = make_config("c3", 640, 360)
    base = np.array(sc.camera.position)
    cams = [base + (0.5 * k, -0.25 * k, 0.0) for k in range(5)]
    refs = []
    ds = local_ctxs[7].scene(sc)
    try:
        for cpos in cams:
            ds.camera["position"][0] = cpos
            refs.append(ds.render(hdr64=False, tonemap=1)["ldr"])
    finally:
        ds.close()
    host, timing = _local_frame(local_ctxs, sc, 4, capi.RT_OUT_LDR,
                                flags=capi.RT_FLAG_PIPELINE | capi.RT_FLAG_TIME_KERNEL,
                                frames=5, cams=cams)
    for k in range(5):
        assert np.array_equal(host[k]["ldr"], refs[k]), k
    assert all(t.frames == 5 for t in timing)


def test_local_8_ranks_full_c4_reference_bytes(local_ctxs, golden):
    """The bench's N=8 workload on one GPU: the full 7680x4320 C4 frame split over 8 ranks in
    16-row blocks, gathered into rank 0 and assembled — the reference's Reinhard bytes."""
    sc = make_config("c4")
    host, timing = _local_frame(local_ctxs, sc, 8, capi.RT_OUT_LDR)
    assert _sha(host[0]["ldr"]) == golden["meta"]["scenes"]["c4_full"]["ldr_sha256"][
        "reinhard_simple"]
    assert sum(t.rows for t in timing) == sc.camera.height


def test_render_multi_shared_device_group_lifetime():
    """rt_render_multi over contexts that share the GPU goes through local communicators cached
    in the first context.  Destroying a NON-root member first releases that cached group (no
    communicator is left pointing at the dead context); a new context list rebuilds it."""
    sc = make_config("c2", 320, 180)
    cs = [capi.Context(0) for _ in range(3)]
    try:
        ref_ds = cs[0].scene(sc)
        ref = ref_ds.render(hdr64=True, tonemap=1, stats=True)
        scenes = [c.scene(sc) for c in cs]
        for _ in range(2):  # the second call reuses the cached group
            m = capi.render_multi(scenes, hdr64=True, tonemap=1, stats=True)
            assert np.array_equal(m["hdr64"], ref["hdr64"])
            assert np.array_equal(m["ldr"], ref["ldr"])
            assert (m["trace_rays"], m["shadow_rays"]) == (ref["trace_rays"], ref["shadow_rays"])
        scenes[1].close()
        cs[1].close()                       # a member of cs[0]'s group goes first
        cs[1] = capi.Context(0)
        scenes[1] = cs[1].scene(sc)
        m = capi.render_multi([scenes[0], scenes[2], scenes[1]], hdr64=True, tonemap=1)
        assert np.array_equal(m["hdr64"], ref["hdr64"])
        for ds in scenes + [ref_ds]:
            ds.close()
    finally:
        for c in cs:
            c.close()                       # root first this time, then the members


# ------------------------------------------------------------------ failure detection
_MISSING_PEER = r'''
import json, sys, time, hashlib
import numpy as np
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
ctx = capi.Context(0)
t0 = time.perf_counter()
status, msg = 0, ""
try:
    c = capi.Comm(ctx, 2, 0, capi.comm_unique_id(), timeout_ms=int(sys.argv[1]))
    c.close()
except capi.RtError as e:
    status, msg = e.status, str(e)
dt = time.perf_counter() - t0
sc = make_config("c2", 192, 108)
ds = ctx.scene(sc)
out = ds.render(hdr64=True, tonemap=1)
ds.close()
print(json.dumps({"status": status, "msg": msg, "seconds": dt,
                  "sha": hashlib.sha256(out["hdr64"].tobytes()).hexdigest()}))
'''


def test_comm_missing_peer_fails_within_deadline_then_renders(oracle):
    """Rank 0 of a 2-rank communicator whose peer never joins: the non-blocking
    ncclCommInitRankConfig polled with a 3 s deadline returns RT_ERR_RCCL (communicator aborted)
    instead of blocking, and the same process then renders a frame equal to the oracle's.  Run
    in a child process under its own time limit, so a regression cannot hang the suite."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    p = subprocess.run([sys.executable, "-c", _MISSING_PEER, "3000"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["status"] == capi.RT_ERR_RCCL, r
    assert "aborted" in r["msg"], r
    assert 2.5 <= r["seconds"] < 30.0, r
    sc = make_config("c2", 192, 108)
    ref, _, _ = oracle.render(sc)
    assert r["sha"] == _sha(ref)


def test_comm_with_deadline_renders_and_synchronizes(ctx):
    """A 1-rank communicator through rt_comm_create_ex (non-blocking init, 10 s deadline) and a
    changed deadline: frames render and synchronize as with rt_comm_create; a negative deadline
    is an invalid argument."""
    c = capi.Comm(ctx, 1, 0, capi.comm_unique_id(), timeout_ms=10000)
    try:
        c.set_timeout(5000)
        sc = make_config("c2", 160, 90)
        ds = ctx.scene(sc)
        try:
            ref = ds.render(tonemap=1)["ldr"]
            d8 = torch.zeros(90 * 160 * 3, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            c.render_gather(ds, capi.default_opts(tonemap=1), capi.RT_OUT_LDR, d_ldr=d8.data_ptr())
            c.synchronize()
            assert np.array_equal(d8.cpu().numpy().reshape(90, 160, 3), ref)
        finally:
            ds.close()
        with pytest.raises(capi.RtError) as e:
            c.set_timeout(-1)
        assert e.value.status == capi.RT_ERR_INVALID_ARG
    finally:
        c.close()


@pytest.mark.parametrize("weight", [1, 2])
def test_create_all_set_root_weight_then_weighted_gather(ctx, weight):
    """rt_comm_set_root_weight on every communicator of an rt_comm_create_all group (blocking
    ncclCommInitAll ranks driven serially from one thread) must not enqueue the agreement
    all-reduce — only rt_comm_create ranks (one process per GPU) agree through RCCL; this group's
    weights are checked on the host by rt_render_gather_all_batch.  Then a weighted batch over
    the group equals the single-GPU frames.  Every device of the box (one on the test box: the
    call path; all of them on a multi-GPU node: the weighted P2P split over RCCL)."""
    ndev = torch.cuda.device_count()
    ctxs = [capi.Context(d) for d in range(ndev)]
    try:
        comms = capi.Comm.create_all(ctxs)
        for c in comms:
            c.set_root_weight(weight)   # returns at once (no collective to hang on)
        sc = make_config("c2", 480, 270)
        W, H, nf = 480, 270, 3
        scenes = [c.scene(sc) for c in ctxs]
        ref = scenes[0].render(hdr64=True, tonemap=1)
        cams = scenes[0].cameras(np.repeat(scenes[0].camera["position"], nf, axis=0))
        with torch.cuda.device(0):
            L8 = torch.zeros(nf * H * W * 3, dtype=torch.uint8, device="cuda:0")
            H64 = torch.zeros(nf * H * W * 3, dtype=torch.float64, device="cuda:0")
        capi.render_gather_all_batch(comms, scenes, cams, capi.default_opts(tonemap=1, row_block=16),
                                     capi.RT_OUT_LDR | capi.RT_OUT_HDR64,
                                     d_hdr64=H64.data_ptr(), d_ldr=L8.data_ptr())
        for c in comms:
            c.synchronize()
        for f in range(nf):
            assert np.array_equal(H64.view(nf, -1)[f].cpu().numpy(), ref["hdr64"].reshape(-1)), f
            assert np.array_equal(L8.view(nf, -1)[f].cpu().numpy(), ref["ldr"].reshape(-1)), f
        for s in scenes:
            s.close()
        for c in comms:
            c.close()
    finally:
        for c in ctxs:
            c.close()
