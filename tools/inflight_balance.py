"""Dev tool: one rank's share of a row-split frame with K frames in flight, on one GPU.

    python tools/inflight_balance.py [ranks] [streams,...] [configs...]

For every rank r of `ranks` (block-cyclic 16-row blocks, the multi-GPU plan of rt_multi.cpp) it
enqueues F frames of rank r's rows (f64 Vec3 rows + fused Reinhard bytes, per-slot buffers)
round-robin over S HIP streams and reports the GPU time per rank-frame.  GPU-bound: every stream
first waits behind ~3 ms of whole frames on stream 0 (real work, so the GPU keeps its sustained
clock — a sleep kernel lets it drop), long enough to cover the host's enqueue of all F frames,
so the launches reach the GPU back to back; the host's own enqueue cost per frame is reported
beside it (`host_us`).  The full frame on one stream, measured the same way, is the reference:
the target is a rank-frame <= 1.3 x full / ranks.  `weighted`: rank 0's and the slowest peer's
time per frame when rank 0 renders w of w + ranks − 1 row sets (rt_comm_set_root_weight), against
bench.py choose_root_weight's model (T·w/V and T/V).
"""
import json
import os
import sys
import time

sys.path.insert(0, '.')
import numpy as np
import torch

from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
from raytracingengine_amd.distributed import render_opts_for, row_ranges

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
STREAMS = [int(s) for s in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "2", "3", "4"])]
CONFIGS = sys.argv[3:] or ["c2"]
BATCHES = [4, 8, 16, 32]
FRAMES = 240
BLOCK = int(os.environ.get("RT_INFLIGHT_BLOCK", "16"))  # rows per block of the split

ctx = capi.Context(0)
streams = [torch.cuda.Stream() for _ in range(max(STREAMS))]


def busy(ds, frames):
    """`frames` whole frames on stream 0: the gate the measured launches queue behind."""
    ctx.set_stream(streams[0].cuda_stream)
    h, l = BUSY
    for _ in range(frames):
        ds.render_device(h.data_ptr(), None, l.data_ptr(), FULL_O)


def run(ds, opts, bufs, S, frames, busy_frames):
    """GPU ms per frame of `frames` frames round-robin over S streams, host us per enqueue."""
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(S)]
    gate = torch.cuda.Event()
    busy(ds, busy_frames)
    with torch.cuda.stream(streams[0]):
        gate.record(streams[0])
        e0.record(streams[0])
    for s in streams[1:S]:
        s.wait_event(gate)
    t0 = time.perf_counter()
    for i in range(frames):
        s = streams[i % S]
        ctx.set_stream(s.cuda_stream)
        h, l = bufs[i % len(bufs)]
        ds.render_device(h.data_ptr(), None, l.data_ptr(), opts)
    host = (time.perf_counter() - t0) / frames * 1e6
    for k in range(S):
        ends[k].record(streams[k])
    torch.cuda.synchronize()
    gpu = max(e0.elapsed_time(e) for e in ends) / frames
    return gpu, host


def run_batch(ds, opts, bbufs, G, batches, busy_frames):
    """GPU ms per frame of `batches` launches of G frames (rt_render_batch) on one stream."""
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = streams[0]
    ctx.set_stream(s.cuda_stream)
    cams = ds.cameras(np.repeat(ds.camera["position"], G, axis=0))
    busy(ds, busy_frames)
    with torch.cuda.stream(s):
        e0.record(s)
    t0 = time.perf_counter()
    for i in range(batches):
        h, l = bbufs[i % len(bbufs)]
        ds.render_batch(cams, h.data_ptr(), None, l.data_ptr(), opts)
    host = (time.perf_counter() - t0) / (batches * G) * 1e6
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (batches * G), host


def warm(ds, opts, bufs, ms=60):
    t_end = time.perf_counter() + ms / 1e3
    ctx.set_stream(streams[0].cuda_stream)
    while time.perf_counter() < t_end:
        for i in range(8):
            h, l = bufs[i % len(bufs)]
            ds.render_device(h.data_ptr(), None, l.data_ptr(), opts)
        torch.cuda.synchronize()


for name in CONFIGS:
    sc = make_config(name)
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    depth = max(STREAMS)
    bufs = [(torch.empty(W * H * 3, dtype=torch.float64, device="cuda"),
             torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")) for _ in range(depth)]
    full_o = capi.default_opts(tonemap=1)
    warm(ds, full_o, bufs)
    for _ in range(4):   # the camera's packet image and tile order exist
        ds.render_device(bufs[0][0].data_ptr(), None, bufs[0][1].data_ptr(), full_o)
    BUSY, FULL_O = bufs[0], full_o
    cyc = 64  # whole frames (~3 ms of C2) ahead of every measured run
    # batches whose two buffer sets fit 16 GiB (C4: up to 8 frames per launch)
    batches = [G for G in BATCHES if 2 * G * W * H * 27 <= 16 << 30] or [1]
    full = {}
    for S in STREAMS:
        warm(ds, full_o, bufs, 30)
        full[S] = run(ds, full_o, bufs, S, 120, cyc)
    out = {"config": name, "ranks": n, "row_block": BLOCK, "frames": FRAMES,
           "full_frame_ms": {S: round(full[S][0], 5) for S in STREAMS},
           "full_host_us": round(full[1][1], 2), "ranks_ms": {}, "host_us": {}}
    for S in STREAMS:
        ts, hs = [], []
        for r in range(n):
            o = render_opts_for(row_ranges(r, n, H, BLOCK), r, n, H, BLOCK, tonemap=1)
            for _ in range(4):
                ds.render_device(bufs[0][0].data_ptr(), None, bufs[0][1].data_ptr(), o)
            warm(ds, o, bufs, 20)
            g, h = run(ds, o, bufs, S, FRAMES, cyc)
            ts.append(g)
            hs.append(h)
        out["ranks_ms"][S] = [round(t, 5) for t in ts]
        out["host_us"][S] = round(sum(hs) / n, 2)
        out.setdefault("max_rank_over_full_div_n", {})[S] = round(max(ts) / (full[1][0] / n), 3)
    for G in batches:
        bbufs = [(torch.empty(G * W * H * 3, dtype=torch.float64, device="cuda"),
                  torch.empty(G * W * H * 3, dtype=torch.uint8, device="cuda")) for _ in range(2)]
        warm(ds, full_o, bufs, 30)
        fg, fh = run_batch(ds, full_o, bbufs, G, max(2, 96 // G), cyc)
        out.setdefault("batch_full_frame_ms", {})[G] = round(fg, 5)
        ts, hs = [], []
        for r in range(n):
            o = render_opts_for(row_ranges(r, n, H, BLOCK), r, n, H, BLOCK, tonemap=1)
            warm(ds, o, bufs, 20)
            g, h = run_batch(ds, o, bbufs, G, max(4, FRAMES // G), cyc)
            ts.append(g)
            hs.append(h)
        out.setdefault("batch_ranks_ms", {})[G] = [round(t, 5) for t in ts]
        out.setdefault("batch_host_us", {})[G] = round(sum(hs) / n, 2)
        out.setdefault("batch_max_rank_over_full_div_n", {})[G] = round(max(ts) / (full[1][0] / n), 3)
        del bbufs
    # the weighted split (rt_comm_set_root_weight): rank 0 renders w of the w + n − 1 row sets
    # (one batch launch per set), every other rank one — measured per frame at the largest batch
    G = batches[-1]
    bbufs = [(torch.empty(G * W * H * 3, dtype=torch.float64, device="cuda"),
              torch.empty(G * W * H * 3, dtype=torch.uint8, device="cuda")) for _ in range(2)]
    Tb = out["batch_full_frame_ms"][G]
    for w in (2, 3):
        V = w + n - 1
        slot_ms = []
        for sl in range(V):
            o = render_opts_for(row_ranges(sl, V, H, BLOCK), sl, V, H, BLOCK, tonemap=1)
            warm(ds, o, bufs, 20)
            g, _ = run_batch(ds, o, bbufs, G, max(4, FRAMES // G), cyc)
            slot_ms.append(g)
        out.setdefault("weighted", {})[w] = {
            "sets": V, "rank0_ms": round(sum(slot_ms[:w]), 5),
            "peer_max_ms": round(max(slot_ms[w:]), 5),
            "model_rank0_ms": round(Tb * w / V, 5), "model_peer_ms": round(Tb / V, 5)}
    del bbufs
    print(json.dumps(out), flush=True)
    ds.close()
ctx.close()
