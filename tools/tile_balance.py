"""Dev tool: kernel time of each rank's rows of a frame, rendered one after another on one GPU —
the load imbalance of the multi-GPU row split measured without 8 GPUs, for
contiguous tiles and for block-cyclic rows — next to the single launch of the whole frame.
    python tools/tile_balance.py [ranks] [blocks,...] [configs...]
Each launch is timed after its own warm-up renders (so the per-camera packet image and the
costliest-first tile order of that launch shape exist, rt_capi.cpp), at the sustained clock."""
import sys, json, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
from raytracingengine_amd.distributed import render_opts_for, row_ranges
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
BLOCKS = [int(b) for b in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "16"])]


def timed(ds, hdr, o, reps=5):
    for _ in range(3):
        ds.render_device(hdr.data_ptr(), None, None, o)
    ctx.reset_stats()
    for _ in range(reps):
        ds.render_device(hdr.data_ptr(), None, None, o)
    st = ctx.stats()
    return st.kernel_ms / st.launches


for name in sys.argv[3:] or ["c2", "c3", "c4", "c5"]:
    sc = make_config(name)
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
    full_o = capi.default_opts(tonemap=-1, flags=capi.RT_FLAG_TIME_KERNEL)
    t_end = time.perf_counter() + 0.05   # the GPU's clock ramp (tools/clock_ramp.py)
    while time.perf_counter() < t_end:
        for _ in range(4):
            ds.render_device(hdr.data_ptr(), None, None, full_o)
        torch.cuda.synchronize()
    full = timed(ds, hdr, full_o)
    for block in BLOCKS:
        ts = []
        for r in range(n):
            ranges = row_ranges(r, n, H, block)
            o = render_opts_for(ranges, r, n, H, block, tonemap=-1, flags=capi.RT_FLAG_TIME_KERNEL)
            ts.append(timed(ds, hdr, o))
        mean = sum(ts) / n
        print(json.dumps({"config": name, "ranks": n, "row_block": block,
                          "ms": [round(t, 4) for t in ts],
                          "max_over_mean": round(max(ts) / mean, 3),
                          "full_frame_ms": round(full, 4),
                          "rank_sum_over_full": round(sum(ts) / full, 3),
                          "ideal_speedup": round(full / max(ts), 2)}), flush=True)
    ds.close()
