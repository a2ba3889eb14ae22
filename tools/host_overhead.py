"""Dev tool (GPU box): where the wall time of a short timed region goes outside the kernel.

bench.py at the driver's `--steps 20` times ONE 20-frame launch; its wall time per frame was
2.8 us above the launch's HIP-event time (41.4 vs 38.6 us).  This measures, for the bench's N=1
step (rt_render_gather_batch on a one-rank communicator, f64 HDR rank-local + Reinhard bytes):
  * host enqueue time of one call, with and without RT_FLAG_TIME_KERNEL events;
  * a region of one 20-frame call: wall (perf_counter around call + synchronize) vs the HIP events
    of the launch (kernel) vs HIP events on the stream around the whole region;
Prints one JSON line per measurement.
"""
import json
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raytracingengine_amd import capi  # noqa: E402
from raytracingengine_amd.configs import make_config  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctx = capi.Context(0)
    stream = torch.cuda.Stream()
    ctx.set_stream(stream.cuda_stream)
    comm = capi.Comm(ctx, 1, 0, capi.comm_unique_id())
    sc = make_config("c2")
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    cams = ds.cameras(np.repeat(ds.camera["position"], 32, axis=0))
    hdr = torch.empty(32 * W * H * 3, dtype=torch.float64, device="cuda")
    ldr = torch.empty(32 * W * H * 3, dtype=torch.uint8, device="cuda")
    plain = capi.default_opts(tonemap=1, flags=capi.RT_FLAG_PIPELINE)
    timed = capi.default_opts(tonemap=1, flags=capi.RT_FLAG_PIPELINE | capi.RT_FLAG_TIME_KERNEL)

    def call(k, opts):
        comm.render_gather_batch(ds, cams[:k], opts, capi.RT_OUT_LDR, d_ldr=ldr.data_ptr(),
                                 rank_hdr64=hdr.data_ptr())

    # clock warm-up
    t_end = time.perf_counter() + 0.2
    while time.perf_counter() < t_end:
        for _ in range(4):
            call(32, plain)
        torch.cuda.synchronize()
    comm.timing(reset=True)
    for name, opts in (("plain", plain), ("timed", timed)):
        host = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            call(n, opts)
            host.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        print(json.dumps({"what": "enqueue_us", "opts": name, "frames": n,
                          "median": round(1e6 * float(np.median(host)), 2),
                          "min": round(1e6 * min(host), 2)}), flush=True)
    comm.timing(reset=True)
    for opts_name, opts in (("timed", timed), ("plain", plain)):
        walls, regions = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            call(n, opts)
            e1.record(stream)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            regions.append(e0.elapsed_time(e1) * 1e-3)
        t = comm.timing(reset=True)
        kern = t.render_ms / max(t.frames, 1) * n * 1e-3
        print(json.dumps({"what": "region", "opts": opts_name, "frames": n,
                          "wall_us": round(1e6 * float(np.median(walls)), 2),
                          "stream_events_us": round(1e6 * float(np.median(regions)), 2),
                          "kernel_events_us": round(1e6 * kern, 2)}), flush=True)
    ds.close()
    comm.close()
    ctx.close()


if __name__ == "__main__":
    main()
