"""Dev tool: the DESIGN §5 config table in one run on the GPU box — every BASELINE config (and
the chain / tree / mesh scenes) at FULL resolution: the GPU frame time (one launch per frame,
and per frame in batches of 8 where the packet kernel renders the scene), its exact ray count,
and the UNMODIFIED reference (oracle/_ref/ref_harness, OpenMP threads bound one per granted
core) timed on the same frame in the same process; C5's area light has no reference semantics,
so its CPU column is the C restatement (oracle/rt_oracle.c, same threads).
    python tools/config_table.py [configs...] > profiles/r04_configs.json"""
import json
import os
import sys
import time

sys.path.insert(0, '.')
import numpy as np
import torch

from oracle import pyoracle as po
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

CONFIGS = [("c1", 1), ("c1", 32), ("c2", 1), ("c3", 1), ("c4", 1), ("c5", 1), ("mirror", 1),
           ("glass", 1), ("mesh", 1), ("bigmesh", 1)]
want = set(sys.argv[1:])
threads = len(os.sched_getaffinity(0))
omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
if omp > 0:
    threads = min(threads, omp)
ctx = capi.Context(0)
s = torch.cuda.Stream()
ctx.set_stream(s.cuda_stream)


def gpu_ms(ds, hdr, ldr, o, batch=None):
    t_end = time.perf_counter() + 0.05   # the GPU's clock ramp (tools/clock_ramp.py)
    while time.perf_counter() < t_end:
        for _ in range(4):
            ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
        torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            if batch is not None:
                ds.render_batch(batch, hdr.data_ptr(), None, ldr.data_ptr(), o)
            else:
                ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
        e1.record(s)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 5 / (len(batch) if batch is not None else 1))
    return best


rows = []
for name, aa in CONFIGS:
    if want and name not in want:
        continue
    sc = make_config(name, aa=aa)
    W, H = sc.camera.width, sc.camera.height
    ds = ctx.scene(sc)
    a = ds.render(hdr64=False, stats=True)
    rays = a["trace_rays"] + a["shadow_rays"]
    hdr = torch.empty(8 * W * H * 3, dtype=torch.float64, device="cuda")
    ldr = torch.empty(8 * W * H * 3, dtype=torch.uint8, device="cuda")
    o = capi.default_opts(tonemap=1)
    g1 = gpu_ms(ds, hdr, ldr, o)
    g8 = None
    if name in ("c2", "c3", "c4", "c5") and W * H <= 3840 * 2160:
        g8 = gpu_ms(ds, hdr, ldr, o, ds.cameras(np.repeat(ds.camera["position"], 8, axis=0)))
    ds.close()
    # the CPU: the unmodified reference (C5: the C restatement), 2 frames, the second timed
    if name == "c5":
        kind = "port"
        ms = []
        for _ in range(2):
            t = time.perf_counter()
            po.render(sc, nthreads=threads)
            ms.append((time.perf_counter() - t) * 1e3)
        used = threads
    else:
        kind = "reference"
        _, ms, used = po.ref_render(sc, repeat=2, threads=threads, want_image=False, bind=True)
    cpu_ms = ms[-1]
    row = {"config": name, "aa": aa, "resolution": [W, H], "rays_per_frame": int(rays),
           "gpu_ms_per_frame": round(g1, 5), "gpu_mrays_s": round(rays / g1 / 1e3, 1),
           "gpu_ms_per_frame_batch8": round(g8, 5) if g8 else None,
           "gpu_mrays_s_batch8": round(rays / g8 / 1e3, 1) if g8 else None,
           "cpu_kind": kind, "cpu_threads": used, "cpu_ms_per_frame": round(cpu_ms, 2),
           "cpu_mrays_s": round(rays / cpu_ms / 1e3, 2),
           "gpu_over_cpu": round(cpu_ms / g1, 1)}
    rows.append(row)
    print(json.dumps(row), file=sys.stderr, flush=True)
print(json.dumps({"host_threads": threads, "rows": rows,
                  "note": "GPU: HIP events around 5 launches, best of 3, after 50 ms of clock "
                          "warm-up; f64 HDR + fused Reinhard bytes.  CPU: full-resolution frames "
                          "of the unmodified reference Scene::RenderImage (OpenMP, threads bound "
                          "one per core), the second of two frames; C5: the C restatement."},
                 indent=1))
ctx.close()
