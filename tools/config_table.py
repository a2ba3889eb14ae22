"""Dev tool (GPU box): every config through the default path — kernel time by HIP events,
Mrays/s (primary+shadow, exact counts from the counting pass) — next to the unmodified reference
(oracle/_ref/ref_harness) timed on the host cores on a bounded sample: the same scene at a
reduced resolution (same field of view) so each reference frame takes at most a few seconds.
Writes one JSON object (list of rows) to stdout."""
import json, os, sys, time
sys.path.insert(0, '.')
import torch
from oracle import pyoracle as po
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

CPU_SCALE = {"c1": 4, "c2": 4, "c3": 8, "c4": 16, "c5": 8, "mirror": 4, "glass": 4, "mesh": 4,
             "c1_aa32": 10, "bigmesh": 8}


def config(name, w=None, h=None):
    """`c1_aa32`: the reference main()'s own sampling (Camera::antiAliasingAmount = 32)."""
    if name == "c1_aa32":
        return make_config("c1", w, h, aa=32) if w else make_config("c1", aa=32)
    return make_config(name, w, h) if w else make_config(name)
# the cores this process may run on (capped by OMP_NUM_THREADS), one bound thread per core
threads = len(os.sched_getaffinity(0))
if int(os.environ.get("OMP_NUM_THREADS", "0") or 0) > 0:
    threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
rows = []
names = sys.argv[1:] or ["c1", "c1_aa32", "c2", "c3", "c4", "c5", "mirror", "glass", "mesh",
                          "bigmesh"]
for name in names:
    sc = config(name)
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
    ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    a = ds.render(hdr64=False, stats=True)
    rays = a["trace_rays"] + a["shadow_rays"]
    o = capi.default_opts(tonemap=1, flags=capi.RT_FLAG_TIME_KERNEL)
    t_end = time.perf_counter() + 0.05   # the GPU's clock ramp (tools/clock_ramp.py)
    while time.perf_counter() < t_end:
        for _ in range(4):
            ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
        torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        ctx.reset_stats()
        for _ in range(5):
            ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
        st = ctx.stats(); best = min(best, st.kernel_ms / st.launches)
    ds.close()
    row = {"config": name, "resolution": [W, H], "aa": sc.camera.antiAliasingAmount,
           "triangles": len(sc.triangle_array()), "spheres": len(sc.spheres),
           "planes": len(sc.planes), "lights": len(sc.lights), "rays_per_frame": rays,
           "gpu_ms_per_frame": round(best, 4), "gpu_mrays_s": round(rays / best / 1e3, 1)}
    if po.ref_available():
        k = CPU_SCALE[name]
        small = config(name, W // k, H // k)
        dss = ctx.scene(small)
        b = dss.render(hdr64=False, stats=True)
        dss.close()
        srays = b["trace_rays"] + b["shadow_rays"]
        _, ms, used = po.ref_render(small, repeat=3, threads=threads, want_image=False,
                                    bind=True)
        med = sorted(ms)[len(ms) // 2]
        row.update({"cpu_sample": f"same scene at {W // k}x{H // k}, 3 frames, median",
                    "cpu_threads": used, "cpu_ms_per_sample_frame": round(med, 2),
                    "cpu_mrays_s": round(srays / med / 1e3, 2)})
        ratio = round(rays / best / (srays / med), 1)
        if name == "bigmesh":
            # not a speed-up of the same algorithm: the GPU path traverses a triangle BVH, the
            # reference tests every triangle of every model for every ray (Shape.h:263-307)
            row["gpu_bvh_over_cpu_brute_force"] = ratio
        else:
            row["gpu_over_cpu"] = ratio
    rows.append(row)
    print(json.dumps(row), file=sys.stderr, flush=True)
print(json.dumps(rows, indent=1))
