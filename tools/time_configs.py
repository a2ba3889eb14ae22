"""Dev tool: kernel time and Mrays/s of every config through the default path selection."""
import sys, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
for name in sys.argv[1:] or ["c1", "c2", "c3", "c4", "c5", "mirror", "glass", "mesh"]:
    sc = make_config(name)
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
    print(f"{name:7s} {W}x{H} {best:9.3f} ms  {rays / best / 1e3:10.1f} Mrays/s  rays/px {rays / (W * H):.2f}", flush=True)
    ds.close()
