"""Dev tool (GPU box): per-batch time of the headline frame from a cold start — how long the
GPU takes to reach its sustained clock under this kernel (bench.py's untimed clock warm-up)."""
import sys, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
sc = make_config("c2")
ds = ctx.scene(sc)
W, H = sc.camera.width, sc.camera.height
hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
o = capi.default_opts(tonemap=1)
t_start = time.perf_counter()
for b in range(80):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"batch {b:3d} at {1e3 * (t0 - t_start):7.1f} ms: {1e6 * (t1 - t0) / 50:6.2f} us/frame", flush=True)
    if b == 40:
        time.sleep(0.5)   # idle gap: does the clock drop back?
