"""Dev tool: packet-kernel time with a camera that moves every frame (no cached packet image:
every workgroup forms it) and with a static one; RTAMD_LIB selects the build."""
import sys, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
for name in sys.argv[1:] or ["c2"]:
    sc = make_config(name)
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
    ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    o = capi.default_opts(tonemap=1)
    base = ds.camera["position"][0].copy()
    res = []
    for moving in (True, False):
        k = 0
        def frame():
            global k
            if moving:
                ds.camera["position"][0] = base + (k * 1e-7, 0.0, 0.0)
            k += 1
            ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
        t_end = time.perf_counter() + 0.05
        while time.perf_counter() < t_end:
            for _ in range(8):
                frame()
            torch.cuda.synchronize()
        best = 1e9
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                frame()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / 50)
        res.append(best)
    ds.camera["position"][0] = base
    print(name, "moving %.1f us static %.1f us" % (res[0] * 1e6, res[1] * 1e6), flush=True)
    ds.close()
