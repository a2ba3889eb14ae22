"""Dev tool: a steady stream of one config's frames for rocprofv3 PC sampling / counters.
    python tools/pcs_driver.py c2 [seconds]"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from raytracingengine_amd import capi  # noqa: E402
from raytracingengine_amd.configs import make_config  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c2"
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
ctx = capi.Context(0)
sc = make_config(name)
ds = ctx.scene(sc)
W, H = sc.camera.width, sc.camera.height
hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
o = capi.default_opts(tonemap=1)
n = 0
t_end = time.perf_counter() + secs
while time.perf_counter() < t_end:
    for _ in range(16):
        ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
    ctx.synchronize()
    n += 16
print(f"{name}: {n} frames", flush=True)
ds.close()
ctx.close()
