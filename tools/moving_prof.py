"""Dev tool: C2 frame batches with a static camera, then with a camera that moves every frame
(bench.py's moving_camera: x += 1e-7 per frame, never repeating), for rocprofv3 --kernel-trace:
which kernels each kind of batch launches and how long they take.
    python tools/moving_prof.py [batch] [reps]"""
import sys
sys.path.insert(0, '.')
import numpy as np
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
sc = make_config("c2")
ds = ctx.scene(sc)
W, H = sc.camera.width, sc.camera.height
hdr = torch.empty(B * W * H * 3, dtype=torch.float64, device="cuda")
ldr = torch.empty(B * W * H * 3, dtype=torch.uint8, device="cuda")
base = np.array(ds.camera["position"][0], dtype=np.float64)
o = capi.default_opts(tonemap=1, flags=capi.RT_FLAG_TIME_KERNEL)
static = ds.cameras([base] * B)
for _ in range(reps):
    ds.render_batch(static, hdr.data_ptr(), None, ldr.data_ptr(), o)
ctx.synchronize()
ctx.reset_stats()
for _ in range(reps):
    ds.render_batch(static, hdr.data_ptr(), None, ldr.data_ptr(), o)
ctx.synchronize()
st = ctx.stats()
print("static us/frame %.2f" % (st.kernel_ms / st.launches / B * 1e3), flush=True)
k = 0
for phase in ("warm", "timed"):
    if phase == "timed":
        ctx.synchronize()
        ctx.reset_stats()
    for _ in range(reps):
        pos = [base + np.array([1e-7 * (k + f + 1), 0.0, 0.0]) for f in range(B)]
        k += B
        ds.render_batch(ds.cameras(pos), hdr.data_ptr(), None, ldr.data_ptr(), o)
ctx.synchronize()
st = ctx.stats()
print("moving us/frame %.2f" % (st.kernel_ms / st.launches / B * 1e3), flush=True)
ds.close()
