"""Dev tool: render a config N times with the bench's outputs (float64 Vec3 HDR framebuffer +
fused tonemap bytes), for rocprofv3 kernel-trace / counter collection."""
import sys, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
name = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
flags = int(sys.argv[3]) if len(sys.argv) > 3 else 0
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
sc = make_config(name)
ds = ctx.scene(sc)
W, H = sc.camera.width, sc.camera.height
hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
o = capi.default_opts(tonemap=1, flags=flags)
# the GPU's clock ramp (tools/clock_ramp.py): 50 ms of the same renders first, so the counted
# dispatches run at the sustained clock (counter passes average every dispatch of the kernel)
t_end = time.perf_counter() + 0.05
while time.perf_counter() < t_end:
    for _ in range(8):
        ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
    ctx.synchronize()
for _ in range(reps):
    ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
ctx.synchronize()
