"""Dev tool: render a config N times with the bench's outputs (float64 Vec3 HDR framebuffer +
fused tonemap bytes), for rocprofv3 kernel-trace / counter collection.
    python tools/profile_kernel.py CONFIG [reps] [flags] [batch]
batch > 1: each render is one rt_render_batch launch of `batch` frames (the bench's launch)."""
import sys, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
name = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
flags = int(sys.argv[3]) if len(sys.argv) > 3 else 0
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
sc = make_config(name)
ds = ctx.scene(sc)
W, H = sc.camera.width, sc.camera.height
hdr = torch.empty(batch * W * H * 3, dtype=torch.float64, device="cuda")
ldr = torch.empty(batch * W * H * 3, dtype=torch.uint8, device="cuda")
cams = ds.cameras([ds.camera["position"][0]] * batch)


def render():
    if batch > 1:
        ds.render_batch(cams, hdr.data_ptr(), None, ldr.data_ptr(), o)
    else:
        ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
o = capi.default_opts(tonemap=1, flags=flags)
# the GPU's clock ramp (tools/clock_ramp.py): 50 ms of the same renders first, so the counted
# dispatches run at the sustained clock (counter passes average every dispatch of the kernel)
t_end = time.perf_counter() + 0.05
while time.perf_counter() < t_end:
    for _ in range(8):
        render()
    ctx.synchronize()
for _ in range(reps):
    render()
ctx.synchronize()
