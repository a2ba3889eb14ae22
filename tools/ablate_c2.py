"""Dev tool: time C2 variants (sky only, no lights, no spheres, no tonemap, full) to split the
kernel time by stage.  Scene-level ablations, so every variant is a legitimate render."""
import sys, copy
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
W, H = 1920, 1080
hdr = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")

def t(sc, tonemap=1, max_rec=10, reps=30):
    ds = ctx.scene(sc)
    o = capi.default_opts(tonemap=tonemap, max_recursion=max_rec, flags=capi.RT_FLAG_TIME_KERNEL)
    for _ in range(3): ds.render_device(None, hdr.data_ptr(), ldr.data_ptr() if tonemap >= 0 else None, o)
    best = 1e9
    for _ in range(3):
        ctx.reset_stats()
        for _ in range(reps): ds.render_device(None, hdr.data_ptr(), ldr.data_ptr() if tonemap >= 0 else None, o)
        st = ctx.stats(); best = min(best, st.kernel_ms / st.launches)
    ds.close()
    return best * 1e3

base = make_config("c2")
print("full            %.1f us" % t(base))
print("no tonemap      %.1f us" % t(base, tonemap=-1))
print("sky only        %.1f us" % t(base, max_rec=0))
nl = copy.deepcopy(base); nl.lights = []
print("no lights       %.1f us" % t(nl))
ns = copy.deepcopy(base); ns.spheres = []
print("no spheres      %.1f us" % t(ns))
np_ = copy.deepcopy(base); np_.planes = []
print("no planes       %.1f us" % t(np_))
