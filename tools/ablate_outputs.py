"""Dev tool: C2 kernel time by output set (hdr32 / ldr / both / none) and by scene stage."""
import sys, copy
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
W, H = 1920, 1080
hdr = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
h64 = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")


def t(sc, h32=True, l8=True, d64=False, tonemap=1, max_rec=10, reps=30):
    ds = ctx.scene(sc)
    o = capi.default_opts(tonemap=tonemap if l8 else -1, max_recursion=max_rec,
                          flags=capi.RT_FLAG_TIME_KERNEL)
    args = (h64.data_ptr() if d64 else None, hdr.data_ptr() if h32 else None,
            ldr.data_ptr() if l8 else None, o)
    for _ in range(3):
        ds.render_device(*args)
    best = 1e9
    for _ in range(3):
        ctx.reset_stats()
        for _ in range(reps):
            ds.render_device(*args)
        st = ctx.stats()
        best = min(best, st.kernel_ms / st.launches)
    ds.close()
    return best * 1e3


base = make_config(sys.argv[1] if len(sys.argv) > 1 else "c2")
print("hdr32+ldr       %.1f us" % t(base))
print("hdr32 only      %.1f us" % t(base, l8=False))
print("ldr only        %.1f us" % t(base, h32=False))
print("hdr64 only      %.1f us" % t(base, h32=False, l8=False, d64=True))
try:
    print("no outputs      %.1f us" % t(base, h32=False, l8=False))
except Exception as e:  # noqa: BLE001
    print("no outputs      refused:", e)
print("sky only (ldr+h32) %.1f us" % t(base, max_rec=0))
nl = copy.deepcopy(base); nl.lights = []
print("no lights       %.1f us" % t(nl))
ns = copy.deepcopy(base); ns.spheres = []
print("no spheres      %.1f us" % t(ns))
