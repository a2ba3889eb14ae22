"""Dev tool: separate fixed from per-pixel cost of the packet kernel (sky-only / empty scenes,
output sets, image sizes)."""
import sys, copy
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
NMAX = 3840 * 2160 * 3
hdr = torch.empty(NMAX, dtype=torch.float32, device="cuda")
h64 = torch.empty(NMAX, dtype=torch.float64, device="cuda")
ldr = torch.empty(NMAX, dtype=torch.uint8, device="cuda")


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


base = make_config("c2")
empty = copy.deepcopy(base); empty.spheres = []; empty.planes = []; empty.lights = []
print("c2 sky-only, no outputs     %.1f us" % t(base, h32=False, l8=False, max_rec=0))
print("c2 sky-only, hdr32          %.1f us" % t(base, l8=False, max_rec=0))
print("c2 sky-only, hdr32+ldr      %.1f us" % t(base, max_rec=0))
print("empty scene, hdr32+ldr      %.1f us" % t(empty))
print("empty scene, no outputs     %.1f us" % t(empty, h32=False, l8=False))
for (w, h) in [(480, 270), (960, 540), (1920, 1080), (3840, 2160)]:
    sc = make_config("c2", w, h)
    print("c2 %4dx%4d full   %.1f us   sky-only %.1f us" % (w, h, t(sc), t(sc, max_rec=0)))
