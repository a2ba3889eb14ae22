"""Dev tool: per-phase s_memtime cycles of the packet kernel, from an -DRT_STAMPS build
(RTAMD_LIB=tools/variants/stamps.so).  Averages per wave over 10 C2 frames."""
import ctypes, sys
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
NAMES = ["-", "ray gen", "cone cull", "closest", "shading setup", "light: L + packet cull",
         "occlusion", "light: accumulate", "material + AA acc", "outputs", "-", "-"]
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
lib = capi.load_library()
f = lib.rt_debug_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
for name in sys.argv[1:] or ["c2"]:
    sc = make_config(name)
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
    ldr = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    o = capi.default_opts(tonemap=1)
    for _ in range(3):
        ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
    ctx.synchronize()
    f(buf, 1)
    for _ in range(10):
        ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
    ctx.synchronize()
    f(buf, 1)
    waves = buf[15]
    tot = sum(buf[i] for i in range(12))
    print(f"{name}: {waves} waves, {tot / waves:.0f} stamped cycles per wave")
    for i in range(12):
        if buf[i]:
            print(f"  {NAMES[i]:24s} {buf[i] / waves:8.0f}  {100 * buf[i] / tot:5.1f}%")
    ds.close()
