"""Dev tool (with an RT_STATS build via RTAMD_LIB): shadow candidates per shadow ray and the
fraction of shadow rays the fast occlusion test leaves undecided."""
import sys
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
ctx = capi.Context(0)
for name in sys.argv[1:] or ["c2"]:
    sc = make_config(name)
    ds = ctx.scene(sc)
    ref = ds.render(hdr64=False, stats=True) if False else None
    out = ds.render(hdr64=True, stats=True)
    ds.close()
    # the normal library's counts are needed for the shadow-ray total
    print(name, "candidates", out["trace_rays"], "undecided", out["shadow_rays"], flush=True)
