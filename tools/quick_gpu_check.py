"""Dev tool: render every parity scene small on cuda:0 and diff against the C oracle."""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
from oracle import pyoracle as po

ctx = capi.Context(0)
x = np.random.default_rng(1).uniform(0.01, 50, 4096); y = np.random.default_rng(2).uniform(0.1, 8, 4096)
dev = ctx.debug_f64_ops(x, y)
print("div exact", np.array_equal(dev[:,0], x/y), "sqrt exact", np.array_equal(dev[:,1], np.sqrt(x)),
      "pow ulp-max", np.max(np.abs(dev[:,2]-np.power(x,y))/np.spacing(np.power(x,y))), "log ulp-max", np.max(np.abs(dev[:,3]-np.log(x))/np.spacing(np.abs(np.log(x)))))
for name in ["c1","c2","c3","c4","c5","mirror","glass","mesh"]:
    sc = make_config(name, 96, 54)
    ds = ctx.scene(sc)
    out = ds.render(hdr64=True, tonemap=1, stats=True)
    ref, nt, ns = po.render(sc)
    d = np.abs(out["hdr64"] - ref)
    print(f"{name:8s} maxdiff {d.max():.3e} n_neq {int((out['hdr64']!=ref).sum())} rays gpu {out['trace_rays']},{out['shadow_rays']} oracle {nt},{ns} ldr_eq {np.array_equal(out['ldr'], po.tonemap(ref,1).reshape(out['ldr'].shape))}", flush=True)
sc = make_config("c2")
ds = ctx.scene(sc)
out = ds.render(hdr64=True, stats=True)
t0 = time.time(); ref, nt, ns = po.render(sc); t1 = time.time()
print("c2 full maxdiff", np.abs(out["hdr64"]-ref).max(), "n_neq", int((out["hdr64"]!=ref).sum()), "rays", out["trace_rays"], out["shadow_rays"], nt, ns, "oracle s", t1-t0)
import torch
W,H = 1920,1080
buf = torch.empty(H*W*3, dtype=torch.float32, device='cuda')
o = capi.default_opts(tonemap=-1)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
for _ in range(5): ds.render_device(None, buf.data_ptr(), None, o)
torch.cuda.synchronize()
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): ds.render_device(None, buf.data_ptr(), None, o)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1)/50
print(f"c2 frame {ms:.4f} ms  Mrays/s {(nt+ns)/ms/1e3:.1f}")
