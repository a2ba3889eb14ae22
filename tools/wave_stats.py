"""Dev tool (GPU box): per-wave durations and work counters of the packet kernel, from the
diagnostic build of tools/build_wavestats.sh (tools/diag/wavestats.so): how the occlusion
iterations, undecided shadow lanes, exact-march iterations and camera candidates relate to the
slowest waves, and where those waves are.   python tools/wave_stats.py CONFIG"""
import os, sys
sys.path.insert(0, '.')
import numpy as np
os.environ.setdefault("RTAMD_LIB", "tools/diag/wavestats.so")
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
ctx = capi.Context(0)
ds = ctx.scene(make_config(name))
for _ in range(3):
    img = ds.render(hdr64=True, tonemap=1)["hdr64"]
st = img[0::8, 0::8, :]
raw = np.ascontiguousarray(st).view(np.int64)
t0, t1 = raw[..., 0].ravel(), raw[..., 1].ravel()
dur = (t1 - t0) * 10e-3
c1 = img[0::8, 1::8, :].reshape(-1, 3)
occ, undec, march = c1[:, 0], c1[:, 1], c1[:, 2]
cam = img[0::8, 2::8, 0].ravel()
ty, tx = np.divmod(np.arange(dur.size), st.shape[1])
cols = {"occl": occ, "undec": undec, "march": march, "cam": cam}
print(f"{name}: {dur.size} waves, duration mean {dur.mean():.2f} us median {np.median(dur):.2f}; "
      + ", ".join(f"{k} mean {v.mean():.1f}" for k, v in cols.items()))
for q in (50, 90, 99, 99.9):
    th = np.percentile(dur, q)
    sel = dur >= th
    print(f"waves >= p{q} ({th:.1f} us): n {sel.sum()}, "
          + ", ".join(f"{k} {v[sel].mean():.1f}" for k, v in cols.items()))
order = np.argsort(-dur)[:20]
print("slowest (tx, ty, us, occl iters, undecided lanes, march iters, camera iters):")
for i in order:
    print(f"  {tx[i]:4d} {ty[i]:4d} {dur[i]:7.1f} {occ[i]:7.0f} {undec[i]:5.0f} {march[i]:7.0f} {cam[i]:6.0f}")
c = np.corrcoef(np.vstack([dur, occ, undec, march, cam]))
print("corr(duration, occl/undec/march/cam):", np.round(c[0, 1:], 3).tolist())
