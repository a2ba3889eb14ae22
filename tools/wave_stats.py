"""Dev tool (GPU box): per-wave durations and work counters of the packet kernel, from the
diagnostic build of tools/build_wavestats.sh (tools/stampvariants/wavestats.so).  Prints how
the exact-march iterations, undecided shadow rays and shadow-candidate counts relate to the
slowest waves."""
import os, sys
sys.path.insert(0, '.')
import numpy as np
os.environ.setdefault("RTAMD_LIB", "tools/stampvariants/wavestats.so")
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
cnt = img[0::8, 1::8, :].reshape(-1, 3)
iters, undec, cand = cnt[:, 0], cnt[:, 1], cnt[:, 2]
ty, tx = np.divmod(np.arange(dur.size), st.shape[1])
print(f"{name}: {dur.size} waves, duration mean {dur.mean():.2f} us; march iterations / wave "
      f"mean {iters.mean():.1f}, undecided / wave mean {undec.mean():.2f}, shadow candidates "
      f"(lane-sum) / wave mean {cand.mean():.0f}")
for q in (50, 90, 99, 99.9):
    th = np.percentile(dur, q)
    sel = dur >= th
    print(f"waves >= p{q} ({th:.1f} us): n {sel.sum()}, iters {iters[sel].mean():.1f}, "
          f"undecided {undec[sel].mean():.2f}, candidates {cand[sel].mean():.0f}")
order = np.argsort(-dur)[:15]
print("slowest (tx, ty, us, march iters, undecided, candidates):")
for i in order:
    print(f"  {tx[i]:4d} {ty[i]:4d} {dur[i]:7.1f} {iters[i]:7.0f} {undec[i]:5.0f} {cand[i]:7.0f}")
c = np.corrcoef(np.vstack([dur, iters, undec, cand]))
print("corr(duration, iters/undecided/candidates):", np.round(c[0, 1:], 3).tolist())
