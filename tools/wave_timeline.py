"""Dev tool (GPU box): per-wave start/end timestamps of the packet kernel, from a diagnostic
build (tools/variants/stamps.so, made by `python tools/build_variant.py stamps ...` with the
patch in tools/stamps_patch.txt) that overwrites each 8x8 tile's first pixel of the float64
framebuffer with (s_memrealtime at kernel entry, at exit, XCC/HW_ID).  Prints the launch
timeline: wave durations, how many waves are resident over time, and the ramp/tail idle."""
import os, sys
sys.path.insert(0, '.')
import numpy as np
os.environ.setdefault("RTAMD_LIB", "tools/variants/stamps.so")
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

name = sys.argv[1] if len(sys.argv) > 1 else "c2"
ctx = capi.Context(0)
sc = make_config(name)
ds = ctx.scene(sc)
for _ in range(3):
    out = ds.render(hdr64=True, tonemap=1)
img = out["hdr64"]
H, W, _ = img.shape
tiles = img[0::8, 0::8, :]                      # each wave's top-left pixel
raw = np.ascontiguousarray(tiles).view(np.int64)
t0, t1 = raw[..., 0].ravel(), raw[..., 1].ravel()
hw = tiles[..., 2].ravel().astype(np.int64)
ok = (t1 > t0) & (t0 > 0)
t0, t1, hw = t0[ok], t1[ok], hw[ok]
base = t0.min()
s, e = (t0 - base) * 10e-3, (t1 - base) * 10e-3    # 100 MHz -> microseconds
dur = e - s
span = e.max()
print(f"{name}: {ok.sum()} waves, span {span:.1f} us, wave duration min/median/mean/max "
      f"{dur.min():.2f}/{np.median(dur):.2f}/{dur.mean():.2f}/{dur.max():.2f} us")
# resident waves over time (1 us bins)
bins = np.arange(0, span + 1.0, 1.0)
res = np.array([((s <= b) & (e > b)).sum() for b in bins])
full = np.percentile(res, 90)
print("resident waves per us:", " ".join(str(int(r)) for r in res))
work = dur.sum()
print(f"sum of wave time {work:.0f} wave-us; at the 90th-percentile residency ({full:.0f}) the "
      f"launch would take {work / full:.1f} us (measured span {span:.1f})")
# per-row-of-tiles mean duration (tile rows of 8 px)
rows = np.zeros(tiles.shape[0]); cnt = np.zeros(tiles.shape[0])
ty = np.repeat(np.arange(tiles.shape[0]), tiles.shape[1])[ok.ravel()] if False else None
T = tiles.shape[0] * tiles.shape[1]
ry = np.repeat(np.arange(tiles.shape[0]), tiles.shape[1])[ok]
np.add.at(rows, ry, dur); np.add.at(cnt, ry, 1)
print("mean wave duration per tile row (top to bottom):",
      " ".join(f"{v:.1f}" for v in rows / np.maximum(cnt, 1)))
xcc = hw >> 32
print("waves per XCC:", np.bincount(xcc, minlength=8).tolist(),
      "last end per XCC (us):", [round(float(e[xcc == k].max()), 1) if (xcc == k).any() else None
                                 for k in range(8)])
# the slowest waves: tile coordinates (8x8 px tiles) and when they ran
tx = np.tile(np.arange(tiles.shape[1]), tiles.shape[0])[ok]
order = np.argsort(-dur)[:12]
print("slowest waves (tile x, tile y, start us, duration us):",
      [(int(tx[i]), int(ry[i]), round(float(s[i]), 1), round(float(dur[i]), 1)) for i in order])
hist, edges = np.histogram(dur, bins=[0, 5, 7.5, 10, 15, 20, 30, 50, 100, 200, 1e9])
print("duration histogram (us):", list(zip([float(x) for x in edges[:-1]], hist.tolist())))
