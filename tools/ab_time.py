"""Dev tool: packet-kernel time only (no bit-exactness check), for ablation builds whose images
are deliberately wrong.  RTAMD_LIB selects the build."""
import os, sys, json, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
for name in sys.argv[1:] or ["c2"]:
    base, _, aa = name.partition("_aa")  # e.g. c1_aa32, mirror_aa4
    sc = make_config(base, aa=int(aa) if aa else 1)
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    B = int(os.environ.get("AB_BATCH", "1"))  # > 1: rt_render_batch launches of B frames
    hdr = torch.empty(B * W * H * 3, dtype=torch.float64, device="cuda")
    ldr = torch.empty(B * W * H * 3, dtype=torch.uint8, device="cuda")
    cams = ds.cameras([ds.camera["position"][0]] * B)

    def render(o):
        if B > 1:
            ds.render_batch(cams, hdr.data_ptr(), None, ldr.data_ptr(), o)
        else:
            ds.render_device(hdr.data_ptr(), None, ldr.data_ptr(), o)
    o = capi.default_opts(tonemap=1, flags=capi.RT_FLAG_TIME_KERNEL | int(os.environ.get("AB_FLAGS", "0")))
    if os.environ.get("AB_RANKS"):  # one rank's block-cyclic rows of an N-rank split (AB_BLOCK rows)
        n = int(os.environ["AB_RANKS"])
        blk = int(os.environ.get("AB_BLOCK", "16"))
        o.row_begin, o.row_end, o.row_block, o.row_cycle = 0, H, blk, n
    t_end = time.perf_counter() + 0.05   # the GPU's clock ramp (tools/clock_ramp.py)
    while time.perf_counter() < t_end:
        for _ in range(8):
            render(o)
        torch.cuda.synchronize()
    best = 1e9
    for _ in range(4):
        ctx.reset_stats()
        for _ in range(20 if B == 1 else 4):
            render(o)
        st = ctx.stats(); best = min(best, st.kernel_ms / st.launches / B)
    print(name, "%.1f us" % (best * 1e3) + (f" per frame (batches of {B})" if B > 1 else ""), flush=True)
    ds.close()
