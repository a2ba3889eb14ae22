"""Dev tool: kernel time of each rank's rows of a frame, rendered one after another on one GPU —
the load imbalance of the multi-GPU row split measured without 8 GPUs, for
contiguous tiles and for block-cyclic rows."""
import sys, json
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
from raytracingengine_amd.distributed import plan_rows, render_opts_for, row_ranges
ctx = capi.Context(0)
s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
BLOCKS = [int(b) for b in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "16"])]
for name in sys.argv[3:] or ["c2", "c3", "c4"]:
    sc = make_config(name)
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    hdr = torch.empty(W * H * 3, dtype=torch.float64, device="cuda")
    for block in BLOCKS:
        ts = []
        for r in range(n):
            ranges = row_ranges(r, n, H, block)
            o = render_opts_for(ranges, r, n, H, block, tonemap=-1, flags=capi.RT_FLAG_TIME_KERNEL)
            for _ in range(2):
                ds.render_device(hdr.data_ptr(), None, None, o)
            ctx.reset_stats()
            for _ in range(5):
                ds.render_device(hdr.data_ptr(), None, None, o)
            st = ctx.stats()
            ts.append(st.kernel_ms / st.launches)
        mean = sum(ts) / n
        print(json.dumps({"config": name, "ranks": n, "row_block": block,
                          "ms": [round(t, 4) for t in ts],
                          "max_over_mean": round(max(ts) / mean, 3)}), flush=True)
    ds.close()
