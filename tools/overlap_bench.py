"""Dev tool: frames back to back on one stream vs alternating two streams (tail overlap)."""
import sys, time
sys.path.insert(0, '.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config


def main():
    ctx = capi.Context(0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    sc = make_config(sys.argv[1] if len(sys.argv) > 1 else "c2")
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    bufs = [(torch.empty(W * H * 3, dtype=torch.float64, device="cuda"),
             torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")) for _ in range(2)]
    o = capi.default_opts(tonemap=1)
    K = 400
    for nst in (1, 2, 1, 2):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(K):
                k = i % nst
                ctx.set_stream(streams[k].cuda_stream)
                h, l = bufs[k]
                ds.render_device(h.data_ptr(), None, l.data_ptr(), o)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / K
        print(f"{nst} stream(s): {dt * 1e6:.1f} us/frame", flush=True)


if __name__ == "__main__":
    main()
