"""Dev tool (GPU box, under rocprofv3 --kernel-trace): C2 frame batches of 1..32 frames through
the fix-up variant (RTAMD_PK_FIX=1), 30 launches each after a clock warm-up, so the kernel trace
gives packet_fixup_kernel's duration against the size of its list (~1 600 pixels per frame).
    rocprofv3 --kernel-trace --output-format csv -d OUT -o fx -- python3 tools/fixup_scaling.py
    python3 tools/fixup_scaling.py --summarize OUT"""
import csv, glob, json, os, sys, time
from collections import defaultdict
sys.path.insert(0, '.')


def summarize(out):
    rows = []
    for f in glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    res = defaultdict(list)
    last_z = None
    for r in rows:
        k = r["Kernel_Name"]
        if "packet_direct_kernel" in k:
            last_z = int(r.get("Grid_Size_Z", r.get("Grid_Z", 1)) or 1)
        elif "packet_fixup_kernel" in k and last_z:
            res[last_z].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out_rows = {z: {"n": len(v), "median_us": sorted(v)[len(v) // 2]} for z, v in sorted(res.items())}
    print(json.dumps(out_rows))


if __name__ == "__main__":
    if "--summarize" in sys.argv:
        summarize(sys.argv[-1])
        sys.exit(0)
    os.environ["RTAMD_PK_FIX"] = "1"
    import torch
    from raytracingengine_amd import capi
    from raytracingengine_amd.configs import make_config
    ctx = capi.Context(0)
    s = torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
    sc = make_config("c2")
    ds = ctx.scene(sc)
    W, H = sc.camera.width, sc.camera.height
    hdr = torch.empty(32 * W * H * 3, dtype=torch.float64, device="cuda")
    ldr = torch.empty(32 * W * H * 3, dtype=torch.uint8, device="cuda")
    o = capi.default_opts(tonemap=1)
    for n in (1, 2, 4, 8, 16, 20, 32):
        cams = ds.cameras([ds.camera["position"][0]] * n)
        t_end = time.perf_counter() + 0.05
        while time.perf_counter() < t_end:
            ds.render_batch(cams, hdr.data_ptr(), None, ldr.data_ptr(), o)
            torch.cuda.synchronize()
        for _ in range(30):
            ds.render_batch(cams, hdr.data_ptr(), None, ldr.data_ptr(), o)
        torch.cuda.synchronize()
