"""Dev tool: splits a rocprofv3 kernel trace of tools/ab_moving.py into its phases (the packet
kernel's dispatches in order: moving-camera warm-up + 4x50 timed, then static warm-up + 4x50) and
prints the average duration of the last 200 dispatches of each phase.
    python tools/trace_split.py gpurun_out/moving/kernel_trace.csv"""
import csv, json, sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "packet_direct_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
img = [r for r in csv.DictReader(open(sys.argv[1])) if "packet_image_kernel" in r["Kernel_Name"]]
t_img = int(img[0]["Start_Timestamp"]) if img else None  # the static camera's setup launch
mv = [r for r in rows if t_img is None or int(r["Start_Timestamp"]) < t_img]
st = [r for r in rows if t_img is not None and int(r["Start_Timestamp"]) > t_img]
dur = lambda rs: [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs]
out = {"moving_last200_avg_ns": sum(dur(mv[-200:])) / 200, "moving_dispatches": len(mv),
       "static_last200_avg_ns": sum(dur(st[-200:])) / 200, "static_dispatches": len(st)}
print(json.dumps(out))
