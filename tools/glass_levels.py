"""Dev tool: per-level view of the breadth-first renderer (glass) from tools/pmc_passes.sh
counter passes and a rocprofv3 kernel trace: each frame is fill, fill, level 0..K, folds K-1..1,
final, fix-up; dispatches are matched to their position in the frame.
    python tools/glass_levels.py gpurun_out/glass_pmc [gpurun_out/glass/stats/run_kernel_trace.csv]"""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
trace = sys.argv[2] if len(sys.argv) > 2 else None


def frames(rows):
    """Split a dispatch-ordered list of (name, ...) into frames starting at each level-0 launch."""
    fr, cur, seen_level = [], [], False
    for r in rows:
        name = r[0]
        if "wf_level_kernel" in name and not seen_level:
            if cur:
                fr.append(cur)
            cur, seen_level = [], True
        if "wf_level_kernel" not in name:
            seen_level = False
        cur.append(r)
    if cur:
        fr.append(cur)
    return fr


def tag(frame):
    out, lv, fo = [], 0, 0
    for r in frame:
        n = r[0]
        if "wf_level_kernel" in n:
            out.append((f"level{lv}", r)); lv += 1
        elif "wf_fold" in n:
            out.append((f"fold{fo}", r)); fo += 1
        elif "wf_final" in n:
            out.append(("final", r))
        elif "trace_kernel" in n:
            out.append(("fixup", r))
    return out


cnt = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    disp = defaultdict(dict)
    names = {}
    for row in csv.DictReader(open(f)):
        d = int(row["Dispatch_Id"])
        names[d] = row["Kernel_Name"]
        disp[d][row["Counter_Name"]] = float(row["Counter_Value"])
    rows = [(names[d], disp[d]) for d in sorted(disp)]
    for fr in frames([r for r in rows if "rocclr" not in r[0]])[2:]:  # skip the clock warm-up's first
        for t, (n, c) in tag(fr):
            for k, v in c.items():
                cnt[t][k].append(v)
dur = defaultdict(list)
if trace:
    rows = []
    for row in csv.DictReader(open(trace)):
        rows.append((row["Kernel_Name"], (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3))
    for fr in frames([r for r in rows if "rocclr" not in r[0]])[2:]:
        for t, (n, us) in tag(fr):
            dur[t].append(us)
order = sorted(cnt, key=lambda t: (t[0] != "l", t[0] == "f" and t != "final", t))
tot = 0.0
for t in sorted(set(cnt) | set(dur), key=lambda t: ({"l": 0, "f": 1, "fi": 2}.get(t[:2] if t == "final" else t[0], 3), len(t), t)):
    c = {k: sum(v) / len(v) for k, v in cnt[t].items()}
    w = c.get("SQ_WAVES", 0) or 1
    us = sum(dur[t]) / len(dur[t]) if dur[t] else float("nan")
    tot += us if dur[t] else 0
    print(f"{t:8s} {us:8.1f} us  waves {c.get('SQ_WAVES', 0):8.0f}  valu/wave {c.get('SQ_INSTS_VALU', 0) / w:7.0f}  "
          f"busy_valu {4 * c.get('SQ_ACTIVE_INST_VALU', 0) / max(1, c.get('GRBM_GUI_ACTIVE', 0) * 1024 / 8):5.2f}  "
          f"fetch {2 * c.get('FETCH_SIZE', 0) / 1024:7.1f} MB  write {c.get('WRITE_SIZE', 0) / 1024:7.1f} MB")
print(f"total {tot:.1f} us per frame")
