"""Dev tool: average rocprofv3 per-dispatch counters per kernel over the pass directories."""
import csv, glob, json, os, sys
from collections import defaultdict
out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if not any(s in k for s in ("trace", "packet", "wf_", "box_chain", "level", "fold")):
            continue
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {}
for k, d in acc.items():
    res[k[:80]] = {c: sum(v) / len(v) for c, v in sorted(d.items())}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
