"""Dev tool: average rocprofv3 per-dispatch counters per kernel over the pass directories.
The summary records the build the passes ran (`_build`: rt_build_info's source digest), so a
summary taken from other sources than the tree's is marked stale where it is reported."""
import csv, glob, json, os, sys
from collections import defaultdict
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
from raytracingengine_amd import capi  # noqa: E402  (loads the library; no GPU call)
info = capi.build_info()
res["_build"] = {"source_sha256": info.get("source_sha256"), "matches_tree": info["matches_tree"]}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
