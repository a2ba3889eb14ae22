"""Dev tool: per-wave instruction counts of the trace kernels from tools/pmc_ab.sh passes."""
import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "*"))):
    if not os.path.isdir(d):
        continue
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "packet" not in k and "trace" not in k:
                continue
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, c in acc.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        w = m.get("SQ_WAVES", 1.0)
        print(f"{os.path.basename(d):24s} {k[:48]:48s} waves {w:9.0f} valu/wave {m.get('SQ_INSTS_VALU', 0)/w:7.1f} "
              f"salu/wave {m.get('SQ_INSTS_SALU', 0)/w:6.1f} br/wave {m.get('SQ_INSTS_BRANCH', 0)/w:6.1f} lds/wave {m.get('SQ_INSTS_LDS', 0)/w:5.1f} trans/wave {m.get('SQ_INSTS_VALU_TRANS_F64', 0)/w:5.1f} "
              f"active_valu/wave {m.get('SQ_ACTIVE_INST_VALU', 0)/w:7.1f} wave_cycles/wave {m.get('SQ_WAVE_CYCLES', 0)/w:8.1f}")
