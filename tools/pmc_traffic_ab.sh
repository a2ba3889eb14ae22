#!/bin/bash
# Dev tool (GPU box): HBM traffic per launch (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction) of
# the packet kernel for the in-tree build and tools/variants/*.so.   bash tools/pmc_traffic_ab.sh c2
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmctraffic
mkdir -p $OUT
for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
  tag=$(basename $lib .so)
  for cfg in "$@"; do
    for grp in FETCH_SIZE WRITE_SIZE; do
      RTAMD_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/${tag}_${cfg}_$grp -o pmc -- python3 tools/profile_kernel.py $cfg 10 > $OUT/${tag}_${cfg}_$grp.log 2>&1
    done
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
vals = defaultdict(list)
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    tag = os.path.relpath(f, out).split(os.sep)[0].rsplit("_", 2)[0]
    for row in csv.DictReader(open(f)):
        if "packet" in row["Kernel_Name"]:
            vals[(tag, row["Counter_Name"])].append(float(row["Counter_Value"]))
for tag in sorted({t for t, _ in vals}):
    fs = sum(vals[(tag, "FETCH_SIZE")]) / max(1, len(vals[(tag, "FETCH_SIZE")]))
    ws = sum(vals[(tag, "WRITE_SIZE")]) / max(1, len(vals[(tag, "WRITE_SIZE")]))
    print(f"{tag:28s} fetch {fs*1024*2/1e6:8.2f} MB  write {ws*1024/1e6:8.2f} MB  total {(fs*2+ws)*1024/1e6:8.2f} MB")
PY
