#!/bin/bash
# GPU call (dev tool): per-kernel times of the glass frame with the deferred direct pass
# (RTAMD_WF_DEFER=1) and without it (0), rocprofv3 kernel traces of 20 frames each.
set -eu
export TMPDIR=/tmp
OUT=gpurun_out/glass_ab
mkdir -p $OUT
for d in 1 0; do
  RTAMD_WF_DEFER=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/defer$d -o run -- python3 tools/profile_kernel.py glass 20 > $OUT/defer$d.log 2>&1
  echo "== RTAMD_WF_DEFER=$d"
  cut -d, -f1-4 $OUT/defer$d/run_kernel_stats.csv | cut -c1-160
done
