#!/bin/bash
# GPU call (dev tool): per-kernel times of the breadth-first refraction-tree renderer (glass).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/glass
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 tools/profile_kernel.py glass 20 > $OUT/run.log 2>&1 || { tail $OUT/run.log; exit 1; }
cat $OUT/stats/run_kernel_stats.csv | cut -c1-220
