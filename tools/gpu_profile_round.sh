#!/bin/bash
# GPU call (dev tool): the round's evidence in one call — GPU suite + smoke + bench + rocprofv3
# kernel-trace stats of the bench (tools/gpu_round_end.sh), per-config kernel times and the
# 8-rank row-split balance (tools/gpu_measure.sh) with the counter passes of the given configs,
# and the per-kernel trace of the breadth-first glass renderer.
#   bash tools/gpu_profile_round.sh TAG "c2 c1 glass c3"
set -u
TAG=${1:-prof}
bash tools/gpu_round_end.sh $TAG || exit 1
bash tools/gpu_measure.sh $TAG "${2:-c2}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/glass_stats -o run -- \
  python3 tools/profile_kernel.py glass 20 > $OUT/glass_run.log 2>&1 || { tail $OUT/glass_run.log; exit 1; }
find $OUT/glass_stats -name "*kernel_stats.csv" -exec cp {} $OUT/glass_kernel_stats.csv \;
cut -c1-200 $OUT/glass_kernel_stats.csv
