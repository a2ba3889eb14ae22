#!/bin/bash
# GPU call (dev tool): rocprofv3 kernel trace + stats of tools/ab_time.py over the given configs.
#   bash tools/gpu_ktrace.sh TAG "c1 c2"
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 tools/ab_time.py ${2:-c1} > $OUT/log.txt 2>&1 || { tail -20 $OUT/log.txt; exit 1; }
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
grep -v "^W2026" $OUT/log.txt | tail -5
cut -c1-180 $OUT/kernel_stats.csv
