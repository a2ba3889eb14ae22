#!/bin/bash
# Dev tool (GPU box): rocprofv3 kernel trace of tools/ab_moving.py c2 (moving-camera frames, then
# static ones) -> gpurun_out/moving/ ; tools/trace_split.py splits the dispatches by phase.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/moving
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run \
    -- python3 tools/ab_moving.py c2 > $OUT/ab.txt 2> $OUT/prof.err
find $OUT/stats -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cat $OUT/ab.txt
