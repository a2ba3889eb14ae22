#!/bin/bash
# GPU call (dev tool): per-wave durations and work counters (tools/build_wavestats.sh build).
set -u
OUT=gpurun_out/${1:-ws}
mkdir -p $OUT
for c in ${2:-c3}; do
  timeout -k 10 120 python -u tools/wave_stats.py $c > $OUT/wavestats_$c.txt 2>&1 || { tail $OUT/wavestats_$c.txt; exit 1; }
  cat $OUT/wavestats_$c.txt
done
