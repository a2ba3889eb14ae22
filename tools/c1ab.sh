#!/bin/bash
# Dev tool (GPU box): C1 / mirror chain-kernel A/B over the chain register budgets
# (RTAMD_CHAIN_WAVES = 2, 3, 4 waves/SIMD) and the library builds in tools/variants.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/c1ab
mkdir -p $OUT
: > $OUT/time.txt
for w in 2 3 4 2 3 4; do
  echo "== waves $w" >> $OUT/time.txt
  RTAMD_CHAIN_WAVES=$w timeout -k 10 120 python tools/ab_time.py c1 mirror >> $OUT/time.txt 2>&1
done
