#!/bin/bash
# GPU call (dev tool, round 6): rank 0's rows of an N-rank C2 split (8-row blocks) rendered ALONE on
# one GPU in batches of 5 / 10 / 20 frames per launch — the render side of bench.py's
# default_batch at N > 1 (a dedicated GPU per rank; kernel time per frame from HIP events).
set -eu
OUT=gpurun_out/rank_batch
mkdir -p $OUT
for r in 2 4 8; do for b in 5 10 20; do
  echo "ranks $r batch $b: $(AB_RANKS=$r AB_BLOCK=8 AB_BATCH=$b timeout -k 10 120 python tools/ab_time.py c2 2>/dev/null)"
done; done | tee $OUT/sweep.txt
