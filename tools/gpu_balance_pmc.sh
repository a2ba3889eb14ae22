#!/bin/bash
# GPU call (dev tool): the 8-rank row-split balance of C2-C5 (tools/tile_balance.py) and the C3
# counter passes (LDS conflicts, VALU, HBM traffic) of the in-tree build.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u tools/tile_balance.py 8 8,16 c2 c3 c4 c5 > $OUT/balance.jsonl 2> $OUT/balance.err \
    || { tail -20 $OUT/balance.err; exit 1; }
cat $OUT/balance.jsonl
for cfg in ${2:-c3}; do
  bash tools/pmc_passes.sh $OUT/pmc_$cfg $cfg 10 > $OUT/pmc_$cfg.log 2>&1 || { tail -20 $OUT/pmc_$cfg.log; exit 1; }
done
