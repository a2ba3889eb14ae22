#!/bin/bash
# GPU call (dev tool): per-config kernel times, the 8-rank row-split balance of C2-C5 and the
# counter passes (tools/pmc_passes.sh) of the given configs.   bash tools/gpu_measure.sh TAG "c3 glass"
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u tools/time_configs.py > $OUT/configs.txt 2>&1 || { tail $OUT/configs.txt; exit 1; }
cat $OUT/configs.txt
timeout -k 10 300 python -u tools/tile_balance.py 8 16 c2 c3 c4 c5 > $OUT/balance.jsonl 2> $OUT/balance.err \
    || { tail -20 $OUT/balance.err; exit 1; }
cat $OUT/balance.jsonl
for cfg in ${2:-}; do
  bash tools/pmc_passes.sh $OUT/pmc_$cfg $cfg 10 > $OUT/pmc_$cfg.log 2>&1 || { tail -20 $OUT/pmc_$cfg.log; exit 1; }
done
