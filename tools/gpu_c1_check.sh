#!/bin/bash
# GPU call (dev tool): C1 parity tests of the in-tree build, then the chain-variant A/B on C1.
set -u
OUT=gpurun_out/c1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "c1 or chain or box" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  AB_TOOL=tools/ab_time.py timeout -k 10 300 bash tools/ab_variants.sh c1 2>&1 | grep -v amdgpu.ids
done > $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
