#!/bin/bash
# GPU call (dev tool): GPU suite, then C1 AA=32 A/B of the sphere-free multi-sample chain variant.
set -u
OUT=gpurun_out/c1aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  AB_TOOL=tools/ab_time.py timeout -k 10 300 bash tools/ab_variants.sh c1_aa32 c1 2>&1 | grep -v amdgpu.ids
done > $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
