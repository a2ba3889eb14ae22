#!/bin/bash
# GPU call (dev tool): GPU suite, then the single-light lean variant A/B (C2; C3 as control).
set -u
OUT=gpurun_out/l1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  AB_TOOL=tools/ab_time.py timeout -k 10 300 bash tools/ab_variants.sh c2 c3 2>&1 | grep -v amdgpu.ids
done > $OUT/ab.txt || { cat $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
