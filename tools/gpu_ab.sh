#!/bin/bash
# GPU call (dev tool): GPU parity suite of the in-tree build, interleaved A/B kernel times of the
# in-tree build against tools/variants/*.so, and (BAL=1) the 8-rank row-split balance of each.
#   bash tools/gpu_ab.sh TAG "configs" [pytest -k expr]
set -u
OUT=gpurun_out/$1
CFGS=${2:-c2 c3 c4 c5}
mkdir -p $OUT
if [ -n "${3:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider -k "$3" > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
N=${N:-3} timeout -k 10 600 bash tools/ab_rounds.sh $CFGS > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
if [ "${BAL:-0}" = 1 ]; then
  for lib in raytracingengine_amd/librtamd.so tools/variants/*.so; do
    echo "== $lib"
    RTAMD_LIB=$lib timeout -k 10 200 python -u tools/tile_balance.py 8 8,16 ${BALCFG:-c3 c4} || exit 1
  done > $OUT/balance.log 2>&1
  grep -E "==|max_over" $OUT/balance.log | sed 's/"ms": \[[^]]*\], //'
fi
