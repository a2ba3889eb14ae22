#!/bin/bash
# GPU call (dev tool): tests (pytest -k), interleaved A/B kernel times, then the 8-rank
# row-split balance for the in-tree build and each tools/variants/*.so.
#   bash tools/gpu_ab_bal.sh TAG "ab configs" "balance configs" [pytest -k expr]
set -u
bash tools/gpu_ab.sh $1 "$2" "${4:-}" || exit 1
for lib in raytracingengine_amd/librtamd.so tools/variants/*.so; do
  echo "== $lib"
  RTAMD_LIB=$lib timeout -k 10 200 python -u tools/tile_balance.py 8 16 $3 || exit 1
done > gpurun_out/$1/balance.log 2>&1
grep -E "==|rank_sum" gpurun_out/$1/balance.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip()); continue
    d = json.loads(l); print(d['config'], 'max/mean', d['max_over_mean'], 'full', d['full_frame_ms'], 'sum/full', d['rank_sum_over_full'], 'ideal x', d['ideal_speedup'])
"
