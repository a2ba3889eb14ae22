#!/bin/bash
# Dev tool (GPU box): moving/static camera times with the in-launch image hand-off off
# (RTAMD_PK_PUB=0), on (default first round), and with other first-round sizes, interleaved.
#   bash tools/ab_pub.sh [configs...]
set -e
for r in 1 2 3; do
  for v in "RTAMD_PK_PUB=1" "RTAMD_PK_PUB=0" "RTAMD_PK_PUB_FIRST=0" "RTAMD_PK_PUB_FIRST=5120"; do
    echo "== $v $(env $v timeout -k 10 120 python tools/ab_moving.py ${*:-c2 c3 c5} | tr '\n' ' ')"
  done
done
