#!/bin/bash
# Dev tool (GPU box): C2 moving-camera time against the hand-off's first-round threshold.
set -e
for r in 1 2 3; do
  for v in 2560 1280 1920 3200; do
    echo "== first=$v $(RTAMD_PK_PUB_FIRST=$v timeout -k 10 120 python tools/ab_moving.py c2 | tr '\n' ' ')"
  done
done
