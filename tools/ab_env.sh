#!/bin/bash
# Dev tool (GPU box): interleaved A/B rounds of tools/ab_time.py between environment settings of
# the in-tree library (e.g. RTAMD_PK_AXIS=1 vs RTAMD_PK_AXIS=0).
#   N=3 AB_BATCH=32 bash tools/ab_env.sh "RTAMD_PK_AXIS=1" "RTAMD_PK_AXIS=0" -- c2 c3
set -e
N=${N:-3}
envs=()
while [ "$1" != "--" ]; do envs+=("$1"); shift; done
shift
for r in $(seq $N); do
  for e in "${envs[@]}"; do
    echo "== $e $(env $e timeout -k 10 120 python tools/ab_time.py "$@" | tr '\n' ' ')"
  done
done
