#!/bin/bash
# Dev tool: interleaved A/B rounds (in-tree lib + tools/variants/*.so), N rounds of ab_time.
set -e
N=${N:-3}
for r in $(seq $N); do
  for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
    echo "== $(basename $lib) $(RTAMD_LIB=$lib timeout -k 10 120 python tools/ab_time.py "$@" | tr '\n' ' ')"
  done
  if [ -n "${AB_FLAGS_EXTRA:-}" ]; then  # the in-tree build once more with extra render flags
    echo "== flags=$AB_FLAGS_EXTRA $(AB_FLAGS=$AB_FLAGS_EXTRA timeout -k 10 120 python tools/ab_time.py "$@" | tr '\n' ' ')"
  fi
done
