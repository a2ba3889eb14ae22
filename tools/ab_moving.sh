#!/bin/bash
# Dev tool (GPU box): interleaved moving/static camera A/B of the in-tree build and tools/variants/*.so
set -e
for r in 1 2 3; do
  for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
    echo "== $(basename $lib) $(RTAMD_LIB=$lib timeout -k 10 120 python tools/ab_moving.py ${*:-c2 c3} | tr '\n' ' ')"
  done
done
