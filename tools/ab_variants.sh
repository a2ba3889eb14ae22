#!/bin/bash
# Dev tool: time the packet kernel of several library builds (tools/variants/*.so, git-ignored)
# against the in-tree librtamd.so on the same box.  Usage: bash tools/ab_variants.sh c2 c3
# (AB_TOOL=tools/ab_time.py times the headline mode: f64 HDR + fused Reinhard bytes)
set -e
mkdir -p gpurun_out
for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
  echo "== $lib"
  RTAMD_LIB=$lib timeout -k 10 300 python ${AB_TOOL:-tools/ab_kernels.py} "$@"
done


