#!/bin/bash
# GPU call (dev tool, round 6): what the deferred direct pass's time is made of — the in-tree
# pass against ablations with wrong images (tools/variants/dq_nomask.so: every sphere in every
# shadow packet; dq_nomarch.so: T = 1, no computeTransmittance march), kernel traces.
set -eu
export TMPDIR=/tmp
OUT=gpurun_out/glass_ablate
mkdir -p $OUT
for v in intree dq_nomask dq_nomarch; do
  lib=$PWD/raytracingengine_amd/librtamd.so
  [ $v != intree ] && lib=$PWD/tools/variants/$v.so
  RTAMD_WF_DEFER=1 RTAMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/$v -o run -- python3 tools/profile_kernel.py glass 20 > $OUT/$v.log 2>&1
  echo "== $v"
  cut -d, -f1-3 $OUT/$v/run_kernel_stats.csv | cut -c1-160
done
