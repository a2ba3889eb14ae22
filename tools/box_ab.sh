#!/bin/bash
# GPU call (dev tool, round 6): box kernel A/B — in-tree vs tools/variants/$V.so on mirror and C1
set -eu
OUT=gpurun_out/box_ab
mkdir -p $OUT
L=$PWD/raytracingengine_amd/librtamd.so
N=${N:-3} bash tools/ab_env.sh "RTAMD_LIB=$L" "RTAMD_LIB=$PWD/tools/variants/${V:-box_pipe}.so" \
  -- mirror c1 > $OUT/ab_${V:-box_pipe}.txt 2>&1
grep "==" $OUT/ab_${V:-box_pipe}.txt
