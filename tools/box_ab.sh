#!/bin/bash
# GPU call (dev tool, round 6): box kernel A/B — in-tree vs tools/variants/box_*.so on mirror and C1
set -eu
OUT=gpurun_out/box_ab
mkdir -p $OUT
L=$PWD/raytracingengine_amd/librtamd.so
N=${N:-3} bash tools/ab_env.sh "RTAMD_LIB=$L" "RTAMD_LIB=$PWD/tools/variants/box_maxilp.so" \
  "RTAMD_LIB=$PWD/tools/variants/box_occ_unroll2.so" -- mirror c1 > $OUT/ab.txt 2>&1
grep "==" $OUT/ab.txt
