#!/bin/bash
# GPU call (dev tool, round 6): waves/SIMD of the AA=1 packet variants C3 / C4 take (5 in-tree)
# against 4 and 6 (tools/variants/aa1w4.so, aa1w6.so), batches of 4 frames, interleaved.
set -eu
OUT=gpurun_out/c34_waves
mkdir -p $OUT
V=$PWD/tools/variants
AB_BATCH=4 N=${N:-3} bash tools/ab_env.sh "RTAMD_LIB=$PWD/raytracingengine_amd/librtamd.so" \
  "RTAMD_LIB=$V/aa1w4.so" "RTAMD_LIB=$V/aa1w6.so" -- c3 c4 > $OUT/ab.txt 2>&1
grep "==" $OUT/ab.txt
