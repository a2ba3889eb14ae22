#!/bin/bash
# GPU call (dev tool, round 6): packet kernel A/B — in-tree vs tools/variants/$V.so, C2-C4 in
# batches (AB_BATCH) and C2 one frame per launch, interleaved.
set -eu
OUT=gpurun_out/pk_ab
mkdir -p $OUT
V=${V:-pk_nowin}
AB_BATCH=${AB_BATCH:-20} N=${N:-4} bash tools/ab_env.sh "RTAMD_LIB=$PWD/raytracingengine_amd/librtamd.so" \
  "RTAMD_LIB=$PWD/tools/variants/$V.so" -- c2 c3 c4 > $OUT/ab_$V.txt 2>&1
grep "==" $OUT/ab_$V.txt
