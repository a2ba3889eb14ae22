#!/bin/bash
# GPU call (dev tool, round 6): the deferred direct pass with its queue windows reordered by hit
# primitive (in-tree, RT_WF_DQ_SORT=4) against queue order (tools/variants/dqsort0.so) and against
# the level kernels shading in place (RTAMD_WF_DEFER=0): parity tests, interleaved A/B, kernel trace.
set -eu
export TMPDIR=/tmp
OUT=gpurun_out/glass_sort
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "deferred_direct" tests/test_gpu_fullsize.py::test_full_glass_deferred_direct_equals_in_level \
  > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
N=${N:-4} bash tools/ab_env.sh "RTAMD_WF_DEFER=1" "RTAMD_WF_DEFER=1 RTAMD_LIB=tools/variants/dqsort0.so" \
  "RTAMD_WF_DEFER=0" -- glass > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
for v in sorted unsorted; do
  lib=librtamd.so; [ $v = unsorted ] && lib=../tools/variants/dqsort0.so
  RTAMD_WF_DEFER=1 RTAMD_LIB=$PWD/raytracingengine_amd/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/$v -o run -- python3 tools/profile_kernel.py glass 20 > $OUT/$v.log 2>&1
  echo "== $v"
  cut -d, -f1-4 $OUT/$v/run_kernel_stats.csv | cut -c1-160
done
