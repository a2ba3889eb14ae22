#!/bin/bash
# GPU call (dev tool, round 6): the refilling deferred direct pass (wf_direct_refill_kernel) —
# parity tests, then interleaved A/B: in-tree (RT_WF_REFILL=32, 4 waves) vs refill 16 / 48, 3 waves,
# the per-record kernels (refill0), and the level kernels shading in place (RTAMD_WF_DEFER=0).
set -eu
export TMPDIR=/tmp
OUT=gpurun_out/glass_refill
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "deferred_direct" tests/test_gpu_fullsize.py::test_full_glass_deferred_direct_equals_in_level \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
V=$PWD/tools/variants
N=${N:-3} bash tools/ab_env.sh "RTAMD_WF_DEFER=1" "RTAMD_WF_DEFER=1 RTAMD_LIB=$V/refill16.so" \
  "RTAMD_WF_DEFER=1 RTAMD_LIB=$V/refill48.so" "RTAMD_WF_DEFER=1 RTAMD_LIB=$V/refill_w3.so" \
  "RTAMD_WF_DEFER=1 RTAMD_LIB=$V/refill0.so" "RTAMD_WF_DEFER=0" -- glass > $OUT/ab.txt 2>&1
grep "==" $OUT/ab.txt
RTAMD_WF_DEFER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $OUT/kt -o run -- python3 tools/profile_kernel.py glass 20 > $OUT/kt.log 2>&1
cut -d, -f1-4 $OUT/kt/run_kernel_stats.csv | cut -c1-150
