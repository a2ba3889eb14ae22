#!/bin/bash
# GPU call: grazing-shadow test on the pre-fix build (expected to fail) and the fixed build,
# the whole GPU suite, then interleaved A/B timing.
set -u
mkdir -p gpurun_out/s3
RTAMD_LIB=tools/variants/before.so timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -k grazing -q -p no:cacheprovider > gpurun_out/s3/before.log 2>&1; rc=$?
echo "before-fix grazing test rc=$rc"; tail -4 gpurun_out/s3/before.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s3/gpu_tests.log 2>&1 || { tail -30 gpurun_out/s3/gpu_tests.log; exit 1; }
tail -2 gpurun_out/s3/gpu_tests.log
N=2 timeout -k 10 400 bash tools/ab_rounds.sh c2 c3 c5 > gpurun_out/s3/ab.log 2>&1 || exit $?
cat gpurun_out/s3/ab.log
