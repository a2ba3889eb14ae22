#!/bin/bash
# GPU call (dev tool): the hand-off's parity tests, its moving-camera A/B, then the round-end suite.
set -u
OUT=gpurun_out/pub
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q \
    -k "moving or packet_image or fresh" --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 bash tools/ab_pub.sh c2 c3 c5 > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
[ "${1:-r02f}" = none ] || bash tools/gpu_round_end.sh ${1:-r02f}
