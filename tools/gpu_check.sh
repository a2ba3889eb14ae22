#!/bin/bash
# GPU call: the whole GPU suite, then interleaved A/B timing of the in-tree build against
# tools/variants/*.so.   bash tools/gpu_check.sh TAG [configs...]
set -u
TAG=$1; shift
CFGS=${*:-c2 c3 c5}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$TAG/gpu_tests.log
N=${N:-3} timeout -k 10 500 bash tools/ab_rounds.sh $CFGS > gpurun_out/$TAG/ab.log 2>&1 || { cat gpurun_out/$TAG/ab.log; exit 1; }
grep "==" gpurun_out/$TAG/ab.log
