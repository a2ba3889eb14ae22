#!/bin/bash
# GPU call (dev tool): the GPU test suite (with -s: the parity tests print their byte-flip
# counts, "FLIPS ..."), smoke(), and the default bench line of the current tree, each under its
# own time limit.   bash tools/gpu_suite.sh TAG
set -u
TAG=${1:-suite}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
grep FLIPS $OUT/gpu_tests.log > $OUT/flips.txt || true
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
