#!/bin/bash
# GPU call (dev tool): tests, the driver-shaped bench line, and interleaved A/B rounds of the
# in-tree library against tools/variants/*.so.   bash tools/gpu_round.sh TAG [ab configs...]
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06}; shift || true
mkdir -p $OUT
echo "== tests"
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
echo "== bench"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; cat $OUT/bench.json | head -c 2000; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print({k:d[k] for k in ('value','ms_per_step','kernel_ms_per_frame','parity')})"
if [ $# -gt 0 ]; then
  echo "== ab $*"
  for B in 20 1; do
    AB_BATCH=$B N=3 timeout -k 10 600 bash tools/ab_rounds.sh "$@" > $OUT/ab_b$B.txt 2>&1 || { tail $OUT/ab_b$B.txt; exit 1; }
    cat $OUT/ab_b$B.txt
  done
fi
echo done
