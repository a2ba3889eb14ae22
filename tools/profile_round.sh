#!/bin/bash
# GPU call (dev tool): the evidence of a round in one call.   bash tools/profile_round.sh TAG
#   * the GPU test suite (-s: the parity tests print their byte-flip counts);
#   * the default bench line, and rocprofv3 --kernel-trace --stats of the headline command;
#   * rocprofv3 counter passes (tools/pmc_passes.sh) of the C2 batch launch (32 frames) and of the
#     bigmesh triangle variant, incl. FETCH_SIZE / WRITE_SIZE for the HBM traffic;
#   * the 8-rank row split with frames in flight (tools/inflight_balance.py).
# Summaries afterwards: tools/valu_summary.py, tools/traffic_summary.py.  Every step has its own
# time limit; the script stops at the first failure.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
step() { echo "== $1"; }
step tests
timeout -k 10 600 python -u -m pytest -q -s -m gpu --timeout 300 --timeout-method thread tests/ \
  > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
step bench
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
head -c 400 $OUT/bench.json; echo
step kernel-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 bench.py --no-cpu-baseline --no-extras > $OUT/bench_prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -4 $OUT/kernel_stats.csv | cut -c1-160
step pmc-c2
timeout -k 10 500 bash tools/pmc_passes.sh $OUT/pmc_c2 c2 6 0 32 > $OUT/pmc_c2.log 2>&1 || { tail $OUT/pmc_c2.log; exit 1; }
step pmc-bigmesh
timeout -k 10 500 bash tools/pmc_passes.sh $OUT/pmc_bigmesh bigmesh 10 > $OUT/pmc_bigmesh.log 2>&1 || { tail $OUT/pmc_bigmesh.log; exit 1; }
step inflight
timeout -k 10 400 python -u tools/inflight_balance.py 8 1,2 c2 c5 > $OUT/inflight.jsonl 2> $OUT/inflight.err || { tail $OUT/inflight.err; exit 1; }
echo done
