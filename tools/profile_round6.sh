#!/bin/bash
# GPU call (dev tool): round 6's profile evidence in one call.   bash tools/profile_round6.sh TAG
#   * rocprofv3 --kernel-trace --stats of the driver-shaped headline command;
#   * a kernel trace of tools/profile_kernel.py (C2, 32-frame launches) for the counter passes'
#     duration, then the counter passes (tools/pmc_passes.sh: VALU mix, GRBM clock, FETCH/WRITE);
#   * FETCH/WRITE passes of C5 (batches of 20) and of glass.
# Every step has its own time limit; the script stops at the first failure.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof6}
mkdir -p $OUT
step() { echo "== $1"; }
step kernel-trace-bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/bench_prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
step kernel-trace-c2-batch32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt32 -o kt -- \
  python3 tools/profile_kernel.py c2 6 0 32 > $OUT/kt32.log 2>&1 || { tail $OUT/kt32.log; exit 1; }
step pmc-c2
timeout -k 10 600 bash tools/pmc_passes.sh $OUT/pmc_c2 c2 6 0 32 > $OUT/pmc_c2.log 2>&1 || { tail $OUT/pmc_c2.log; exit 1; }
step traffic-c5
timeout -k 10 400 bash tools/traffic_passes.sh $OUT/tr_c5 c5 6 20 > $OUT/tr_c5.log 2>&1 || { tail $OUT/tr_c5.log; exit 1; }
step traffic-glass
timeout -k 10 400 bash tools/traffic_passes.sh $OUT/tr_glass glass 6 1 > $OUT/tr_glass.log 2>&1 || { tail $OUT/tr_glass.log; exit 1; }
echo done
