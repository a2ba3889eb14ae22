#!/bin/bash
# Dev tool (GPU box): the round-2 profiles.  FP64 issue rates (tools/micro/fp64_rates.hip), the
# counter passes of the C2 packet kernel and the C1 chain kernel (tools/pmc_passes.sh), and the
# rocprofv3 kernel-trace summary of the headline bench command.  -> gpurun_out/r02/
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/micro/fp64_rates.hip -o /tmp/fp64_rates
timeout -k 10 120 /tmp/fp64_rates > $OUT/fp64_rates.txt 2>&1
timeout -k 10 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
timeout -k 10 400 bash tools/pmc_passes.sh $OUT/pmc_c2 c2 20 > $OUT/pmc_c2.log 2>&1
timeout -k 10 400 bash tools/pmc_passes.sh $OUT/pmc_c1 c1 10 > $OUT/pmc_c1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --no-cpu-baseline --no-extras > $OUT/bench_prof.json 2> $OUT/prof.err
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
