#!/bin/bash
# GPU call (dev tool): the GPU test suite, smoke(), the default bench line, and the rocprofv3
# kernel-trace summary of the headline bench command, each step under its own time limit.
#   bash tools/gpu_round_end.sh TAG   -> gpurun_out/TAG/
set -u
TAG=${1:-final}
OUT=gpurun_out/$TAG
bash tools/gpu_suite.sh $TAG || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run \
    -- python3 bench.py --no-cpu-baseline --no-extras > $OUT/bench_prof.json 2> $OUT/prof.err \
    || { tail -20 $OUT/prof.err; exit 1; }
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cat $OUT/bench_prof.json
head -5 $OUT/kernel_stats.csv
