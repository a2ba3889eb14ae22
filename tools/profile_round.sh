#!/bin/bash
# Dev tool (runs on the GPU box): the profiles committed for a round.
#   bash tools/profile_round.sh r01_v5
# -> gpurun_out/<tag>/{bench.json, stats/, pmc/} ; copy the summaries into profiles/.
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python bench.py --no-cpu-baseline --inflight 2 > $OUT/bench_pipelined.json 2>> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --no-cpu-baseline --steps 200 > $OUT/bench_prof.json 2> $OUT/prof.err
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc/p_$grp -o pmc -- python3 tools/profile_kernel.py c2 20 > $OUT/pmc_$grp.log 2>&1
done
python3 tools/pmc_summary.py $OUT/pmc > /dev/null
python3 tools/traffic_summary.py $OUT/pmc/summary.json $OUT/pmc_c2_frames.json c2 $((1920*1080*27))
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cat $OUT/bench.json
