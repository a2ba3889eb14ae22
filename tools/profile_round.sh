#!/bin/bash
# GPU call (dev tool): the profiles of a round.   bash tools/profile_round.sh TAG
#   * rocprofv3 counter passes (tools/pmc_passes.sh) of the C2 packet kernel, the C3 packet kernel
#     and the C1 chain kernel, incl. FETCH_SIZE / WRITE_SIZE for the HBM traffic;
#   * rocprofv3 --kernel-trace --stats of the headline bench command;
#   * every config's kernel time (tools/time_configs.py) and the 8-rank row-split balance.
# Summaries are made afterwards with tools/pmc_summary.py / valu_summary.py / traffic_summary.py.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
for c in c2 c3 c1; do
  timeout -k 10 500 bash tools/pmc_passes.sh $OUT/pmc_$c $c 10 > $OUT/pmc_$c.log 2>&1 || { tail $OUT/pmc_$c.log; exit 1; }
  echo "pmc $c done"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 bench.py --no-cpu-baseline --no-extras > $OUT/bench_prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cat $OUT/bench_prof.json
timeout -k 10 300 python -u tools/time_configs.py > $OUT/configs.txt 2>&1 || { tail $OUT/configs.txt; exit 1; }
cat $OUT/configs.txt
timeout -k 10 300 python -u tools/tile_balance.py 8 0,16 c2 c3 c4 c5 > $OUT/balance.jsonl 2>&1 || { tail $OUT/balance.jsonl; exit 1; }
grep max_over $OUT/balance.jsonl | sed 's/"ms": \[[^]]*\], //'
