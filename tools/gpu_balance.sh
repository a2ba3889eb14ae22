#!/bin/bash
# GPU call (dev tool): every config's kernel time through the default path, and the 8-rank
# row-split balance of C3/C4/C5 for several block sizes.   bash tools/gpu_balance.sh TAG
set -u
OUT=gpurun_out/${1:-bal}
mkdir -p $OUT
timeout -k 10 300 python -u tools/time_configs.py > $OUT/configs.txt 2>&1 || { tail $OUT/configs.txt; exit 1; }
cat $OUT/configs.txt
timeout -k 10 300 python -u tools/tile_balance.py 8 0,8,16,32 c3 c4 c5 > $OUT/balance.jsonl 2>&1 || { tail $OUT/balance.jsonl; exit 1; }
cat $OUT/balance.jsonl
