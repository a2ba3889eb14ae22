#!/bin/bash
# GPU call (round 6, end): the driver's bench shapes on this tree — the default line (256 frames,
# extras, cpu_baseline) and the driver's --steps 20 --warmup 5 line.
set -eu
OUT=gpurun_out/final
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err
python -c "
import json
for f in ('bench_default', 'bench_s20'):
    d = json.load(open('$OUT/' + f + '.json'))
    print(f, d['value'], d['ms_per_step'], d['kernel_ms_per_frame'], d['parity'], d['build']['matches_tree'])"
