#!/bin/bash
# Dev tool (GPU box): interleaved driver-shaped bench lines (--steps 20 --warmup 5, headline only)
# of the in-tree library and tools/variants/*.so.   N=3 bash tools/bench_ab.sh OUT [bench args]
set -u
OUT=$1; shift
N=${N:-3}
mkdir -p $(dirname $OUT)
: > $OUT
for r in $(seq $N); do
  for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
    line=$(RTAMD_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline "$@" 2>/dev/null) || { echo "fail $lib"; exit 1; }
    echo "$line" | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$(basename $lib)', d['value'], d['ms_per_step'], d['kernel_ms_per_frame'])" | tee -a $OUT
  done
done
