#!/bin/bash
# GPU call (dev tool): HBM traffic of one config's launches — rocprofv3 FETCH_SIZE and WRITE_SIZE
# in separate passes over tools/profile_kernel.py — for the in-tree build and every
# tools/variants/*.so, one pmc_summary.py summary per build (OUT/<build>/summary.json; bytes =
# FETCH_SIZE x 2 (gfx950) + WRITE_SIZE, KiB).
#   bash tools/traffic_passes.sh OUT CONFIG [REPS] [BATCH]
set -e
export TMPDIR=/tmp
OUT=$1; CFG=$2; REPS=${3:-6}; BATCH=${4:-1}
for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
  name=$(basename $lib .so)
  O=$OUT/$name
  mkdir -p $O
  for p in 1:FETCH_SIZE 2:WRITE_SIZE; do
    RTAMD_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc ${p#*:} --output-format csv \
      -d $O/p${p%%:*} -o pmc -- python3 tools/profile_kernel.py $CFG $REPS 0 $BATCH > $O/p${p%%:*}.log 2>&1
  done
  python3 tools/pmc_summary.py $O > /dev/null
  echo done $name
done
