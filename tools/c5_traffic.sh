#!/bin/bash
# GPU call (dev tool): HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, separate passes) of the C5 launch
# for the in-tree build and every tools/variants/*.so.   bash tools/c5_traffic.sh OUTDIR
set -e
export TMPDIR=/tmp
OUT=$1
for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
  name=$(basename $lib .so)
  O=$OUT/$name
  mkdir -p $O
  RTAMD_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p1 -o pmc -- python3 tools/profile_kernel.py c5 6 > $O/p1.log 2>&1
  RTAMD_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p2 -o pmc -- python3 tools/profile_kernel.py c5 6 > $O/p2.log 2>&1
  python3 tools/pmc_summary.py $O > /dev/null
  echo done $name
done
