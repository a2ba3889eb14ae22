#!/bin/bash
# Dev tool (GPU box): packet_fixup_kernel duration (tools/fixup_scaling.py under a kernel trace)
# for the in-tree library and every tools/variants/*.so.   bash tools/fixup_ab.sh OUT
set -u
export TMPDIR=/tmp
OUT=$1
mkdir -p $OUT
for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
  name=$(basename $lib .so)
  RTAMD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o fx -- \
    python3 tools/fixup_scaling.py > $OUT/$name.log 2>&1 || { echo "fail $name"; tail -3 $OUT/$name.log; exit 1; }
  echo "$name $(python3 tools/fixup_scaling.py --summarize $OUT/$name)"
done
