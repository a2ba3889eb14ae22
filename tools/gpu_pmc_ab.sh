#!/bin/bash
# GPU call (dev tool): per-wave instruction counts (one rocprofv3 --pmc pass per library build,
# config and flag set) of the in-tree build vs tools/variants/*.so.
#   bash tools/gpu_pmc_ab.sh TAG "c1 c2" [flags-for-an-extra-in-tree-pass]
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
CFGS=${2:-c2}
mkdir -p $OUT
run() {  # lib tag cfg flags
  RTAMD_LIB=$1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH \
      SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 \
      --output-format csv -d $OUT/${2}_$3 -o pmc -- python3 tools/profile_kernel.py $3 5 $4 \
      > $OUT/${2}_$3.log 2>&1 || { echo "pmc pass $2 $3 failed"; tail -5 $OUT/${2}_$3.log; exit 1; }
}
for cfg in $CFGS; do
  run raytracingengine_amd/librtamd.so new $cfg 0
  [ -n "${3:-}" ] && run raytracingengine_amd/librtamd.so newflag$3 $cfg $3
  for lib in $(ls tools/variants/*.so 2>/dev/null); do run $lib $(basename $lib .so) $cfg 0; done
done
python3 tools/pmc_ab_summary.py $OUT | tee $OUT/summary.txt
