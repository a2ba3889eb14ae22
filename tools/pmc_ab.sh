#!/bin/bash
# Dev tool (GPU box): VALU / SALU instructions per wave of the packet kernel for several library
# builds and configs (one rocprofv3 counter pass each).  Usage: bash tools/pmc_ab.sh c2 c4 c5
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmcab
mkdir -p $OUT
for lib in raytracingengine_amd/librtamd.so $(ls tools/variants/*.so 2>/dev/null); do
  tag=$(basename $lib .so)
  for cfg in "$@"; do
    RTAMD_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU \
      --output-format csv -d $OUT/${tag}_$cfg -o pmc -- python3 tools/profile_kernel.py $cfg 5 > $OUT/${tag}_$cfg.log 2>&1
  done
done
python3 tools/pmc_ab_summary.py $OUT
