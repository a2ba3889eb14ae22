#!/bin/bash
# Dev tool (GPU box): per-wave instruction counts of one config's launch under several
# environment settings of the in-tree library (one rocprofv3 counter pass each).
#   bash tools/pmc_env.sh c2 32 "RTAMD_PK_AXIS=1" "RTAMD_PK_AXIS=0"
set -e
export TMPDIR=/tmp
cfg=$1; batch=$2; shift 2
OUT=gpurun_out/pmcenv_$cfg
rm -rf $OUT; mkdir -p $OUT
for e in "$@"; do
  tag=$(echo "$e" | tr ' =' '__')
  env $e timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH \
    --output-format csv -d $OUT/$tag -o pmc -- python3 tools/profile_kernel.py $cfg 5 0 $batch > $OUT/$tag.log 2>&1
done
python3 tools/pmc_ab_summary.py $OUT
