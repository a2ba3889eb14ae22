#!/bin/bash
# Dev tool: rocprofv3 counter passes (one --pmc group per run) over tools/profile_kernel.py.
# usage: tools/pmc_passes.sh <outdir> <config> [reps] [flags]
set -e
OUT=$1; CFG=$2; REPS=${3:-10}; FLAGS=${4:-0}; BATCH=${5:-1}
mkdir -p $OUT
export TMPDIR=/tmp
P=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH" \
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  P=$((P+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$P -o pmc -- python3 tools/profile_kernel.py $CFG $REPS $FLAGS $BATCH > $OUT/p$P.log 2>&1
done
python3 tools/pmc_summary.py $OUT
