#!/bin/bash
# GPU call (dev tool): rocprofv3 PC sampling (beta) of one config's frames.
#   bash tools/gpu_pcs.sh TAG cfg [method] [unit] [interval]
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; CFG=${2:-c2}; M=${3:-host_trap}; U=${4:-time}; I=${5:-1}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/list_avail.txt 2>&1 || true
grep -i -A12 "pc.sampl" $OUT/list_avail.txt | head -60
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M \
    --pc-sampling-unit $U --pc-sampling-interval $I --output-format csv -d $OUT/pcs -o pcs \
    -- python3 tools/pcs_driver.py $CFG 1.0 > $OUT/pcs.log 2>&1
echo "pcs rc=$?"; tail -5 $OUT/pcs.log; find $OUT/pcs -type f | head
