#!/bin/bash
# GPU call (dev tool): interleaved A/B kernel times (tools/gpu_ab.sh) then the in-tree build's
# counter passes for the given configs (tools/pmc_passes.sh).
#   bash tools/gpu_ab_pmc.sh TAG "ab configs" "pmc configs" [pytest -k expr]
set -u
bash tools/gpu_ab.sh $1 "$2" "${4:-}" || exit 1
export TMPDIR=/tmp
for cfg in $3; do
  bash tools/pmc_passes.sh gpurun_out/$1/pmc_$cfg $cfg 10 > gpurun_out/$1/pmc_$cfg.log 2>&1 \
      || { tail -20 gpurun_out/$1/pmc_$cfg.log; exit 1; }
done
