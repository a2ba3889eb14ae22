#!/bin/bash
# GPU call (dev tool, round 6): counter passes (tools/pmc_passes.sh) and kernel traces of glass
# (breadth-first level kernels) and mirror (box chain kernel, spheres), for
# tools/valu_summary.py's issue fraction and lane activity.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/valu_gm
mkdir -p $OUT
for cfg in glass mirror; do
  echo "== $cfg"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$cfg -o kt -- \
    python3 tools/profile_kernel.py $cfg 10 > $OUT/kt_$cfg.log 2>&1 || { tail $OUT/kt_$cfg.log; exit 1; }
  timeout -k 10 600 bash tools/pmc_passes.sh $OUT/pmc_$cfg $cfg 10 > $OUT/pmc_$cfg.log 2>&1 || { tail $OUT/pmc_$cfg.log; exit 1; }
done
echo done
