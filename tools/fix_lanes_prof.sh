#!/bin/bash
# Dev tool (GPU box): rocprofv3 kernel stats of the C2 32-frame launch pair (packet kernel + fix-up)
# for the in-tree library and each tools/variants/NAME.so given.   bash tools/fix_lanes_prof.sh OUT l64 l32
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in tree "$@"; do
  if [ "$v" = tree ]; then unset RTAMD_LIB; else export RTAMD_LIB="tools/variants/$v.so"; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/$v" -o run -- python3 tools/profile_kernel.py c2 10 0 32 > "$OUT/$v.log" 2>&1
  echo "== $v $(grep -h fixup "$OUT/$v"/run_kernel_stats.csv | cut -d, -f2,4,6,7)"
done
