#!/bin/bash
# Dev tool: VGPRs / scratch / occupancy of every kernel of one HIP source of a tree (default:
# this repo), full kernel names.   bash tools/isa/resources.sh rt_trace_lean.hip [ROOT] [flags]
set -eu
SRC=$1; ROOT=${2:-$(cd "$(dirname "$0")/../.." && pwd)}; shift; shift || true
EXTRA=""
[ "$SRC" = "rt_packet.hip" ] && EXTRA="-mllvm -amdgpu-sched-strategy=max-ilp"
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off -fPIC $EXTRA "$@" \
    -I$ROOT/include -c -o /dev/null $ROOT/raytracingengine_amd/csrc/$SRC \
    -Rpass-analysis=kernel-resource-usage 2>&1 | \
  awk '/Function Name:/{n=$(NF-1)} /VGPRs: /{v=$(NF-1)} /ScratchSize/{s=$(NF-1)} /Occupancy/{print n, "VGPR="v, "scratch="s, "occ="$(NF-1)}'
