#!/bin/bash
# Dev tool: registers / scratch / occupancy (and the ISA census) of ONE packet-kernel variant,
# compiled alone from rt_packet.hip (RT_PACKET_PROBE) — seconds instead of the whole file.
#   bash tools/isa/probe.sh "1,0,false,false,1" [extra hipcc flags...]
set -eu
V=$1; shift
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=/tmp/probe_$$.s
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off \
    -mllvm -amdgpu-sched-strategy=max-ilp --cuda-device-only -S -o $OUT \
    "-DRT_PACKET_PROBE=$V" "$@" -I$ROOT/include $ROOT/raytracingengine_amd/csrc/rt_packet.hip \
    -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "VGPRs:|AGPRs:|ScratchSize|Occupancy|SGPRs:" | sed 's/.*remark: //'
python3 $ROOT/tools/isa/census.py $OUT packet_direct_kernel
rm -f $OUT
