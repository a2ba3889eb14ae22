#!/bin/bash
# GPU call (dev tool): round-end suite of the current tree, then per-config kernel times.
set -u
bash tools/gpu_round_end.sh ${1:-r02i} || exit 1
RTAMD_LIB=raytracingengine_amd/librtamd.so timeout -k 10 200 python tools/ab_time.py c5 c1 c2 c3 \
    2>&1 | grep -v amdgpu.ids > gpurun_out/${1:-r02i}/times.txt || exit 1
cat gpurun_out/${1:-r02i}/times.txt
