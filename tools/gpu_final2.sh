#!/bin/bash
# GPU call (dev tool): round-end suite of the current tree, then C1 / mirror kernel times.
set -u
bash tools/gpu_round_end.sh ${1:-r02h} || exit 1
RTAMD_LIB=raytracingengine_amd/librtamd.so timeout -k 10 200 python tools/ab_time.py c1 mirror c2 \
    2>&1 | grep -v amdgpu.ids > gpurun_out/${1:-r02h}/times.txt || exit 1
cat gpurun_out/${1:-r02h}/times.txt
