#!/bin/bash
# Dev tool: per-wave counters variant of the packet kernel (timestamps in each 8x8 tile's first
# pixel as tools/stamps_patch.txt, counters in its second pixel: exact-march iterations,
# undecided shadow rays, shadow candidate spheres summed over lanes).  -> tools/stampvariants/wavestats.so
set -e
python3 tools/build_stamps.py wavestats \
 '// computeTransmittance (Scene.h:35-77) over the candidate spheres of the shadow packet.' \
 '__shared__ unsigned pk_dbg[16];
// computeTransmittance (Scene.h:35-77) over the candidate spheres of the shadow packet.' \
 '        PkHit h;
        if (!closest_masked' \
 '        PkHit h;
        atomicAdd(&pk_dbg[(threadIdx.x >> 6) * 4 + 0], 1u);
        if (!closest_masked' \
 '    const int occ = pk_occlusion<MAXC, FEAT>(S, M, nchunks, so, L, dist - bias, bias);' \
 '    const int occ = pk_occlusion<MAXC, FEAT>(S, M, nchunks, so, L, dist - bias, bias);
    if (occ == 2) atomicAdd(&pk_dbg[(threadIdx.x >> 6) * 4 + 1], 1u);
    { unsigned pc = 0; for (int c = 0; c < MAXC; ++c) pc += __builtin_popcountll(M.m[c]);
      atomicAdd(&pk_dbg[(threadIdx.x >> 6) * 4 + 2], pc); }' \
 '    for (int i = tid; i < kLtStride * nl; i += kWgThreads) s_lt[i] = P.lt[i];
    __syncthreads();' \
 '    for (int i = tid; i < kLtStride * nl; i += kWgThreads) s_lt[i] = P.lt[i];
    if (tid < 16) pk_dbg[tid] = 0u;
    __syncthreads();' \
 '            if (lane == 0) {
                const uint64_t stamp1' \
 '            if (lane == 1) {
                P.out64[3 * o + 0] = pk_dbg[wave * 4 + 0];
                P.out64[3 * o + 1] = pk_dbg[wave * 4 + 1];
                P.out64[3 * o + 2] = pk_dbg[wave * 4 + 2];
            }
            if (lane == 0) {
                const uint64_t stamp1'
mkdir -p tools/stampvariants
mv tools/variants/wavestats.so tools/stampvariants/
