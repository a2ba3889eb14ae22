#!/bin/bash
# Dev tool: per-wave counters variant of the packet kernel -> tools/diag/wavestats.so.
# Each 8x8 tile's first pixel holds the wave's s_memrealtime stamps at entry / exit (int64 bits
# of the first two doubles); its second pixel: occlusion-classification loop iterations,
# undecided shadow lanes, exact-march candidate iterations; its third pixel: camera-ray
# candidate iterations.  Loop iterations are counted per WAVE (what costs issue time), not per
# lane.  Time with tools/wave_stats.py; the images of this build are deliberately wrong.
set -e
python3 tools/build_variant.py wavestats rt_packet.hip \
 'struct PacketScene {' \
 '__shared__ unsigned pk_dbg[64];
#define PK_DBG_WAVE(k) do { if (__lane_id() == __builtin_ctzll(__ballot(1))) atomicAdd(&pk_dbg[(threadIdx.x >> 6) * 4 + (k)], 1u); } while (0)
struct PacketScene {' \
 '                const double* q = S.pre + 4 * i;' \
 '                PK_DBG_WAVE(3);
                const double* q = S.pre + 4 * i;' \
 '            const double* s = S.sph + kSphStride * i;
            const d3 oc = o - mk(s[0], s[1], s[2]);
            const double b = 2.0 * dot(oc, d);
            const double cc = dot(oc, oc) - s[3];
            const double disc = b * b - four_a * cc;
            if (regular)' \
 '            PK_DBG_WAVE(2);
            const double* s = S.sph + kSphStride * i;
            const d3 oc = o - mk(s[0], s[1], s[2]);
            const double b = 2.0 * dot(oc, d);
            const double cc = dot(oc, oc) - s[3];
            const double disc = b * b - four_a * cc;
            if (regular)' \
 '            const double disc = b * b - four_a * cc;
            if (disc < 0.0) continue;  // miss' \
 '            const double disc = b * b - four_a * cc;
            PK_DBG_WAVE(0);
            if (disc < 0.0) continue;  // miss' \
 '    const bool undecided = need && occ == 2;' \
 '    const bool undecided = need && occ == 2;
    if (undecided) atomicAdd(&pk_dbg[(threadIdx.x >> 6) * 4 + 1], 1u);' \
 '    __syncthreads();

    PacketScene S;' \
 '    if (tid < 64) pk_dbg[tid] = 0u;
    __syncthreads();
    const uint64_t dbg_t0 = __builtin_amdgcn_s_memrealtime();

    PacketScene S;' \
 '    if constexpr (COUNT) {
        uint32_t t = cnt.trace' \
 '    {
        const uint64_t dbg_t1 = __builtin_amdgcn_s_memrealtime();
        const size_t o = static_cast<size_t>(yl) * P.width + x;
        if (valid && P.out64 && lane == 0) {
            P.out64[3 * o + 0] = __longlong_as_double(static_cast<long long>(dbg_t0));
            P.out64[3 * o + 1] = __longlong_as_double(static_cast<long long>(dbg_t1));
        }
        if (valid && P.out64 && lane == 1) {
            P.out64[3 * o + 0] = pk_dbg[wave * 4 + 0];
            P.out64[3 * o + 1] = pk_dbg[wave * 4 + 1];
            P.out64[3 * o + 2] = pk_dbg[wave * 4 + 2];
        }
        if (valid && P.out64 && lane == 2) P.out64[3 * o + 0] = pk_dbg[wave * 4 + 3];
    }
    if constexpr (COUNT) {
        uint32_t t = cnt.trace' \
 "$@"
mkdir -p tools/diag
mv tools/variants/wavestats.so tools/diag/
