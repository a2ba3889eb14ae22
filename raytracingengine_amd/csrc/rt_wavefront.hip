// rt_wavefront.hip — breadth-first ("wavefront") TraceRay for scenes with secondary rays.
//
// The reference recursion (Scene.h:131-198) spawns, per hit, a refraction ray (transparent
// materials, Scene.h:181-187) and a reflection ray (Scene.h:189-195), so every pixel sample is a
// binary tree of TraceRay calls.  Walking that tree per thread (rt_trace.hip, trace_tree) keeps
// a 16-frame stack in scratch and leaves most lanes of a wave idle while the deepest tree of the
// wave finishes.  Here the tree is processed level by level instead:
//
//   level kernel k   every ray of depth k is one thread: shade() (closest hit, directLightning
//                    with its shadow rays — the same device code as the per-pixel kernels), the
//                    node record (local value, refraction / reflection weights) is written, and
//                    the child rays are appended to level k+1 with one atomic per wave;
//   fold kernel k    deepest level first, value = (local + refraction_child·fw) +
//                    reflection_child·rw — the reference's accumulation order (Scene.h:176-195);
//   final kernel     the roots' fold, the AA average of each pixel's root values, stored like
//                    GeneratePixelAt.
//
// Every ray is computed by the same instructions as in the per-pixel kernels and every node is
// folded in the reference's order, so the image is bit-identical to them.  Node/ray records live
// in one HBM arena of fixed capacity; a sample whose tree does not fit is flagged and its pixel
// is re-rendered by the per-pixel kernel (P.redo) in the same stream, so capacity never changes
// the result.  No host synchronisation: the ray count of each level lives in device memory and
// the level kernels are persistent grids that loop over it.
#include <algorithm>
#include <cstdlib>

#include "rt_trace_common.hpp"
#include "rt_wavefront.hpp"

#pragma clang fp contract(off)

namespace rtamd {
#ifdef RT_LEAN_GENERIC
// rt_wavefront_lean.hip: the same level / fold / final kernels without the triangle / BVH and
// area-light code (rt_trace_common.hpp), for scenes that have neither (rtamd::lean).
namespace lean {
#endif

namespace {

constexpr int kWfThreads = 256;
#ifndef RT_WF_WG_ALLOC
#define RT_WF_WG_ALLOC 1
#endif

__device__ __forceinline__ uint32_t lane_prefix(uint64_t mask) {  // set bits below this lane
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mask), 0u));
}

// rays of level `level`: [base, base + n) in node ids, clamped to the arena
__device__ __forceinline__ void level_range(const WfArena& A, int level, uint32_t& base,
                                            uint32_t& n) {
    if (level == 0) {
        base = 0;
        n = A.n0;
        return;
    }
    base = A.ctl->base[level];
    const uint32_t want = A.ctl->count[level];
    n = base >= A.cap ? 0u : min(want, A.cap - base);
}

// Level 0's lanes take the camera rays in 8×8 pixel tiles (row-major over the tiles) when both
// sides are multiples of 8, so each wave — and, through the wave-ordered child append, each
// wave of the deeper levels — holds one coherent tile.  Node ids stay row-major (id = root).
__device__ __forceinline__ uint32_t wf_tile_order(const TraceParams& P, uint32_t i, uint32_t aa) {
    if ((P.width & 7u) != 0 || (P.rows & 7u) != 0) return i;
    const uint32_t t = i / aa, s = i - t * aa;
    const uint32_t tile = t >> 6, w = t & 63u, tiles_x = P.width >> 3;
    const uint32_t x = (tile % tiles_x) * 8u + (w & 7u), yl = (tile / tiles_x) * 8u + (w >> 3);
    return (yl * P.width + x) * aa + s;
}

// level kernels: 2 waves/SIMD, 3 in the lean build (213 → 168 VGPRs: glass 1.58 → 1.54 ms).
// RT_WF_SAVE=1 RT_WF_LEVEL_WAVES=4 (shade()'s hit point / normal / direction parked in LDS across
// the light loop: 128 VGPRs at 4 waves/SIMD) renders glass 1.2 % faster (964 vs 975 µs) but
// spills 144-160 B/lane, which costs 1.08 GB of HBM traffic per 1080p frame: 215 B per ray
// against 127 B at 3 waves (profiles/r04_glass_traffic.json, r04_ab_glass_level_save.txt).
#ifndef RT_WF_SAVE
#define RT_WF_SAVE 0
#endif
#ifdef RT_LEAN_GENERIC
#ifndef RT_WF_LEVEL_WAVES
#define RT_WF_LEVEL_WAVES 3
#endif
constexpr int kWfLevelWaves = RT_WF_LEVEL_WAVES;
#else
constexpr int kWfLevelWaves = 2;
#endif
// Deferred direct lighting (the shadow stage, RTAMD_WF_DEFER, tree scenes): the level kernels
// find each ray's closest hit and spawn its children, but leave directLightning — the light loop
// and its computeTransmittance marches, 40 % of a glass frame spent at 57 % lane activity inside
// the level kernels (profiles/r04_ab_glass_marches.txt, r04_glass_level_valu.json) — to
// wf_direct_kernel, which shades every queued hit of every level in one launch with no other
// work in its lanes.  Both run shade_hit (rt_trace_common.hpp) on the same hit, so the node
// values are the same bits.
constexpr uint32_t kDqIdxBits = 26;  // hit code: primitive index | kind << 26 | level << 28
__device__ __forceinline__ uint32_t dq_code(const Hit& h, int level) {
    return static_cast<uint32_t>(h.idx) | (static_cast<uint32_t>(h.kind) << kDqIdxBits) |
           (static_cast<uint32_t>(level) << 28);
}

#ifndef RT_WF_DEFER_LEVEL_WAVES
#define RT_WF_DEFER_LEVEL_WAVES 4
#endif
template <bool TREE, bool LDS, bool DEFER>
__global__ __launch_bounds__(kWfThreads, DEFER ? RT_WF_DEFER_LEVEL_WAVES : kWfLevelWaves) void
wf_level_kernel(TraceParams P, WfArena A, int level) {
    extern __shared__ double smem[];
    const SceneView S = stage_scene<LDS>(P, smem, threadIdx.x, kWfThreads);
#if RT_WF_SAVE
    __shared__ double s_save[9 * kWfThreads];  // shade()'s parked hit point, normal, direction
    double* const save = DEFER ? nullptr : s_save + threadIdx.x;
#else
    double* const save = nullptr;
#endif
    uint32_t base, n;
    level_range(A, level, base, n);
    const uint32_t next = base + n;  // first node id of level + 1
    if (blockIdx.x == 0 && threadIdx.x == 0) A.ctl->base[level + 1] = next;
    const int lane = threadIdx.x & 63;
    const d3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
    const uint32_t aa = static_cast<uint32_t>(P.aa);
    // the last shading level (depth maxRecursion − 1): its children are TraceRay calls at depth
    // maxRecursion, which return the sky (Scene.h:132-134), so each node is folded right here —
    // no child slots, no ray records, no level and no fold launch of their own
    const bool leaves = level + 1 >= P.max_rec;
    Counts cnt{0u, 0u};
#if RT_WF_WG_ALLOC
    // Child slots of level + 1 (and deferred-direct records) are reserved with ONE device atomic
    // per workgroup and iteration (the four waves' counts summed in LDS): a single counter hit by
    // every wave of the chip serialises at memory, one atomic per wave cost the deep levels most
    // of their time.
    __shared__ uint32_t s_wtot[kWfThreads / 64], s_wbase;
    __shared__ uint32_t s_dtot[kWfThreads / 64], s_dbase;
    const int wave = threadIdx.x >> 6;
    // workgroup-uniform grid-stride loop (the barriers below): every wave of the workgroup runs
    // every iteration, lanes past n idle (ballots below)
    for (uint32_t b0 = blockIdx.x * kWfThreads; b0 < n; b0 += gridDim.x * kWfThreads) {
        const uint32_t i = b0 + threadIdx.x;
#else
    static_assert(!DEFER, "the deferred direct queue is allocated per workgroup");
    // wave-uniform grid-stride loop: all 64 lanes run every iteration (ballots below)
    for (uint32_t i0 = blockIdx.x * kWfThreads + (threadIdx.x & ~63u); i0 < n;
         i0 += gridDim.x * kWfThreads) {
        const uint32_t i = i0 + lane;
#endif
        const bool active = i < n;
        const uint32_t id = base + (active ? (level == 0 ? wf_tile_order(P, i, aa) : i) : 0u);
        uint32_t root;
        d3 o, d;
        if (level == 0) {
            root = id;
            const uint32_t pl = root / aa, s = root % aa;
            const uint32_t x = pl % P.width, y = image_row(P, pl / P.width);
            o = cam;
            d = camera_dir(P, cam, x, y, static_cast<uint64_t>(y) * P.width + x,
                           static_cast<int>(s));
        } else {
            const size_t r = id - A.n0;
            root = A.root[r];
            o = mk(A.ray[r], A.ray[A.cap_r + r], A.ray[2 * A.cap_r + r]);
            d = mk(A.ray[3 * A.cap_r + r], A.ray[4 * A.cap_r + r], A.ray[5 * A.cap_r + r]);
        }
        const uint32_t pl = root / aa, sample = root % aa;
        const uint64_t pix =
            static_cast<uint64_t>(image_row(P, pl / P.width)) * P.width + pl % P.width;
        // this root's overflow flag starts clear (level 0 visits every root once, before any
        // level can flag it: no memset of the whole array on the stream)
        if (level == 0 && active) A.redo[root] = 0;
        Node nd;
        nd.hit = false;
        nd.refl = false;
        nd.refr = false;
        nd.fw = 0.0;
        nd.rw = 0.0;
        bool defer = false;  // this node's local term is left to wf_direct_kernel
        Hit h;
        h.t = 0.0;
        h.kind = 0;
        h.idx = 0;
        if (active) {
            if (level >= P.max_rec) {
                nd.value = sky(d);  // TraceRay at depth >= maxRecursion
            } else if constexpr (DEFER) {
                if (!closest(S, o, d, h)) {
                    nd.value = sky(d);
                } else {
                    nd = shade_hit<TREE, false, false>(S, P, o, d, h, pix, sample, level, cnt);
                    // fin = local·(1 − tr) only when tr < 1 (Scene.h:175-179): else no local term
                    defer = sclamp(material_of(S, h)[5], 0.0, 1.0) < 1.0;
                }
            } else {
                nd = shade<TREE, false>(S, P, o, d, pix, sample, level, cnt, save, kWfThreads);
            }
        }
        const bool want_f = active && TREE && nd.hit && nd.refr;
        const bool want_r = active && nd.hit && nd.refl;
        uint32_t dslot = 0;  // this lane's deferred record
        if constexpr (DEFER) {
            // one atomic per workgroup for the deferred records of its four waves, in wave order
            const uint64_t bd = __ballot(defer);
            if (lane == 0) s_dtot[wave] = __builtin_popcountll(bd);
            __syncthreads();
            if (threadIdx.x == 0) {
                const uint32_t sum = s_dtot[0] + s_dtot[1] + s_dtot[2] + s_dtot[3];
                s_dbase = sum ? atomicAdd(leaves ? &A.ctl->dleaf : &A.ctl->dcount, sum) : 0u;
            }
            __syncthreads();
            dslot = s_dbase + lane_prefix(bd);
            for (int w = 0; w < wave; ++w) dslot += s_dtot[w];
            __syncthreads();  // s_dtot / s_dbase are rewritten by the next iteration
            if (leaves) dslot = A.cap - 1u - dslot;  // the last level's records from the back
            if (defer) {  // at most one record per node: the queue holds cap records
                A.dq_id[dslot] = id;
                A.dq_code[dslot] = dq_code(h, level);
                A.dq_t[dslot] = h.t;
            }
        }
        if (leaves) {  // uniform: children at depth maxRecursion are the sky (Scene.h:132-134)
            if (active && !defer) {
                // the fold of this node with those children, in the reference's order
                // (Scene.h:176-195): (local + refraction·fw) + reflection·rw (a deferred node is
                // folded by wf_direct_kernel once its local term is known)
                d3 v = nd.value;
                if (want_f) v = v + sky(nd.fd) * nd.fw;
                if (want_r) v = v + sky(nd.rd) * nd.rw;
                A.val[id] = v.x;
                A.val[A.cap + id] = v.y;
                A.val[2 * A.cap + id] = v.z;
            }
            if (active) {
                A.child[id] = -1;
                A.child[A.cap + id] = -1;
            }
            continue;
        }
        const uint64_t bf = __ballot(want_f), br = __ballot(want_r);
        const uint32_t total = __builtin_popcountll(bf) + __builtin_popcountll(br);
        uint32_t wbase = 0;
#if RT_WF_WG_ALLOC
        // one atomic per workgroup for all children of its four waves, in wave order
        if (lane == 0) s_wtot[wave] = total;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t sum = s_wtot[0] + s_wtot[1] + s_wtot[2] + s_wtot[3];
            s_wbase = sum ? atomicAdd(&A.ctl->count[level + 1], sum) : 0u;
        }
        __syncthreads();
        wbase = s_wbase;
        for (int w = 0; w < wave; ++w) wbase += s_wtot[w];
        __syncthreads();  // s_wtot / s_wbase are rewritten by the next iteration
#else
        // one atomic per wave for all children of the wave
        if (total) {
            if (lane == 0) wbase = atomicAdd(&A.ctl->count[level + 1], total);
            wbase = __shfl(wbase, 0, 64);
        }
#endif
        int32_t cf = -1, cr = -1;
        bool lost = false;
        if (want_f) {
            const uint32_t cid = next + wbase + lane_prefix(bf);
            if (cid < A.cap) {
                const size_t r = cid - A.n0;
                A.ray[r] = nd.fo.x;
                A.ray[A.cap_r + r] = nd.fo.y;
                A.ray[2 * A.cap_r + r] = nd.fo.z;
                A.ray[3 * A.cap_r + r] = nd.fd.x;
                A.ray[4 * A.cap_r + r] = nd.fd.y;
                A.ray[5 * A.cap_r + r] = nd.fd.z;
                A.root[r] = root;
                cf = static_cast<int32_t>(cid);
            } else {
                lost = true;
            }
        }
        if (want_r) {
            const uint32_t cid =
                next + wbase + __builtin_popcountll(bf) + lane_prefix(br);
            if (cid < A.cap) {
                const size_t r = cid - A.n0;
                A.ray[r] = nd.ro.x;
                A.ray[A.cap_r + r] = nd.ro.y;
                A.ray[2 * A.cap_r + r] = nd.ro.z;
                A.ray[3 * A.cap_r + r] = nd.rd.x;
                A.ray[4 * A.cap_r + r] = nd.rd.y;
                A.ray[5 * A.cap_r + r] = nd.rd.z;
                A.root[r] = root;
                cr = static_cast<int32_t>(cid);
            } else {
                lost = true;
            }
        }
        if (lost) {  // the tree of this sample does not fit: per-pixel fix-up
            A.redo[root] = 1;
            A.ctl->lost = 1u;
        }
        if (active) {
            if (!defer) {  // a deferred node's value is written by wf_direct_kernel
                A.val[id] = nd.value.x;
                A.val[A.cap + id] = nd.value.y;
                A.val[2 * A.cap + id] = nd.value.z;
            }
            A.fw[id] = nd.fw;
            A.rw[id] = nd.rw;
            A.child[id] = cf;
            A.child[A.cap + id] = cr;
        }
    }
}

// The deferred direct lighting of every level's queued hits: shade_hit with directLightning
// (the same function and values as a level kernel's own shade), the node's value written, and at
// the last shading level its fold with the sky children (as the level kernel does for the nodes
// it shades itself).  Persistent grid over the queue; the records of a workgroup are consecutive
// nodes of one level, so a wave's hits stay as coherent as the level kernel's were.
#ifndef RT_WF_DIRECT_WAVES
#define RT_WF_DIRECT_WAVES 4
#endif
template <bool TREE, bool LDS, bool LEAF>
__global__ __launch_bounds__(kWfThreads, RT_WF_DIRECT_WAVES) void wf_direct_kernel(TraceParams P,
                                                                                   WfArena A) {
    extern __shared__ double smem[];
    const SceneView S = stage_scene<LDS>(P, smem, threadIdx.x, kWfThreads);
    // the inner levels' records [0, dcount), the last level's [cap − dleaf, cap)
    const uint32_t n = min(LEAF ? A.ctl->dleaf : A.ctl->dcount, A.cap);
    const uint32_t q0 = LEAF ? A.cap - n : 0u;
    const d3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
    const uint32_t aa = static_cast<uint32_t>(P.aa);
    const double bias = P.bias;
    const int lane = threadIdx.x & 63;
    Counts cnt{0u, 0u};
    // wave-uniform grid-stride loop: every lane takes part in the shadow packets' ballots
    for (uint32_t i0 = blockIdx.x * kWfThreads + (threadIdx.x & ~63u); i0 < n;
         i0 += gridDim.x * kWfThreads) {
        const uint32_t qi = i0 + lane;
        const bool active = qi < n;
        const uint32_t q = q0 + (active ? qi : 0u);
        uint32_t id = 0;
        Hit h;
        h.t = 0.0;
        h.kind = 1;
        h.idx = 0;
        d3 o = mk(0.0, 0.0, 0.0), d = mk(0.0, 0.0, 1.0);
        uint64_t pix = 0;
        uint32_t sample = 0;
        int level = 0;
        if (active) {
            id = A.dq_id[q];
            const uint32_t code = A.dq_code[q];
            h.t = A.dq_t[q];
            h.idx = static_cast<int>(code & ((1u << kDqIdxBits) - 1u));
            h.kind = static_cast<int>((code >> kDqIdxBits) & 3u);
            level = static_cast<int>(code >> 28);
            uint32_t root;
            if (id < A.n0) {  // a camera ray: the level kernel's own getRay
                root = id;
                const uint32_t pl = root / aa, s = root % aa;
                const uint32_t x = pl % P.width, y = image_row(P, pl / P.width);
                o = cam;
                d = camera_dir(P, cam, x, y, static_cast<uint64_t>(y) * P.width + x,
                               static_cast<int>(s));
            } else {
                const size_t r = id - A.n0;
                root = A.root[r];
                o = mk(A.ray[r], A.ray[A.cap_r + r], A.ray[2 * A.cap_r + r]);
                d = mk(A.ray[3 * A.cap_r + r], A.ray[4 * A.cap_r + r], A.ray[5 * A.cap_r + r]);
            }
            const uint32_t pl = root / aa;
            sample = root % aa;
            pix = static_cast<uint64_t>(image_row(P, pl / P.width)) * P.width + pl % P.width;
        }
        // shade_hit's shading inputs (Scene.h:147-154) and directLightning (Scene.h:79-129)
        // with one shadow packet per light for the wave
        const d3 hp = o + d * h.t;  // Rayon::pointAtDistance
        d3 nn = mk(0.0, 1.0, 0.0), view = mk(0.0, 0.0, 0.0);
        const double* m = S.sph_mat;
        if (active) {
            const d3 gn = normal_of(S, h, hp);
            m = material_of(S, h);
            const d3 inc = unit(d);
            const bool front = dot(gn, inc) < 0.0;
            view = -inc;
            nn = unit(front ? gn : -gn);  // directLightning's own normalize (Scene.h:81)
        }
        d3 diff = mk(0.0, 0.0, 0.0), spec = mk(0.0, 0.0, 0.0);
        for (int l = 0; l < S.nl; ++l) {
            const double* lt = S.lt + kLtStride * l;
            light_term_wave<false>(S, active, hp, nn, view, m, mk(lt[0], lt[1], lt[2]),
                                   mk(lt[3], lt[4], lt[5]), bias, diff, spec, cnt);
        }
#ifndef RT_LEAN_GENERIC  // the build-defined area light: per-lane sample points, full marches
        if (active && P.al_samples > 0) {
            const uint32_t stream = 0x10000u + (sample << 6) + static_cast<uint32_t>(level);
            const double k = static_cast<double>(P.al_k);
            const d3 corner = mk(P.al_corner[0], P.al_corner[1], P.al_corner[2]);
            const d3 eu = mk(P.al_u[0], P.al_u[1], P.al_u[2]);
            const d3 ev = mk(P.al_v[0], P.al_v[1], P.al_v[2]);
            const d3 E = mk(P.al_E[0], P.al_E[1], P.al_E[2]);
            for (int s = 0; s < P.al_samples; ++s) {
                const double r1 = u01(P.seed, pix, stream, 2u * static_cast<uint32_t>(s));
                const double r2 = u01(P.seed, pix, stream, 2u * static_cast<uint32_t>(s) + 1u);
                const double fu = (static_cast<double>(s % P.al_k) + r1) / k;
                const double fv = (static_cast<double>(s / P.al_k) + r2) / k;
                const d3 lp = (corner + eu * fu) + ev * fv;
                light_term<false, false>(S, hp, nn, view, m, lp, E, bias, diff, spec, cnt);
            }
        }
#endif
        if (!active) continue;
        const d3 local = hmul(mk(m[0], m[1], m[2]), diff) + spec * m[4];
        const double tr = sclamp(m[5], 0.0, 1.0);
        d3 v = mk(0.0, 0.0, 0.0);
        if (tr < 1.0) v = v + local * (1.0 - tr);  // Scene.h:175-179 (fin)
        if constexpr (LEAF) {
            // the last shading level: fold with the sky children (the child rays of the same hit,
            // shade_hit without directLightning)
            const Node nd = shade_hit<TREE, false, false, true>(S, P, o, d, h, pix, sample, level,
                                                                cnt);
            if (TREE && nd.refr) v = v + sky(nd.fd) * nd.fw;
            if (nd.refl) v = v + sky(nd.rd) * nd.rw;
        }
        A.val[id] = v.x;
        A.val[A.cap + id] = v.y;
        A.val[2 * A.cap + id] = v.z;
    }
}

// value = (local + refraction·fw) + reflection·rw, deepest level first (Scene.h:176-195)
__global__ __launch_bounds__(kWfThreads) void wf_fold_kernel(WfArena A, int level) {
    uint32_t base, n;
    level_range(A, level, base, n);
    for (uint32_t i = blockIdx.x * kWfThreads + threadIdx.x; i < n; i += gridDim.x * kWfThreads) {
        const uint32_t id = base + i;
        const int32_t cf = A.child[id], cr = A.child[A.cap + id];
        if (cf < 0 && cr < 0) continue;
        d3 v = mk(A.val[id], A.val[A.cap + id], A.val[2 * A.cap + id]);
        if (cf >= 0) v = v + mk(A.val[cf], A.val[A.cap + cf], A.val[2 * A.cap + cf]) * A.fw[id];
        if (cr >= 0) v = v + mk(A.val[cr], A.val[A.cap + cr], A.val[2 * A.cap + cr]) * A.rw[id];
        A.val[id] = v.x;
        A.val[A.cap + id] = v.y;
        A.val[2 * A.cap + id] = v.z;
    }
}

// GeneratePixelAt (Scene.h:283-304): each root folded with its children, accumulated / samples,
// then the outputs
__global__ __launch_bounds__(kWfThreads) void wf_final_kernel(TraceParams P, WfArena A) {
    const size_t npx = static_cast<size_t>(P.rows) * P.width;
    const size_t p = static_cast<size_t>(blockIdx.x) * kWfThreads + threadIdx.x;
    if (p >= npx) return;
    const size_t aa = P.aa > 0 ? static_cast<size_t>(P.aa) : 0;
    for (size_t s = 0; s < aa; ++s)
        if (A.redo[p * aa + s]) return;  // rendered by the fix-up pass
    d3 acc = mk(0.0, 0.0, 0.0);
    int samples = 0;
    for (size_t s = 0; s < aa; ++s) {
        const size_t id = p * aa + s;
        // the root's fold (wf_fold_kernel for level 0, same operations) done here
        d3 v = mk(A.val[id], A.val[A.cap + id], A.val[2 * A.cap + id]);
        const int32_t cf = A.child[id], cr = A.child[A.cap + id];
        if (cf >= 0) v = v + mk(A.val[cf], A.val[A.cap + cf], A.val[2 * A.cap + cf]) * A.fw[id];
        if (cr >= 0) v = v + mk(A.val[cr], A.val[A.cap + cr], A.val[2 * A.cap + cr]) * A.rw[id];
        acc = acc + v;
        samples += 1;
    }
    const d3 v = samples > 0 ? sdiv(acc, static_cast<double>(samples)) : mk(0.0, 0.0, 0.0);
    store_pixel(P, p, v);
}

template <bool TREE, bool LDS, bool DEFER>
hipError_t launch_levels(const TraceParams& p, const WfArena& A, size_t lds_bytes,
                         hipStream_t stream) {
    const int max_level = p.max_rec > 0 ? p.max_rec : 0;
    // level 0 exactly covers the roots; deeper levels are persistent grids over the arena
    const uint32_t g0 = static_cast<uint32_t>((A.n0 + kWfThreads - 1) / kWfThreads);
    // Deeper levels: one resident round of workgroups (kWfLevelWaves per CU for the level
    // kernels, 8 for the folds), not more — a level holds far fewer rays than the frame has
    // pixels, and surplus workgroups that find nothing to do still cost their dispatch.
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
        cus = 256;
    const size_t rounds = (A.cap_r + kWfThreads - 1) / kWfThreads;
    const uint32_t gf = static_cast<uint32_t>(std::min<size_t>(static_cast<size_t>(cus) * 8, rounds));
    const size_t lds = LDS ? lds_bytes : 0;
    const uint32_t waves = DEFER ? RT_WF_DEFER_LEVEL_WAVES : kWfLevelWaves;
    const uint32_t gk = static_cast<uint32_t>(
        std::min<size_t>(static_cast<size_t>(cus) * waves, rounds));
    if (g0 > 0)
        hipLaunchKernelGGL((wf_level_kernel<TREE, LDS, DEFER>), dim3(g0), dim3(kWfThreads), lds,
                           stream, p, A, 0);
    // levels 1 .. maxRecursion − 1 (depth maxRecursion is folded in by the last of them)
    for (int k = 1; k < max_level && gk > 0; ++k)
        hipLaunchKernelGGL((wf_level_kernel<TREE, LDS, DEFER>), dim3(gk), dim3(kWfThreads), lds,
                           stream, p, A, k);
    if constexpr (DEFER) {
        // every level's deferred hits: one resident round of workgroups over the queue
        const size_t qrounds = (A.cap + kWfThreads - 1) / kWfThreads;
        const uint32_t gd = static_cast<uint32_t>(
            std::min<size_t>(static_cast<size_t>(cus) * RT_WF_DIRECT_WAVES, qrounds));
        if (max_level > 1 && gd > 0)  // the inner levels' hits
            hipLaunchKernelGGL((wf_direct_kernel<TREE, LDS, false>), dim3(gd), dim3(kWfThreads),
                               lds, stream, p, A);
        if (max_level > 0 && gd > 0)  // the last shading level's hits, folded with the sky
            hipLaunchKernelGGL((wf_direct_kernel<TREE, LDS, true>), dim3(gd), dim3(kWfThreads),
                               lds, stream, p, A);
    }
    // folds of levels maxRecursion − 2 .. 1 (the last shading level folded its nodes itself)
    for (int k = max_level - 2; k >= 1 && gf > 0; --k)
        hipLaunchKernelGGL(wf_fold_kernel, dim3(gf), dim3(kWfThreads), 0, stream, A, k);
    const size_t npx = static_cast<size_t>(p.rows) * p.width;
    if (npx > 0)
        hipLaunchKernelGGL(wf_final_kernel, dim3(static_cast<uint32_t>((npx + kWfThreads - 1) /
                                                                       kWfThreads)),
                           dim3(kWfThreads), 0, stream, p, A);
    return hipGetLastError();
}

}  // namespace

#ifndef RT_LEAN_GENERIC
bool wf_defer_selected() {
    const char* defer_env = std::getenv("RTAMD_WF_DEFER");
    return defer_env && std::atoi(defer_env) == 1;
}

size_t wf_arena_bytes(size_t n0, size_t cap, bool defer) {
    const size_t cap_r = cap - n0;
    return sizeof(double) * (5 * cap + 6 * cap_r) + sizeof(int32_t) * 2 * cap +
           sizeof(uint32_t) * cap_r + (defer ? (sizeof(double) + 2 * sizeof(uint32_t)) * cap : 0) +
           n0 + 64;
}

WfArena wf_arena_layout(void* mem, size_t n0, size_t cap, WfCtl* ctl, bool defer) {
    WfArena A;
    A.n0 = static_cast<uint32_t>(n0);
    A.cap = static_cast<uint32_t>(cap);
    A.cap_r = static_cast<uint32_t>(cap - n0);
    A.defer = defer;
    char* q = static_cast<char*>(mem);
    A.val = reinterpret_cast<double*>(q);
    q += sizeof(double) * 3 * cap;
    A.fw = reinterpret_cast<double*>(q);
    q += sizeof(double) * cap;
    A.rw = reinterpret_cast<double*>(q);
    q += sizeof(double) * cap;
    A.ray = reinterpret_cast<double*>(q);
    q += sizeof(double) * 6 * A.cap_r;
    A.dq_t = nullptr;
    if (defer) {
        A.dq_t = reinterpret_cast<double*>(q);
        q += sizeof(double) * cap;
    }
    A.child = reinterpret_cast<int32_t*>(q);
    q += sizeof(int32_t) * 2 * cap;
    A.root = reinterpret_cast<uint32_t*>(q);
    q += sizeof(uint32_t) * A.cap_r;
    A.dq_id = A.dq_code = nullptr;
    if (defer) {
        A.dq_id = reinterpret_cast<uint32_t*>(q);
        q += sizeof(uint32_t) * cap;
        A.dq_code = reinterpret_cast<uint32_t*>(q);
        q += sizeof(uint32_t) * cap;
    }
    A.redo = reinterpret_cast<uint8_t*>(q);
    A.ctl = ctl;
    return A;
}
#endif

hipError_t launch_wavefront(const TraceParams& p, int path, const WfArena& A, bool lds,
                            size_t lds_bytes, hipStream_t stream) {
    // (the overflow flags A.redo are cleared by the level-0 kernel, root by root)
    hipError_t e = hipMemsetAsync(A.ctl, 0, sizeof(WfCtl), stream);
    if (e != hipSuccess) return e;
    // deferred direct lighting for refraction trees (RTAMD_WF_DEFER=1; off by default: measured
    // on glass 994 vs 971 us per frame, the level kernels 848 -> 480 us but the direct pass 390 us,
    // profiles/r05_glass_defer.txt)
    const bool defer = A.defer;  // wf_defer_selected() when the arena was laid out
    // (the queue's hit code holds a primitive index below 2^26 and a level below 16)
    static_assert(kMaxDepth <= 16, "dq_code level bits");
    const bool fits = p.ns < (1 << 26) && p.np < (1 << 26) && p.nt < (1 << 26);
    if (path == kPathTree && defer && fits)
        e = lds ? launch_levels<true, true, true>(p, A, lds_bytes, stream)
                : launch_levels<true, false, true>(p, A, lds_bytes, stream);
    else if (path == kPathTree)
        e = lds ? launch_levels<true, true, false>(p, A, lds_bytes, stream)
                : launch_levels<true, false, false>(p, A, lds_bytes, stream);
    else
        e = lds ? launch_levels<false, true, false>(p, A, lds_bytes, stream)
                : launch_levels<false, false, false>(p, A, lds_bytes, stream);
    if (e != hipSuccess) return e;
    // fix-up: the per-pixel kernel for pixels whose sample trees overflowed the arena (the lean
    // build's own, rtamd::lean::launch_trace)
    TraceParams q = p;
    q.redo = A.redo;
    q.redo_any = &A.ctl->lost;
#ifdef RT_LEAN_GENERIC
    return rtamd::lean::launch_trace(q, path, false, lds, lds_bytes, stream);
#else
    return rtamd::launch_trace(q, path, false, lds, lds_bytes, stream);
#endif
}

#ifdef RT_LEAN_GENERIC
}  // namespace lean
#endif
}  // namespace rtamd
