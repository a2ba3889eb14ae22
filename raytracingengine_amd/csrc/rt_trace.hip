// rt_trace.hip — the per-pixel FP64 trace kernels for gfx950 (MI355X).
//
// One thread per pixel (per AA sample loop), one wave = an 8×8 tile, one 256-thread workgroup
// = an 8×32 tile.  Sphere/plane/light records are staged into LDS once per
// workgroup and read as wave-uniform broadcasts; materials are read from HBM (L2) for the
// winning primitive only.  Geometry is evaluated in IEEE binary64 with the reference's
// operation order (no FMA contraction), so radiance is bit-identical to
// /root/reference/RaytracingEngine/Scene.h except for libm pow (Blinn-Phong, Fresnel).
//
// Reference call graph restated here (Scene.h):
//   RenderImage :311-328 → GeneratePixelAt :283-304 → getRay (Math.h:99-121) → TraceRay :131-198
//   → IntersectClosest :218-257 (Sphere::Intersect Shape.h:72-98, Plane::Intersect :149-159,
//     Triangle::Intersect :202-220) → directLightning :79-129 → computeTransmittance :35-77.
// The recursion of TraceRay becomes a linear chain accumulated front to back (opaque mirrors,
// trace_chain) or a DFS stack for the refraction tree (the reference's order).
#include "rt_trace_common.hpp"

#pragma clang fp contract(off)

namespace rtamd {
#ifndef RT_CHAIN_NOSPH_WAVES
#define RT_CHAIN_NOSPH_WAVES 3
#endif
#ifdef RT_LEAN_GENERIC
// rt_trace_lean.hip: the per-pixel kernels again, without the triangle / BVH and area-light code
// (rt_trace_common.hpp), for scenes that have neither: fewer registers, C1 / mirror ~5 % faster.
namespace lean {
#endif

// MINW: minimum waves per SIMD the register budget is compiled for; SINGLE: one sample per pixel
// (AA = 1: no sample loop, no accumulator live across the trace).
// NOSPH: the scene has no spheres (C1, the reference's own box of planes): the sphere loops and
// the sphere shading code compile away (AA = 1 chain: 80 -> 48 B/lane of spills at 3 waves/SIMD,
// C1 489 -> 453 us on MI355X; at 4 waves it spills 224 B/lane and takes 808 us, at 5 1256 us).
// SPAR: sample-parallel multi-sample frames (2 ≤ aa ≤ kAaParallelMax, direct / chain paths, never
// the fix-up pass): thread t of the workgroup traces sample t mod aa of pixel t div aa (256 / aa
// consecutive pixels of the row-major frame per workgroup, a 1-D grid) with the single-sample
// code and register budget; the colours meet in LDS and one thread per pixel adds them in sample
// order and divides by aa (GeneratePixelAt, Scene.h:292-300) — the per-thread loop's operations
// in its order, so the same image (RT_FLAG_NO_SAMPLE_PARALLEL keeps the loop).
template <int PATH, bool COUNT, bool LDS, int MINW = 2, bool SINGLE = false, bool NOSPH = false,
          bool SPAR = false>
__global__ __launch_bounds__(kTileW * kTileH, MINW) void trace_kernel(TraceParams P) {
    extern __shared__ double smem[];
    constexpr int kThreads = kTileW * kTileH;
    __shared__ double s_c[SPAR ? 3 * kThreads : 1];
    const int tid = threadIdx.y * kTileW + threadIdx.x;
    const int ppw = SPAR ? kThreads / P.aa : 1;           // pixels per workgroup (SPAR)
    const int spl = SPAR ? tid / P.aa : 0, ss = SPAR ? tid - spl * P.aa : 0;
    const uint64_t slin = static_cast<uint64_t>(blockIdx.x) * ppw + spl;
    const uint32_t x = SPAR ? static_cast<uint32_t>(slin % P.width) : blockIdx.x * kTileW + threadIdx.x;
    const uint32_t yl = SPAR ? static_cast<uint32_t>(slin / P.width) : blockIdx.y * kTileH + threadIdx.y;
    Counts cnt{0u, 0u};
    bool run = SPAR ? (spl < ppw && slin < static_cast<uint64_t>(P.width) * P.rows)
                    : (x < P.width && yl < P.rows);
    if (P.redo) {  // uniform
        // fix-up pass of the wavefront renderer: only pixels with an incomplete sample tree,
        // and workgroups without one leave before staging the scene (all of them at once when
        // no tree overflowed: one scalar load)
        if (P.redo_any && *P.redo_any == 0u) return;
        if (run) {
            const size_t r0 = (static_cast<size_t>(yl) * P.width + x) * static_cast<size_t>(P.aa);
            bool any = false;
            for (int s = 0; s < P.aa; ++s) any = any || P.redo[r0 + s] != 0;
            run = any;
        }
        if (!__syncthreads_or(run)) return;
    }
    SceneView S = stage_scene<LDS>(P, smem, tid, kTileW * kTileH);
    if constexpr (NOSPH) S.ns = 0;  // the launcher checked P.ns == 0
    if (run) {
        const uint32_t y = image_row(P, yl);
        const uint64_t pix = static_cast<uint64_t>(y) * P.width + x;
        const d3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
        // GeneratePixelAt (Scene.h:283-304)
        d3 acc = mk(0.0, 0.0, 0.0);
        int samples = 0;
        const int nsamples = (SINGLE || SPAR) ? 1 : P.aa;
        for (int s0 = 0; s0 < nsamples; ++s0) {
            const int s = SPAR ? ss : s0;
            const d3 dir = camera_dir(P, cam, x, y, pix, s);
            d3 c;
            if constexpr (PATH == kPathDirect)
                c = trace_direct<COUNT>(S, P, cam, dir, pix, static_cast<uint32_t>(s), cnt);
            else if constexpr (PATH == kPathChain)
                c = trace_chain<COUNT>(S, P, cam, dir, pix, static_cast<uint32_t>(s), cnt);
            else
                c = trace_tree<COUNT>(S, P, cam, dir, pix, static_cast<uint32_t>(s), cnt);
            acc = acc + c;
            samples += 1;
        }
        if constexpr (SPAR) {
            s_c[tid] = acc.x;  // 0 + c: the colour as the loop's first addition makes it
            s_c[kThreads + tid] = acc.y;
            s_c[2 * kThreads + tid] = acc.z;
        } else {
            const d3 v = samples > 0 ? sdiv(acc, static_cast<double>(samples)) : mk(0.0, 0.0, 0.0);
            store_pixel(P, static_cast<size_t>(yl) * P.width + x, v);
        }
    }
    if constexpr (SPAR) {
        __syncthreads();
        const uint64_t out = static_cast<uint64_t>(blockIdx.x) * ppw + tid;
        if (tid < ppw && out < static_cast<uint64_t>(P.width) * P.rows) {
            d3 acc = mk(0.0, 0.0, 0.0);
            for (int k = 0; k < P.aa; ++k) {
                const int j = tid * P.aa + k;
                acc = acc + mk(s_c[j], s_c[kThreads + j], s_c[2 * kThreads + j]);
            }
            store_pixel(P, static_cast<size_t>(out), sdiv(acc, static_cast<double>(P.aa)));
        }
    }
    if constexpr (COUNT) {
        // wave-reduce the two counters, one 64-bit atomic per wave per counter
        uint32_t t = cnt.trace, s = cnt.shadow;
        for (int off = 32; off > 0; off >>= 1) {
            t += __shfl_xor(t, off, 64);
            s += __shfl_xor(s, off, 64);
        }
        if ((tid & 63) == 0) {
            atomicAdd(P.counters + 0, static_cast<unsigned long long>(t));
            atomicAdd(P.counters + 1, static_cast<unsigned long long>(s));
        }
    }
}

template <int PATH, bool COUNT, bool LDS, int MINW, bool SINGLE, bool NOSPH = false,
          bool SPAR = false>
static hipError_t launch_one(const TraceParams& p, size_t lds_bytes, hipStream_t stream) {
    const dim3 block(kTileW, kTileH);
    dim3 grid((p.width + kTileW - 1) / kTileW, (p.rows + kTileH - 1) / kTileH);
    if constexpr (SPAR) {  // 1-D: 256 / aa pixels per workgroup
        const uint64_t ppw = static_cast<uint64_t>(kTileW * kTileH / p.aa);
        grid = dim3(static_cast<unsigned>((static_cast<uint64_t>(p.width) * p.rows + ppw - 1) / ppw));
    }
    hipLaunchKernelGGL((trace_kernel<PATH, COUNT, LDS, MINW, SINGLE, NOSPH, SPAR>), grid, block,
                       LDS ? lds_bytes : 0, stream, p);
    return hipGetLastError();
}

template <int PATH, int MINW, bool SINGLE, bool NOSPH = false, bool SPAR = false>
static hipError_t launch_lds(const TraceParams& p, bool count, bool lds, size_t lds_bytes,
                             hipStream_t stream) {
    if (count)
        return lds ? launch_one<PATH, true, true, MINW, SINGLE, NOSPH, SPAR>(p, lds_bytes, stream)
                   : launch_one<PATH, true, false, MINW, SINGLE, NOSPH, SPAR>(p, lds_bytes, stream);
    return lds ? launch_one<PATH, false, true, MINW, SINGLE, NOSPH, SPAR>(p, lds_bytes, stream)
               : launch_one<PATH, false, false, MINW, SINGLE, NOSPH, SPAR>(p, lds_bytes, stream);
}

template <int PATH>
static hipError_t launch_path(const TraceParams& p, bool count, bool lds, size_t lds_bytes,
                              hipStream_t stream, bool spar) {
    // multi-sample direct / chain frames: one thread per sample at the single-sample budget
    const bool sp = spar && PATH != kPathTree && !p.redo && p.aa >= 2 && p.aa <= kAaParallelMax;
#ifdef RT_LEAN_GENERIC
    // Reflection chains (C1, mirror) without triangles / area light: compiled for 3 waves/SIMD
    // (168 VGPRs; the forward-accumulated chain needs no stack) — C1 702 -> 568 us, mirror
    // 2189 -> 1684 us on MI355X; 4 waves spills 320 B/lane and loses (C1 900 us).  AA = 1 takes
    // the single-sample instantiation (80 instead of 144 B/lane of spills).
    if constexpr (PATH == kPathChain) {
        if (sp && p.ns == 0)
            return launch_lds<PATH, RT_CHAIN_NOSPH_WAVES, true, true, true>(p, count, lds, lds_bytes, stream);
        if (sp) return launch_lds<PATH, 3, true, false, true>(p, count, lds, lds_bytes, stream);
        if (p.ns == 0 && p.aa == 1 && !p.redo)
            return launch_lds<PATH, RT_CHAIN_NOSPH_WAVES, true, true>(p, count, lds, lds_bytes, stream);
        if (p.aa == 1 && !p.redo) return launch_lds<PATH, 3, true>(p, count, lds, lds_bytes, stream);
        if (p.ns == 0 && !p.redo) return launch_lds<PATH, 3, false, true>(p, count, lds, lds_bytes, stream);
        return launch_lds<PATH, 3, false>(p, count, lds, lds_bytes, stream);
    } else
#endif
    {
        if constexpr (PATH != kPathTree)
            if (sp) return launch_lds<PATH, 2, true, false, true>(p, count, lds, lds_bytes, stream);
        return launch_lds<PATH, 2, false>(p, count, lds, lds_bytes, stream);
    }
}

hipError_t launch_trace(const TraceParams& p, int path, bool count, bool lds, size_t lds_bytes,
                        hipStream_t stream, bool sample_parallel) {
    switch (path) {
    case kPathDirect: return launch_path<kPathDirect>(p, count, lds, lds_bytes, stream, sample_parallel);
    case kPathChain: return launch_path<kPathChain>(p, count, lds, lds_bytes, stream, sample_parallel);
    default: return launch_path<kPathTree>(p, count, lds, lds_bytes, stream, sample_parallel);
    }
}

#ifdef RT_LEAN_GENERIC
}  // namespace lean
#else

// ------------------------------------------------------------------ batch ray queries
__device__ __forceinline__ SceneView global_view(const TraceParams& P) {
    SceneView S;
    S.ns = P.ns;
    S.np = P.np;
    S.nt = P.nt;
    S.nl = P.nl;
    S.al = P.al_samples;
    S.spec = true;
    S.sph = P.sph;
    S.pl = P.pl;
    S.lt = P.lt;
    S.tri = P.tri;
    S.sph_mat = P.sph_mat;
    S.pl_mat = P.pl_mat;
    S.tri_mat = P.tri_mat;
    S.bvh = P.bvh;
    S.bvh_tri = P.bvh_tri;
    return S;
}

// TraceRay(ray, 0, bias) for arbitrary rays (GenerateAntiAliasing's body, Scene.h:306-309).
template <int PATH, bool COUNT>
__global__ __launch_bounds__(256) void trace_rays_kernel(TraceParams P, const double* rays,
                                                         size_t n, double* out) {
    const SceneView S = global_view(P);
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    Counts cnt{0u, 0u};
    if (i < n) {
        const double* r = rays + 6 * i;
        const d3 o = mk(r[0], r[1], r[2]);
        const d3 d = mk(r[3], r[4], r[5]);
        d3 c;
        if constexpr (PATH == kPathDirect) c = trace_direct<COUNT>(S, P, o, d, i, 0u, cnt);
        else if constexpr (PATH == kPathChain) c = trace_chain<COUNT>(S, P, o, d, i, 0u, cnt);
        else c = trace_tree<COUNT>(S, P, o, d, i, 0u, cnt);
        out[3 * i + 0] = c.x;
        out[3 * i + 1] = c.y;
        out[3 * i + 2] = c.z;
    }
    if constexpr (COUNT) {
        uint32_t t = cnt.trace, s = cnt.shadow;
        for (int off = 32; off > 0; off >>= 1) {
            t += __shfl_xor(t, off, 64);
            s += __shfl_xor(s, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(P.counters + 0, static_cast<unsigned long long>(t));
            atomicAdd(P.counters + 1, static_cast<unsigned long long>(s));
        }
    }
}

// IntersectClosest for arbitrary rays: {type, index, t, normal, hit point} per ray.
__global__ __launch_bounds__(256) void intersect_rays_kernel(TraceParams P, const double* rays,
                                                             size_t n, double* out) {
    const SceneView S = global_view(P);
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* r = rays + 6 * i;
    const d3 o = mk(r[0], r[1], r[2]);
    const d3 d = mk(r[3], r[4], r[5]);
    double* w = out + 9 * i;
    Hit h;
    if (!closest(S, o, d, h)) {
        w[0] = 0.0;
        w[1] = -1.0;
        for (int k = 2; k < 9; ++k) w[k] = 0.0;
        return;
    }
    const d3 p = o + d * h.t;
    const d3 nn = normal_of(S, h, p);
    w[0] = static_cast<double>(h.kind);
    w[1] = static_cast<double>(h.idx);
    w[2] = h.t;
    w[3] = nn.x;
    w[4] = nn.y;
    w[5] = nn.z;
    w[6] = p.x;
    w[7] = p.y;
    w[8] = p.z;
}

hipError_t launch_trace_rays(const TraceParams& p, int path, bool count, const double* rays,
                             size_t n, double* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 grid(static_cast<unsigned>((n + 255) / 256)), block(256);
    if (path == kPathDirect) {
        if (count) hipLaunchKernelGGL((trace_rays_kernel<kPathDirect, true>), grid, block, 0, stream, p, rays, n, out);
        else hipLaunchKernelGGL((trace_rays_kernel<kPathDirect, false>), grid, block, 0, stream, p, rays, n, out);
    } else if (path == kPathChain) {
        if (count) hipLaunchKernelGGL((trace_rays_kernel<kPathChain, true>), grid, block, 0, stream, p, rays, n, out);
        else hipLaunchKernelGGL((trace_rays_kernel<kPathChain, false>), grid, block, 0, stream, p, rays, n, out);
    } else {
        if (count) hipLaunchKernelGGL((trace_rays_kernel<kPathTree, true>), grid, block, 0, stream, p, rays, n, out);
        else hipLaunchKernelGGL((trace_rays_kernel<kPathTree, false>), grid, block, 0, stream, p, rays, n, out);
    }
    return hipGetLastError();
}

hipError_t launch_intersect_rays(const TraceParams& p, const double* rays, size_t n, double* out,
                                 hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(intersect_rays_kernel, dim3(static_cast<unsigned>((n + 255) / 256)),
                       dim3(256), 0, stream, p, rays, n, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ tonemap
// op in [0,7): one operator; op == 7: all seven in tonemapAll() order (out is 7 planes).
__global__ __launch_bounds__(256) void tonemap_kernel(const double* __restrict__ hdr, size_t n,
                                                      int op, uint8_t* __restrict__ out) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const d3 c = mk(hdr[3 * i], hdr[3 * i + 1], hdr[3 * i + 2]);
    const int lo = op == 7 ? 0 : op, hi = op == 7 ? 7 : op + 1;
    for (int k = lo; k < hi; ++k) {
        uint8_t* o = out + (op == 7 ? static_cast<size_t>(k) * 3 * n : 0) + 3 * i;
        if (k == 1) {  // the packet kernel's fused Reinhard bytes, the same function
            o[0] = reinhard_byte(c.x);
            o[1] = reinhard_byte(c.y);
            o[2] = reinhard_byte(c.z);
        } else {
            to_color(tonemap_op(c, k), o[0], o[1], o[2]);
        }
    }
}

hipError_t launch_tonemap(const double* hdr, size_t n, int op, uint8_t* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(tonemap_kernel, dim3(blocks), dim3(256), 0, stream, hdr, n, op, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ libm pinning hook
__global__ void debug_f64_kernel(const double* x, const double* y, size_t n, double* out) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[5 * i + 0] = x[i] / y[i];
    out[5 * i + 1] = sqrt(x[i]);
    out[5 * i + 2] = pow(x[i], y[i]);
    out[5 * i + 3] = log(x[i]);
    out[5 * i + 4] = pow_bp(x[i], y[i]);
}

hipError_t launch_debug_f64(const double* x, const double* y, size_t n, double* out,
                            hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(debug_f64_kernel, dim3(blocks), dim3(256), 0, stream, x, y, n, out);
    return hipGetLastError();
}

// Test hook for the sqrt/division cores (rt_device.hpp): per input vector v, the fast and the
// compiler-lowered exact results side by side (a test compares them bit for bit).
//   out[16i + 0..2]  unit(v)          out[16i + 3..5]   unit_exact(v)
//   out[16i + 6..10] light_dir(v): dist, L, 1/(dist·dist)
//   out[16i + 11..15] exact: sqrt(v·v), v/dist, 1/(dist·dist)
__global__ void debug_vec_kernel(const double* v, size_t n, double* out) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const d3 a = mk(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
    double* o = out + 16 * i;
    const d3 u = unit(a), ue = unit_exact(a);
    double dist, inv_d2;
    d3 L;
    light_dir(a, dist, L, inv_d2);
    const double de = length(a);
    const d3 Le = sdiv(a, de);
    const double ie = 1.0 / (de * de);
    const double vals[16] = {u.x,  u.y,  u.z,  ue.x, ue.y, ue.z, dist, L.x,
                             L.y,  L.z,  inv_d2, de, Le.x, Le.y, Le.z, ie};
    for (int k = 0; k < 16; ++k) o[k] = vals[k];
}

hipError_t launch_debug_vec(const double* v, size_t n, double* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(debug_vec_kernel, dim3(blocks), dim3(256), 0, stream, v, n, out);
    return hipGetLastError();
}

#endif  // RT_LEAN_GENERIC
}  // namespace rtamd
