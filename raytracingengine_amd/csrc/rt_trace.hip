// rt_trace.hip — the per-pixel FP64 trace kernels for gfx950 (MI355X).
//
// One thread per pixel (per AA sample loop), one wave = 64 contiguous pixels of a row, one
// 256-thread workgroup = a 64×4 tile.  Sphere/plane/light records are staged into LDS once per
// workgroup and read as wave-uniform broadcasts; materials are read from HBM (L2) for the
// winning primitive only.  Geometry is evaluated in IEEE binary64 with the reference's
// operation order (no FMA contraction), so radiance is bit-identical to
// /root/reference/RaytracingEngine/Scene.h except for libm pow (Blinn-Phong, Fresnel).
//
// Reference call graph restated here (Scene.h):
//   RenderImage :311-328 → GeneratePixelAt :283-304 → getRay (Math.h:99-121) → TraceRay :131-198
//   → IntersectClosest :218-257 (Sphere::Intersect Shape.h:72-98, Plane::Intersect :149-159,
//     Triangle::Intersect :202-220) → directLightning :79-129 → computeTransmittance :35-77.
// The recursion of TraceRay becomes an explicit stack: a linear chain (opaque mirrors) folded
// back-to-front to keep the reference's rounding order, or a DFS stack for the refraction tree.
#include "rt_device.hpp"
#include "rt_internal.hpp"

#pragma clang fp contract(off)

namespace rtamd {

struct SceneView {
    const double* sph;
    const double* pl;
    const double* lt;
    const double* tri;
    const double* sph_mat;
    const double* pl_mat;
    const double* tri_mat;
    int ns, np, nt, nl;
};

struct Hit {
    double t;
    int kind;  // 1 sphere, 2 plane, 3 triangle
    int idx;
};

struct Counts {
    uint32_t trace;
    uint32_t shadow;
};

// Scene::IntersectClosest: spheres, then planes, then triangles; a later candidate replaces
// the current one only when strictly closer (HitInfo::isCloserThan, Shape.h:36).
__device__ __forceinline__ bool closest(const SceneView& S, d3 o, d3 d, Hit& h) {
    bool found = false;
    double best = 0.0;
    int kind = 0, idx = -1;
    const double a = dot(d, d);       // Shape.h:75 (same value for every sphere)
    const double two_a = 2.0 * a;     // Shape.h:85-86 denominator
    const double four_a = 4.0 * a;    // Shape.h:79: (4.0 * a) * c
    for (int i = 0; i < S.ns; ++i) {
        const double* s = S.sph + kSphStride * i;
        const d3 oc = o - mk(s[0], s[1], s[2]);
        const double b = 2.0 * dot(oc, d);
        const double c = dot(oc, oc) - s[3];
        const double disc = b * b - four_a * c;
        if (disc < 0.0) continue;
        const double sq = sqrt(disc);
        double t0 = (-b - sq) / two_a;
        double t1 = (-b + sq) / two_a;
        if (t0 > t1) {
            const double tmp = t0;
            t0 = t1;
            t1 = tmp;
        }
        double t = t0;
        if (t < 1e-6) {
            t = t1;
            if (t < 1e-6) continue;
        }
        if (!found || t < best) {
            found = true;
            best = t;
            kind = 1;
            idx = i;
        }
    }
    for (int i = 0; i < S.np; ++i) {
        const double* p = S.pl + kPlStride * i;
        const d3 n = mk(p[3], p[4], p[5]);
        const double denom = dot(n, d);
        if (fabs(denom) > 1e-6) {
            const d3 p0l0 = mk(p[0], p[1], p[2]) - o;
            const double t = dot(p0l0, n) / denom;
            if (t >= 0.0 && (!found || t < best)) {
                found = true;
                best = t;
                kind = 2;
                idx = i;
            }
        }
    }
    for (int i = 0; i < S.nt; ++i) {
        const double* q = S.tri + kTriStride * i;
        const d3 a0 = mk(q[0], q[1], q[2]);
        const d3 e1 = mk(q[3], q[4], q[5]);
        const d3 e2 = mk(q[6], q[7], q[8]);
        const d3 hv = cross(d, e2);
        const double det = dot(e1, hv);
        if (det > -1e-6 && det < 1e-6) continue;
        const double f = 1.0 / det;
        const d3 sv = o - a0;
        const double u = f * dot(sv, hv);
        if (u < 0.0 || u > 1.0) continue;
        const d3 qv = cross(sv, e1);
        const double v = f * dot(d, qv);
        if (v < 0.0 || u + v > 1.0) continue;
        const double t = f * dot(e2, qv);
        if (t > 1e-6 && (!found || t < best)) {
            found = true;
            best = t;
            kind = 3;
            idx = i;
        }
    }
    h.t = best;
    h.kind = kind;
    h.idx = idx;
    return found;
}

__device__ __forceinline__ const double* material_of(const SceneView& S, const Hit& h) {
    return h.kind == 1 ? S.sph_mat + kMatStride * h.idx
         : h.kind == 2 ? S.pl_mat + kMatStride * h.idx
                       : S.tri_mat + kMatStride * h.idx;
}

// Geometric normal at the winner (Sphere::GetNormalAt Shape.h:100-102, Plane Shape.h:161-163,
// Triangle::GetNormalAt Shape.h:222-227 precomputed on the host).
__device__ __forceinline__ d3 normal_of(const SceneView& S, const Hit& h, d3 p) {
    if (h.kind == 1) {
        const double* s = S.sph + kSphStride * h.idx;
        return unit(p - mk(s[0], s[1], s[2]));
    }
    if (h.kind == 2) {
        const double* q = S.pl + kPlStride * h.idx;
        return mk(q[3], q[4], q[5]);
    }
    const double* q = S.tri + kTriStride * h.idx;
    return mk(q[9], q[10], q[11]);
}

// Scene::computeTransmittance (Scene.h:35-77): closest-hit march of up to 64 steps.
__device__ __forceinline__ double transmittance(const SceneView& S, d3 o, d3 d, double max_dist,
                                                double bias) {
    double T = 1.0, traveled = 0.0;
    int safety = 64;
    while (safety-- > 0 && T > 1e-4 && traveled < max_dist) {
        Hit h;
        if (!closest(S, o, d, h)) break;
        const double t = h.t;
        if (t <= 0.0) {
            o = o + d * bias;
            traveled += bias;
            continue;
        }
        if (t <= bias) {
            o = (o + d * t) + d * bias;
            traveled += t + bias;
            continue;
        }
        if (traveled + t >= max_dist) break;
        T *= sclamp(material_of(S, h)[5], 0.0, 1.0);
        o = (o + d * t) + d * bias;
        traveled += t + bias;
    }
    return sclamp(T, 0.0, 1.0);
}

struct Mat {
    d3 color;
    double shininess, specular, transparency, ior;
};

__device__ __forceinline__ Mat load_mat(const double* m) {
    return Mat{mk(m[0], m[1], m[2]), m[3], m[4], m[5], m[6]};
}

// One iteration of directLightning's light loop (Scene.h:86-124).  E = color*intensity.
template <bool COUNT>
__device__ __forceinline__ void light_term(const SceneView& S, d3 P, d3 n, d3 view, const Mat& m,
                                           d3 lpos, d3 E, double bias, d3& diff, d3& spec,
                                           Counts& cnt) {
    const d3 v = lpos - P;
    const double dist = length(v);
    if (dist <= 0.0) return;
    const d3 L = sdiv(v, dist);
    const double ndl = smax(0.0, dot(n, L));
    if (ndl <= 0.0) return;
    if (dist <= bias) return;
    if (COUNT) cnt.shadow++;
    const double T = transmittance(S, P + n * bias, L, dist - bias, bias);
    if (T <= bias) return;
    const double inv_d2 = 1.0 / (dist * dist);
    diff = diff + ((E * inv_d2) * ndl) * T;
    if (m.transparency <= 0.0 && m.specular > 0.0) {
        const d3 H = unit(L + view);
        const double ndh = smax(0.0, dot(n, H));
        if (ndh > 0.0) {
            const double sf = pow(ndh, m.shininess);
            spec = spec + ((E * inv_d2) * sf) * T;
        }
    }
}

// Scene::directLightning (Scene.h:79-129), plus the build-defined area-light samples.
template <bool COUNT>
__device__ __forceinline__ d3 direct(const SceneView& S, const TraceParams& P, d3 hp, d3 view,
                                     d3 n_in, const Mat& m, uint64_t pix, uint32_t sample,
                                     int depth, Counts& cnt) {
    const double bias = P.bias;
    const d3 n = unit(n_in);
    d3 diff = mk(0.0, 0.0, 0.0), spec = mk(0.0, 0.0, 0.0);
    for (int i = 0; i < S.nl; ++i) {
        const double* l = S.lt + kLtStride * i;
        light_term<COUNT>(S, hp, n, view, m, mk(l[0], l[1], l[2]), mk(l[3], l[4], l[5]), bias,
                          diff, spec, cnt);
    }
    if (P.al_samples > 0) {
        const uint32_t stream = 0x10000u + (sample << 6) + static_cast<uint32_t>(depth);
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
            light_term<COUNT>(S, hp, n, view, m, lp, E, bias, diff, spec, cnt);
        }
    }
    return hmul(m.color, diff) + spec * m.specular;
}

// What one TraceRay invocation yields before its children are traced.
struct Node {
    d3 value;    // sky colour on a miss, else (0,0,0) + local*(1-tr) (Scene.h:175-179)
    d3 ro, rd;   // reflection ray            (Scene.h:189-195)
    d3 fo, fd;   // refraction ray            (Scene.h:181-187)
    double rw;   // reflectiveness
    double fw;   // transparency * (1 - fresnel)
    bool hit, refl, refr;
};

template <bool TREE, bool COUNT>
__device__ __forceinline__ Node shade(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                      uint64_t pix, uint32_t sample, int depth, Counts& cnt) {
    Node nd;
    nd.refl = false;
    nd.refr = false;
    if (COUNT) cnt.trace++;
    Hit h;
    if (!closest(S, o, d, h)) {
        nd.hit = false;
        nd.value = sky(d);
        return nd;
    }
    nd.hit = true;
    const double bias = P.bias;
    const d3 hp = o + d * h.t;  // Rayon::pointAtDistance
    const d3 gn = normal_of(S, h, hp);
    const Mat m = load_mat(material_of(S, h));
    const d3 inc = unit(d);
    const bool front = dot(gn, inc) < 0.0;
    const d3 n = front ? gn : -gn;
    const d3 view = -inc;
    const double tr = sclamp(m.transparency, 0.0, 1.0);
    const d3 local = direct<COUNT>(S, P, hp, view, n, m, pix, sample, depth, cnt);
    d3 fin = mk(0.0, 0.0, 0.0);
    if (tr < 1.0) fin = fin + local * (1.0 - tr);
    nd.value = fin;
    double refl_w = m.specular;
    if (TREE && tr > 0.0) {
        // fresnel (Scene.h:26-28, 161-164); only consumed when tr > 0.
        const double cos_t = smax(0.0, dot(n, view));
        const double eta_t = m.ior;
        const double r0 = (eta_t - 1.0) / (eta_t + 1.0);
        const double f0 = r0 * r0;  // pow(x, 2.0)
        double F = f0 + (1.0 - f0) * pow(1.0 - cos_t, 5.0);
        const double eta = front ? (1.0 / eta_t) : (eta_t / 1.0);
        d3 rd = refract(inc, n, eta);
        if (length(rd) > bias) {
            rd = unit(rd);
            nd.refr = true;
            nd.fd = rd;
            nd.fo = hp + rd * (bias * 1e2);
            nd.fw = tr * (1.0 - F);
        } else {
            F = 1.0;
        }
        refl_w = F;
    }
    if (refl_w > bias) {
        const d3 R = unit(reflect(inc, n));
        nd.refl = true;
        nd.rd = R;
        nd.ro = hp + R * bias;
        nd.rw = refl_w;
    }
    return nd;
}

// TraceRay for scenes where no secondary ray can be spawned.
template <bool COUNT>
__device__ __forceinline__ d3 trace_direct(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                           uint64_t pix, uint32_t sample, Counts& cnt) {
    if (P.max_rec <= 0) return sky(d);
    return shade<false, COUNT>(S, P, o, d, pix, sample, 0, cnt).value;
}

// TraceRay for opaque scenes: a linear reflection chain.  Levels are pushed front-to-back and
// folded back-to-front, final_k = value_k + child_k * rw_k, the reference's rounding order.
template <bool COUNT>
__device__ __forceinline__ d3 trace_chain(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                          uint64_t pix, uint32_t sample, Counts& cnt) {
    d3 base[kMaxDepth];
    double w[kMaxDepth];
    int depth = 0;
    d3 leaf;
    while (true) {
        if (depth >= P.max_rec) {
            leaf = sky(d);
            break;
        }
        const Node nd = shade<false, COUNT>(S, P, o, d, pix, sample, depth, cnt);
        if (!nd.hit || !nd.refl) {
            leaf = nd.value;
            break;
        }
        base[depth] = nd.value;
        w[depth] = nd.rw;
        o = nd.ro;
        d = nd.rd;
        ++depth;
    }
    d3 acc = leaf;
    for (int k = depth - 1; k >= 0; --k) acc = base[k] + acc * w[k];
    return acc;
}

// TraceRay with transparency: depth-first walk of the refraction/reflection tree with an
// explicit stack.  A frame waits first for its refraction child (added with weight fw), then
// for its reflection child (weight rw), in the reference's accumulation order.
template <bool COUNT>
__device__ __forceinline__ d3 trace_tree(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                         uint64_t pix, uint32_t sample, Counts& cnt) {
    struct Frame {
        d3 acc, ro, rd;
        double rw, fw;
        int phase;  // 1: waiting for the refraction child, 2: waiting for the reflection child
        bool refl;
    };
    Frame st[kMaxDepth];
    int sp = 0;
    d3 val;
    while (true) {
        // descend from (o, d) at depth sp
        if (sp >= P.max_rec) {
            val = sky(d);
        } else {
            const Node nd = shade<true, COUNT>(S, P, o, d, pix, sample, sp, cnt);
            if (nd.hit && (nd.refr || nd.refl)) {
                Frame& f = st[sp];
                f.acc = nd.value;
                f.ro = nd.ro;
                f.rd = nd.rd;
                f.rw = nd.rw;
                f.fw = nd.fw;
                f.refl = nd.refl;
                ++sp;
                if (nd.refr) {
                    f.phase = 1;
                    o = nd.fo;
                    d = nd.fd;
                } else {
                    f.phase = 2;
                    o = nd.ro;
                    d = nd.rd;
                }
                continue;
            }
            val = nd.value;
        }
        // ascend: fold `val` into the waiting frames
        bool descend = false;
        while (sp > 0) {
            Frame& f = st[sp - 1];
            if (f.phase == 1) {
                f.acc = f.acc + val * f.fw;
                if (f.refl) {
                    f.phase = 2;
                    o = f.ro;
                    d = f.rd;
                    descend = true;
                    break;
                }
            } else {
                f.acc = f.acc + val * f.rw;
            }
            val = f.acc;
            --sp;
        }
        if (!descend) return val;
    }
}

template <int PATH, bool COUNT, bool LDS>
__global__ __launch_bounds__(kTileW * kTileH) void trace_kernel(TraceParams P) {
    extern __shared__ double smem[];
    SceneView S;
    S.ns = P.ns;
    S.np = P.np;
    S.nt = P.nt;
    S.nl = P.nl;
    S.tri = P.tri;
    S.sph_mat = P.sph_mat;
    S.pl_mat = P.pl_mat;
    S.tri_mat = P.tri_mat;
    if constexpr (LDS) {
        const int tid = threadIdx.y * kTileW + threadIdx.x;
        constexpr int nthr = kTileW * kTileH;
        double* s_sph = smem;
        double* s_pl = s_sph + kSphStride * P.ns;
        double* s_lt = s_pl + kPlStride * P.np;
        for (int i = tid; i < kSphStride * P.ns; i += nthr) s_sph[i] = P.sph[i];
        for (int i = tid; i < kPlStride * P.np; i += nthr) s_pl[i] = P.pl[i];
        for (int i = tid; i < kLtStride * P.nl; i += nthr) s_lt[i] = P.lt[i];
        __syncthreads();
        S.sph = s_sph;
        S.pl = s_pl;
        S.lt = s_lt;
    } else {
        S.sph = P.sph;
        S.pl = P.pl;
        S.lt = P.lt;
    }

    const uint32_t x = blockIdx.x * kTileW + threadIdx.x;
    const uint32_t yl = blockIdx.y * kTileH + threadIdx.y;
    Counts cnt{0u, 0u};
    if (x < P.width && yl < P.rows) {
        const uint32_t y = P.row0 + yl;
        const uint64_t pix = static_cast<uint64_t>(y) * P.width + x;
        const d3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
        // GeneratePixelAt (Scene.h:283-304)
        d3 acc = mk(0.0, 0.0, 0.0);
        int samples = 0;
        for (int s = 0; s < P.aa; ++s) {
            // Camera::getRay (Math.h:99-121); sample 0 is never jittered.
            double sx = static_cast<double>(x) - static_cast<double>(P.width) / 2.0;
            double sy = static_cast<double>(P.height) / 2.0 - static_cast<double>(y);
            double jx = 0.0, jy = 0.0;
            if (s > 0 && P.aa > 1) {
                jx = u01(P.seed, pix, static_cast<uint32_t>(s), 0u);
                jy = u01(P.seed, pix, static_cast<uint32_t>(s), 1u);
            }
            sx += jx;
            sy += jy;
            const d3 dir = unit(mk(sx, sy, cam.z + P.focal) - cam);
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
        const d3 v = samples > 0 ? sdiv(acc, static_cast<double>(samples)) : mk(0.0, 0.0, 0.0);
        const size_t o = static_cast<size_t>(yl) * P.width + x;
        if (P.out64) {
            P.out64[3 * o + 0] = v.x;
            P.out64[3 * o + 1] = v.y;
            P.out64[3 * o + 2] = v.z;
        }
        if (P.out32) {
            P.out32[3 * o + 0] = static_cast<float>(v.x);
            P.out32[3 * o + 1] = static_cast<float>(v.y);
            P.out32[3 * o + 2] = static_cast<float>(v.z);
        }
        if (P.ldr) {
            uint8_t r, g, b;
            to_color(tonemap_op(v, P.tonemap), r, g, b);
            P.ldr[3 * o + 0] = r;
            P.ldr[3 * o + 1] = g;
            P.ldr[3 * o + 2] = b;
        }
    }
    if constexpr (COUNT) {
        // wave-reduce the two counters, one 64-bit atomic per wave per counter
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

template <int PATH, bool COUNT, bool LDS>
static hipError_t launch_one(const TraceParams& p, size_t lds_bytes, hipStream_t stream) {
    const dim3 block(kTileW, kTileH);
    const dim3 grid((p.width + kTileW - 1) / kTileW, (p.rows + kTileH - 1) / kTileH);
    hipLaunchKernelGGL((trace_kernel<PATH, COUNT, LDS>), grid, block, LDS ? lds_bytes : 0,
                       stream, p);
    return hipGetLastError();
}

template <int PATH>
static hipError_t launch_path(const TraceParams& p, bool count, bool lds, size_t lds_bytes,
                              hipStream_t stream) {
    if (count)
        return lds ? launch_one<PATH, true, true>(p, lds_bytes, stream)
                   : launch_one<PATH, true, false>(p, lds_bytes, stream);
    return lds ? launch_one<PATH, false, true>(p, lds_bytes, stream)
               : launch_one<PATH, false, false>(p, lds_bytes, stream);
}

hipError_t launch_trace(const TraceParams& p, int path, bool count, bool lds, size_t lds_bytes,
                        hipStream_t stream) {
    switch (path) {
    case kPathDirect: return launch_path<kPathDirect>(p, count, lds, lds_bytes, stream);
    case kPathChain: return launch_path<kPathChain>(p, count, lds, lds_bytes, stream);
    default: return launch_path<kPathTree>(p, count, lds, lds_bytes, stream);
    }
}

// ------------------------------------------------------------------ batch ray queries
__device__ __forceinline__ SceneView global_view(const TraceParams& P) {
    SceneView S;
    S.ns = P.ns;
    S.np = P.np;
    S.nt = P.nt;
    S.nl = P.nl;
    S.sph = P.sph;
    S.pl = P.pl;
    S.lt = P.lt;
    S.tri = P.tri;
    S.sph_mat = P.sph_mat;
    S.pl_mat = P.pl_mat;
    S.tri_mat = P.tri_mat;
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
        to_color(tonemap_op(c, k), o[0], o[1], o[2]);
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
    out[4 * i + 0] = x[i] / y[i];
    out[4 * i + 1] = sqrt(x[i]);
    out[4 * i + 2] = pow(x[i], y[i]);
    out[4 * i + 3] = log(x[i]);
}

hipError_t launch_debug_f64(const double* x, const double* y, size_t n, double* out,
                            hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(debug_f64_kernel, dim3(blocks), dim3(256), 0, stream, x, y, n, out);
    return hipGetLastError();
}

}  // namespace rtamd
