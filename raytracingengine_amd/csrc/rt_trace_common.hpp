// rt_trace_common.hpp — device building blocks of the trace kernels, shared by the generic
// kernels (rt_trace.hip) and the packet-culled fast kernel (rt_packet.hip).
//
// Reference functions restated (paths relative to /root/reference/RaytracingEngine):
//   IntersectClosest Scene.h:218-257 (Sphere::Intersect Shape.h:72-98, Plane::Intersect
//   Shape.h:149-159, Triangle::Intersect Shape.h:202-220), computeTransmittance Scene.h:35-77,
//   directLightning Scene.h:79-129, TraceRay Scene.h:131-198.
#pragma once

#include "rt_device.hpp"
#include "rt_internal.hpp"

#pragma clang fp contract(off)

namespace rtamd {

// ------------------------------------------------------------------ wave reductions (FP32)
// Every lane must be active.  Floats are reduced as order-preserving int32 keys (sign-magnitude
// to two's complement), so each step is one integer min/max on a DPP-permuted operand: four
// steps reduce each 16-lane row (quad xor-1, quad xor-2, half-mirror, mirror), then the four row
// values are combined in SGPRs.  NaN keys sort above +inf (a max returns NaN, a min skips it).
template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ int f2key(float v) {
    const int b = __float_as_int(v);
    return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float key2f(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }
template <int OP>  // 0 min, 1 max
__device__ __forceinline__ float wave_red(float x) {
    auto op = [](int a, int b) { return OP == 0 ? (a < b ? a : b) : (a < b ? b : a); };
    int v = f2key(x);
    v = op(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp<0x141>(v));  // row_half_mirror
    v = op(v, dpp<0x140>(v));  // row_mirror
    const int r = op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
                     op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
    return key2f(r);
}

// Lane `l`'s double / vector, broadcast to every lane (exact: a bit copy via SGPRs).
__device__ __forceinline__ double lane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ d3 lane_d3(d3 v, int l) {
    return mk(lane_d(v.x, l), lane_d(v.y, l), lane_d(v.z, l));
}

struct SceneView {
    const double* sph;
    const double* pl;
    const double* lt;
    const double* tri;
    const double* sph_mat;
    const double* pl_mat;
    const double* tri_mat;
    const double* bvh;       // triangle BVH (null: every triangle is tested)
    const int32_t* bvh_tri;
    int ns, np, nt, nl;
    int al;  // samples of the build-defined area light (TraceParams.al_samples), 0: none
    bool spec;  // false: no material has specular > 0 (the Blinn-Phong term is not compiled in)
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

// Triangle::Intersect (Shape.h:202-220), Möller–Trumbore with the reference's operation order;
// true with t when the triangle is hit at t > 1e-6.
__device__ __forceinline__ bool tri_hit_v(d3 a0, d3 e1, d3 e2, d3 o, d3 d, double& t) {
    const d3 hv = cross(d, e2);
    const double det = dot(e1, hv);
    if (det > -1e-6 && det < 1e-6) return false;
    const double f = 1.0 / det;
    const d3 sv = o - a0;
    const double u = f * dot(sv, hv);
    if (u < 0.0 || u > 1.0) return false;
    const d3 qv = cross(sv, e1);
    const double v = f * dot(d, qv);
    if (v < 0.0 || u + v > 1.0) return false;
    t = f * dot(e2, qv);
    return t > 1e-6;
}
__device__ __forceinline__ bool tri_hit(const double* tri, int i, d3 o, d3 d, double& t) {
    const double* q = tri + kTriStride * i;
    return tri_hit_v(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]), o, d, t);
}

// Conservative ray / box test (boxes are widened at build time, rt_bvh.cpp): false only when
// no point of the box is on the ray at t >= 0.  tn = entry parameter (a lower bound).
__device__ __forceinline__ bool bvh_box_v(d3 blo, d3 bhi, d3 o, d3 d, d3 inv, double& tn) {
    double lo = -INFINITY, hi = INFINITY;
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z}, ii[3] = {inv.x, inv.y, inv.z};
    const double nd[6] = {blo.x, blo.y, blo.z, bhi.x, bhi.y, bhi.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (dd[k] != 0.0) {
            double t0 = (nd[k] - oo[k]) * ii[k], t1 = (nd[3 + k] - oo[k]) * ii[k];
            if (t0 > t1) {
                const double x = t0;
                t0 = t1;
                t1 = x;
            }
            lo = fmax(lo, t0);  // fmax/fmin drop a NaN operand: a NaN axis does not cull
            hi = fmin(hi, t1);
        } else if (oo[k] < nd[k] || oo[k] > nd[3 + k]) {
            return false;
        }
    }
    tn = lo;
    return !(hi < 0.0) && !(lo > hi + 1e-12 * fabs(hi));
}
__device__ __forceinline__ bool bvh_box(const double* nd, d3 o, d3 d, d3 inv, double& tn) {
    return bvh_box_v(mk(nd[0], nd[1], nd[2]), mk(nd[3], nd[4], nd[5]), o, d, inv, tn);
}

// The triangles' part of IntersectClosest over the BVH.  The reference tests triangles in index
// order and replaces the running hit only when strictly closer, so among triangles it returns
// the smallest t, and among equal smallest t the lowest index; the traversal keeps exactly that
// (t, index) minimum, and a node is skipped only when its entry bound exceeds the current best
// t by a 1e-9 margin (so a tie can never be skipped).  The merge with the sphere/plane result is
// the reference's strict '<'.
__device__ __forceinline__ void bvh_triangles(const double* tri, const double* bvh,
                                              const int32_t* order, d3 o, d3 d, bool& found,
                                              double& best, int& kind, int& idx) {
    const d3 inv = mk(d.x != 0.0 ? 1.0 / d.x : 0.0, d.y != 0.0 ? 1.0 / d.y : 0.0,
                      d.z != 0.0 ? 1.0 / d.z : 0.0);
    bool tf = false;
    double tb = 0.0;
    int ti = 0;
    int stk[kBvhStack];
    int sp = 0;
    double tn;
    if (bvh_box(bvh, o, d, inv, tn)) stk[sp++] = 0;
    while (sp > 0) {
        const double* nd = bvh + kBvhNodeStride * stk[--sp];
        const int first = __double2loint(nd[6]), count = __double2hiint(nd[6]);
        if (count > 0) {
            for (int j = first; j < first + count; ++j) {
                const int i = order[j];
                double t;
                if (tri_hit(tri, i, o, d, t) && (!tf || t < tb || (t == tb && i < ti))) {
                    tf = true;
                    tb = t;
                    ti = i;
                }
            }
            continue;
        }
        const double bound = tf ? (found ? fmin(tb, best) : tb) : (found ? best : INFINITY);
        const double lim = bound * (1.0 + 1e-9);
        double t0, t1;
        const bool h0 = bvh_box(bvh + kBvhNodeStride * first, o, d, inv, t0) && !(t0 > lim);
        const bool h1 = bvh_box(bvh + kBvhNodeStride * (first + 1), o, d, inv, t1) && !(t1 > lim);
        if (h0 && h1) {  // nearer child on top
            const bool near0 = !(t1 < t0);
            stk[sp++] = near0 ? first + 1 : first;
            stk[sp++] = near0 ? first : first + 1;
        } else if (h0) {
            stk[sp++] = first;
        } else if (h1) {
            stk[sp++] = first + 1;
        }
    }
    if (tf && (!found || tb < best)) {
        found = true;
        best = tb;
        kind = 3;
        idx = ti;
    }
}

// Scene::IntersectClosest: spheres, then planes, then triangles; a later candidate replaces
// the current one only when strictly closer (HitInfo::isCloserThan, Shape.h:36).
// MASKED: only the spheres of `mask` (a wave-uniform set of spheres 0..63 that contains every
// sphere the ray can hit, wf_shadow_mask), visited in ascending index order as the full loop
// visits them, so ties resolve alike.
template <bool MASKED>
__device__ __forceinline__ bool closest_t(const SceneView& S, d3 o, d3 d, Hit& h, uint64_t mask) {
    bool found = false;
    double best = 0.0;
    int kind = 0, idx = -1;
    const double a = dot(d, d);       // Shape.h:75 (same value for every sphere)
    const double two_a = 2.0 * a;     // Shape.h:85-86 denominator
    const double four_a = 4.0 * a;    // Shape.h:79: (4.0 * a) * c
    for (int j = 0; MASKED ? mask != 0ull : j < S.ns; ++j) {
        int i = j;
        if constexpr (MASKED) {
            i = __builtin_ctzll(mask);
            mask &= mask - 1ull;
        }
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
#ifndef RT_LEAN_GENERIC  // the lean build (rt_trace_lean.hip) serves scenes without triangles
    if (S.bvh) {
        bvh_triangles(S.tri, S.bvh, S.bvh_tri, o, d, found, best, kind, idx);
    } else {
        for (int i = 0; i < S.nt; ++i) {
            double t;
            if (tri_hit(S.tri, i, o, d, t) && (!found || t < best)) {
                found = true;
                best = t;
                kind = 3;
                idx = i;
            }
        }
    }
#endif
    h.t = best;
    h.kind = kind;
    h.idx = idx;
    return found;
}
__device__ __forceinline__ bool closest(const SceneView& S, d3 o, d3 d, Hit& h) {
    return closest_t<false>(S, o, d, h, 0ull);
}

// Image row of the launch's row-local row yl (contiguous, or block-cyclic for multi-GPU).
__device__ __forceinline__ uint32_t image_row(const TraceParams& P, uint32_t yl) {
    if (P.row_block == 0) return P.row0 + yl;
    return P.row0 + (yl / P.row_block) * P.row_stride + yl % P.row_block;
}

// SceneView over the launch's scene; with LDS, sphere/plane/light records are staged into
// `smem` by the whole workgroup first (every thread of the block must call this).
template <bool LDS>
__device__ __forceinline__ SceneView stage_scene(const TraceParams& P, double* smem, int tid,
                                                 int nthr) {
    SceneView S;
    S.ns = P.ns;
    S.np = P.np;
    S.nt = P.nt;
    S.nl = P.nl;
    S.al = P.al_samples;
    S.spec = true;
    S.tri = P.tri;
    S.sph_mat = P.sph_mat;
    S.pl_mat = P.pl_mat;
    S.tri_mat = P.tri_mat;
    S.bvh = P.bvh;
    S.bvh_tri = P.bvh_tri;
    if constexpr (LDS) {
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
    return S;
}

// GeneratePixelAt's result for row-local pixel offset `o`: float64 / float32 framebuffers and
// the tonemapped bytes (Scene.h:298-300, RaytracingEngine.cpp:113-121).
__device__ __forceinline__ void store_pixel(const TraceParams& P, size_t o, d3 v) {
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

// Camera::getRay (Math.h:99-121) for pixel (x, y) and AA sample s; sample 0 is never jittered.
__device__ __forceinline__ d3 camera_dir(const TraceParams& P, d3 cam, uint32_t x, uint32_t y,
                                         uint64_t pix, int s) {
    double sx = static_cast<double>(x) - static_cast<double>(P.width) / 2.0;
    double sy = static_cast<double>(P.height) / 2.0 - static_cast<double>(y);
    double jx = 0.0, jy = 0.0;
    if (s > 0 && P.aa > 1) {
        jx = u01(P.seed, pix, static_cast<uint32_t>(s), 0u);
        jy = u01(P.seed, pix, static_cast<uint32_t>(s), 1u);
    }
    sx += jx;
    sy += jy;
    return unit(mk(sx, sy, cam.z + P.focal) - cam);
}

__device__ __forceinline__ const double* material_of(const SceneView& S, const Hit& h) {
    // sph_mat heads the material table [spheres | planes | triangles]
    const int base = h.kind == 1 ? 0 : (h.kind == 2 ? S.ns : S.ns + S.np);
    return S.sph_mat + kMatStride * (base + h.idx);
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

// Scene::computeTransmittance (Scene.h:35-77): closest-hit march of up to 64 steps.  MASKED:
// over the spheres of a shadow packet's capsule mask (wf_shadow_mask) — every sphere the march
// can meet before the light is in it, and one it cannot meet only decides a step whose
// closest hit lies beyond the light, where the march stops either way.
template <bool MASKED>
__device__ __forceinline__ double transmittance_t(const SceneView& S, d3 o, d3 d, double max_dist,
                                                  double bias, uint64_t mask) {
    double T = 1.0, traveled = 0.0;
    int safety = 64;
    while (safety-- > 0 && T > 1e-4 && traveled < max_dist) {
        Hit h;
        if (!closest_t<MASKED>(S, o, d, h, mask)) break;
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
__device__ __forceinline__ double transmittance(const SceneView& S, d3 o, d3 d, double max_dist,
                                                double bias) {
    return transmittance_t<false>(S, o, d, max_dist, bias, 0ull);
}

// ------------------------------------------------------------------ shadow packets (direct pass)
// The sphere mask of a wave's shadow rays towards one point light (the breadth-first renderer's
// direct pass, rt_wavefront.hip; every lane calls it): the origins of the casting lanes lie in a
// ball around the first one's origin (radius = the wave maximum of the FP32 distances, rounded
// up), every ray runs from its origin towards the light point within the bias offset of its
// segment (directLightning takes the direction from the hit point, the origin from P + n·bias),
// so each ray of the march stays in the capsule of radius R + bias around [c, light].  Lane k
// keeps sphere k unless its FP32 distance to that capsule clears the inflated radius by more than
// the rounding slack (the packet kernel's cull_capsule test: 1e-4 relative radius margin, 2e-5
// slack of the magnitudes, spheres with |C − c|/r > 1e5 always kept, NaN keeps).  Scenes with
// more than 64 spheres, non-finite origins or radius: every sphere.
constexpr float kShSlack = 2e-5f;
constexpr float kShRel = 1e-4f;
constexpr float kShFar = 1e5f;
__device__ __forceinline__ float sh_f32_up(double v) {
    return static_cast<float>(v) * (1.0f + 1e-6f);
}
__device__ __forceinline__ uint64_t wf_shadow_mask(const SceneView& S, bool casting, d3 so, d3 lpos,
                                                   double bias) {
    const uint64_t all = S.ns >= 64 ? ~0ull : ((1ull << S.ns) - 1ull);
    const uint64_t cast = __ballot(casting);
    if (!cast || S.ns > 64) return all;
    const bool bad = casting && !(isfinite(so.x) && isfinite(so.y) && isfinite(so.z));
    const d3 c = lane_d3(so, __builtin_ctzll(cast));
    float r_lane = 0.0f;
    if (casting) {  // |so − c| in FP32, rounded up (FP64 differences, 5e-7 relative error)
        const float dx = static_cast<float>(so.x - c.x), dy = static_cast<float>(so.y - c.y),
                    dz = static_cast<float>(so.z - c.z);
        r_lane = __builtin_amdgcn_sqrtf(dx * dx + dy * dy + dz * dz) * (1.0f + 1e-5f);
    }
    const float R = wave_red<1>(r_lane);
    if (__ballot(bad) || !isfinite(R) || !isfinite(lpos.x) || !isfinite(lpos.y) ||
        !isfinite(lpos.z))
        return all;
    const float sx = static_cast<float>(lpos.x - c.x), sy = static_cast<float>(lpos.y - c.y),
                sz = static_cast<float>(lpos.z - c.z);
    const float sl2 = sx * sx + sy * sy + sz * sz;
    const float inv_sl2 = 1.0f / sl2;  // only read when sl2 > 0
    const float Rc = R + sh_f32_up(fabs(bias)) * 1.001f;  // |n| ≤ 1 + 2ε
    const int k = static_cast<int>(threadIdx.x & 63u);
    bool keep = false;
    if (k < S.ns) {
        const double* s = S.sph + kSphStride * k;
        const float r = sh_f32_up(sqrt(s[3]));
        const float vx = static_cast<float>(s[0] - c.x), vy = static_cast<float>(s[1] - c.y),
                    vz = static_cast<float>(s[2] - c.z);
        const float vs = vx * sx + vy * sy + vz * sz;
        const float vv = vx * vx + vy * vy + vz * vz;
        float d2;
        if (!(vs > 0.0f) || !(sl2 > 0.0f)) {
            d2 = vv;
        } else if (!(vs < sl2)) {
            const float wx = vx - sx, wy = vy - sy, wz = vz - sz;
            d2 = wx * wx + wy * wy + wz * wz;
        } else {
            d2 = vv - (vs * vs) * inv_sl2;
        }
        const float lim = (r + Rc) * (1.0f + kShRel);
        const float far = kShFar * r - Rc;
        keep = !(d2 > lim * lim + kShSlack * (vv + sl2)) || !(far > 0.0f) || !(vv <= far * far);
    }
    return __ballot(keep);
}

// computeTransmittance for scenes without transparency (the direct and chain paths: any
// transparent material selects the tree path), where it can only return 1 or 0 and is decided
// by its first closest hit t* (blocked iff bias < t* < maxDist).  Each sphere is classified with
// the reference's FP64 discriminant, a FP32 square root and one shared reciprocal of 2a under an
// explicit error bound Δ of the roots; planes by comparing num with x·denom (1e-9 relative
// margin) instead of dividing.  Any root within Δ of a threshold (1e-6, bias, maxDist), any near
// hit, triangles, or values outside the fast ranges return -1 and the exact march runs.
// Same classification as the packet kernel's pk_occlusion (rt_packet.hip), over every sphere.
__device__ __forceinline__ int occlusion_opaque(const SceneView& S, d3 o, d3 d, double max_dist,
                                                double bias) {
    if (S.nt > 0) return -1;
    const double a = dot(d, d);
    const double two_a = 2.0 * a, four_a = 4.0 * a;
    if (!(two_a >= 0x1p-100 && two_a <= 0x1p100)) return -1;
    const double inv2a = rcp_refined(two_a);  // within 1 ulp of 1/2a: far inside the Δ margin
    // The march's zero step (round 6): an origin lying exactly on a plane gives that plane t = ±0,
    // accepted (t >= 0, Shape.h:154) and closer than any other primitive (spheres need t >= 1e-6),
    // so computeTransmittance's first step only moves the origin by bias with traveled = bias
    // (Scene.h:51-55), whatever the other candidates are.  The lane classifies again from
    // origin + direction·bias against maxDist − bias: the margins below are far above the rounding
    // difference between traveled + t >= maxDist and t >= maxDist − bias for every t they decide
    // (t > bias); the march ends first when traveled = bias >= maxDist (clear).  A second zero
    // step is left to the march.  (C2's undecided lanes are all of this kind — the floor hits of
    // the row where the floor meets the back wall — and packet_fixup_kernel renders them with
    // this function: one classification pass instead of the march's two exact closest hits.)
    for (int step = 0;; ++step) {
        bool blocked = false, undecided = false, zero = false;
        for (int i = 0; i < S.ns; ++i) {
            const double* s = S.sph + kSphStride * i;
            const d3 oc = o - mk(s[0], s[1], s[2]);
            const double b = 2.0 * dot(oc, d);
            const double cc = dot(oc, oc) - s[3];
            const double disc = b * b - four_a * cc;
            if (disc < 0.0) continue;  // miss, exactly as the reference decides it
            if (!(disc == 0.0 || (disc > 1e-30 && disc < 1e30))) {
                undecided = true;
                continue;
            }
            // |sq − fl(√disc)| ≤ 5e-7·√disc, so both roots are within Δ of the reference's
            const double sq = static_cast<double>(__builtin_amdgcn_sqrtf(static_cast<float>(disc)));  // ≤ 1 ulp
            const double delta = 2e-6 * (fabs(b) + sq) * inv2a;
            double t = (-b - sq) * inv2a;
            if (!(t >= 1e-6 + delta)) {
                if (!(t < 1e-6 - delta)) {
                    undecided = true;
                    continue;
                }
                t = (-b + sq) * inv2a;
                if (t < 1e-6 - delta) continue;
                if (!(t >= 1e-6 + delta)) {
                    undecided = true;
                    continue;
                }
            }
            if (t >= max_dist + delta) continue;
            if (t > bias + delta && t < max_dist - delta) blocked = true;
            else undecided = true;
        }
        for (int i = 0; i < S.np; ++i) {
            const double* p = S.pl + kPlStride * i;
            const d3 n = mk(p[3], p[4], p[5]);
            const double denom = dot(n, d);
            if (!(fabs(denom) > 1e-6)) continue;
            const double num = dot(mk(p[0], p[1], p[2]) - o, n);
            if (num == 0.0) {  // t = ±0: the zero step above
                zero = true;
                break;
            }
            const double A = denom > 0.0 ? num : -num, B = fabs(denom);
            if (A < -1e-300 * B) continue;
            if (A >= max_dist * B * (1.0 + 1e-9)) continue;
            if (A > bias * B * (1.0 + 1e-9) && A < max_dist * B * (1.0 - 1e-9)) blocked = true;
            else undecided = true;
        }
        if (!zero) return undecided ? -1 : (blocked ? 0 : 1);
        if (step > 0) return -1;           // a second zero step: the exact march
        if (!(bias < max_dist)) return 1;  // traveled = 0 + bias >= maxDist: T = 1 (Scene.h:42)
        o = o + d * bias;                  // r.origin + r.direction * (bias) (Scene.h:52)
        max_dist = max_dist - bias;
    }
}

struct Mat {
    d3 color;
    double shininess, specular, transparency, ior;
};

__device__ __forceinline__ Mat load_mat(const double* m) {
    return Mat{mk(m[0], m[1], m[2]), m[3], m[4], m[5], m[6]};
}

// One iteration of directLightning's light loop (Scene.h:86-124).  E = color*intensity.
template <bool COUNT, bool OPQ>
__device__ __forceinline__ void light_term(const SceneView& S, d3 P, d3 n, d3 view, const double* m,
                                           d3 lpos, d3 E, double bias, d3& diff, d3& spec,
                                           Counts& cnt) {
    double dist, inv_d2;
    d3 L;
    light_dir(lpos - P, dist, L, inv_d2);
    if (dist <= 0.0) return;
    const double ndl = smax(0.0, dot(n, L));
    if (ndl <= 0.0) return;
    if (dist <= bias) return;
    if (COUNT) cnt.shadow++;
    double T;
    if constexpr (OPQ) {
        const int occ = occlusion_opaque(S, P + n * bias, L, dist - bias, bias);
        T = occ >= 0 ? static_cast<double>(occ) : transmittance(S, P + n * bias, L, dist - bias, bias);
    } else {
        T = transmittance(S, P + n * bias, L, dist - bias, bias);
    }
    if (T <= bias) return;
    diff = diff + ((E * inv_d2) * ndl) * T;
    if (S.spec && m[5] <= 0.0 && m[4] > 0.0) {  // transparency, specular
        const d3 H = unit(L + view);
        const double ndh = smax(0.0, dot(n, H));
        if (ndh > 0.0) {
            const double sf = pow_bp(ndh, m[3]);  // shininess
            spec = spec + ((E * inv_d2) * sf) * T;
        }
    }
}

// light_term for a whole wave (every lane calls it, `active` lanes shade): the shadow rays of the
// wave's casting lanes share one capsule mask (wf_shadow_mask) and each march runs over it
// (transmittance_t<true>) — the same steps, hits and T as light_term's march.
template <bool COUNT>
__device__ __forceinline__ void light_term_wave(const SceneView& S, bool active, d3 P, d3 n,
                                                d3 view, const double* m, d3 lpos, d3 E,
                                                double bias, d3& diff, d3& spec, Counts& cnt) {
    double dist = 0.0, inv_d2 = 0.0;
    d3 L = mk(0.0, 0.0, 0.0);
    if (active) light_dir(lpos - P, dist, L, inv_d2);
    bool need = active && !(dist <= 0.0);
    double ndl = 0.0;
    if (need) {
        ndl = smax(0.0, dot(n, L));
        need = !(ndl <= 0.0) && !(dist <= bias);
    }
    const d3 so = P + n * bias;
    const uint64_t mask = wf_shadow_mask(S, need, so, lpos, bias);
    if (!need) return;
    if (COUNT) cnt.shadow++;
    const double T = S.ns > 64 ? transmittance_t<false>(S, so, L, dist - bias, bias, 0ull)
                               : transmittance_t<true>(S, so, L, dist - bias, bias, mask);
    if (T <= bias) return;
    diff = diff + ((E * inv_d2) * ndl) * T;
    if (S.spec && m[5] <= 0.0 && m[4] > 0.0) {  // transparency, specular
        const d3 H = unit(L + view);
        const double ndh = smax(0.0, dot(n, H));
        if (ndh > 0.0) {
            const double sf = pow_bp(ndh, m[3]);  // shininess
            spec = spec + ((E * inv_d2) * sf) * T;
        }
    }
}

// Scene::directLightning (Scene.h:79-129), plus the build-defined area-light samples.
template <bool COUNT, bool OPQ>
__device__ __forceinline__ d3 direct(const SceneView& S, const TraceParams& P, d3 hp, d3 view,
                                     d3 n_in, const double* m, uint64_t pix, uint32_t sample,
                                     int depth, Counts& cnt) {
    const double bias = P.bias;
    const d3 n = unit(n_in);
    d3 diff = mk(0.0, 0.0, 0.0), spec = mk(0.0, 0.0, 0.0);
    for (int i = 0; i < S.nl; ++i) {
        const double* l = S.lt + kLtStride * i;
        light_term<COUNT, OPQ>(S, hp, n, view, m, mk(l[0], l[1], l[2]), mk(l[3], l[4], l[5]), bias,
                          diff, spec, cnt);
    }
#ifndef RT_LEAN_GENERIC  // ... and without the area light
    if (S.al > 0) {
        const uint32_t stream = 0x10000u + (sample << 6) + static_cast<uint32_t>(depth);
        const double k = static_cast<double>(P.al_k);
        const d3 corner = mk(P.al_corner[0], P.al_corner[1], P.al_corner[2]);
        const d3 eu = mk(P.al_u[0], P.al_u[1], P.al_u[2]);
        const d3 ev = mk(P.al_v[0], P.al_v[1], P.al_v[2]);
        const d3 E = mk(P.al_E[0], P.al_E[1], P.al_E[2]);
        for (int s = 0; s < S.al; ++s) {
            const double r1 = u01(P.seed, pix, stream, 2u * static_cast<uint32_t>(s));
            const double r2 = u01(P.seed, pix, stream, 2u * static_cast<uint32_t>(s) + 1u);
            const double fu = (static_cast<double>(s % P.al_k) + r1) / k;
            const double fv = (static_cast<double>(s / P.al_k) + r2) / k;
            const d3 lp = (corner + eu * fu) + ev * fv;
            light_term<COUNT, OPQ>(S, hp, n, view, m, lp, E, bias, diff, spec, cnt);
        }
    }
#endif
    return hmul(mk(m[0], m[1], m[2]), diff) + spec * m[4];
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

// `save` (the breadth-first level kernel, RT_WF_SAVE): this lane's hit point, shading normal and
// incident direction are parked in LDS (structure of arrays, stride nthr) across the light loop
// and read back for the child rays, so that their registers are free while the shadow rays run.
// shade_hit: TraceRay after its closest hit h (Scene.h:147-195).  DIRECT = false leaves out
// directLightning (its value then lacks the local term: the breadth-first renderer's deferred
// direct pass, rt_wavefront.hip, computes that term later from the same hit with DIRECT = true,
// i.e. the same instructions on the same values); the child rays do not depend on it.
// CHILDREN = false leaves out the child rays (that pass, for nodes whose children are traced).
template <bool TREE, bool COUNT, bool DIRECT = true, bool CHILDREN = true>
__device__ __forceinline__ Node shade_hit(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                          const Hit& h, uint64_t pix, uint32_t sample, int depth,
                                          Counts& cnt, double* save = nullptr, int nthr = 0) {
    Node nd;
    nd.refl = false;
    nd.refr = false;
    nd.hit = true;
    const double bias = P.bias;
    const d3 hp = o + d * h.t;  // Rayon::pointAtDistance
    const d3 gn = normal_of(S, h, hp);
    // the material record (r g b shininess specular transparency ior), read at each use: a
    // copy of all seven values stayed live across the light loop (14 VGPRs)
    const double* m = material_of(S, h);
    const d3 inc = unit(d);
    const bool front = dot(gn, inc) < 0.0;
    const d3 n = front ? gn : -gn;
    const d3 view = -inc;
    const double tr = sclamp(m[5], 0.0, 1.0);
    if (save) {
        save[0 * nthr] = hp.x;
        save[1 * nthr] = hp.y;
        save[2 * nthr] = hp.z;
        save[3 * nthr] = n.x;
        save[4 * nthr] = n.y;
        save[5 * nthr] = n.z;
        save[6 * nthr] = inc.x;
        save[7 * nthr] = inc.y;
        save[8 * nthr] = inc.z;
        __asm__ volatile("" ::: "memory");  // no forwarding of the stored values
    }
    d3 local = mk(0.0, 0.0, 0.0);
    if constexpr (DIRECT) local = direct<COUNT, !TREE>(S, P, hp, view, n, m, pix, sample, depth, cnt);
    d3 hp_c = hp, n_c = n, inc_c = inc;  // the values the child rays start from
    if (save) {
        __asm__ volatile("" ::: "memory");
        hp_c = mk(save[0 * nthr], save[1 * nthr], save[2 * nthr]);
        n_c = mk(save[3 * nthr], save[4 * nthr], save[5 * nthr]);
        inc_c = mk(save[6 * nthr], save[7 * nthr], save[8 * nthr]);
    }
    d3 fin = mk(0.0, 0.0, 0.0);
    if (DIRECT && tr < 1.0) fin = fin + local * (1.0 - tr);
    nd.value = fin;
    if constexpr (!CHILDREN) return nd;
    double refl_w = m[4];
    if (TREE && tr > 0.0) {
        // fresnel (Scene.h:26-28, 161-164); only consumed when tr > 0.
        const double cos_t = smax(0.0, dot(n_c, -inc_c));
        const double eta_t = m[6];
        const double r0 = (eta_t - 1.0) / (eta_t + 1.0);
        const double f0 = r0 * r0;  // pow(x, 2.0)
        // pow(1 - cosθ, 5) through pow_bp (rt_device.hpp: ≤ 2e-16 absolute on [0, 1], the
        // libm pow out of line outside (0, 1.5)) instead of the inlined libm pow
        double F = f0 + (1.0 - f0) * pow_bp(1.0 - cos_t, 5.0);
        const double eta = front ? (1.0 / eta_t) : (eta_t / 1.0);
        d3 rd = refract(inc_c, n_c, eta);
        if (length(rd) > bias) {
            rd = unit(rd);
            nd.refr = true;
            nd.fd = rd;
            nd.fo = hp_c + rd * (bias * 1e2);
            nd.fw = tr * (1.0 - F);
        } else {
            F = 1.0;
        }
        refl_w = F;
    }
    if (refl_w > bias) {
        const d3 R = unit(reflect(inc_c, n_c));
        nd.refl = true;
        nd.rd = R;
        nd.ro = hp_c + R * bias;
        nd.rw = refl_w;
    }
    return nd;
}

template <bool TREE, bool COUNT>
__device__ __forceinline__ Node shade(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                      uint64_t pix, uint32_t sample, int depth, Counts& cnt,
                                      double* save = nullptr, int nthr = 0) {
    if (COUNT) cnt.trace++;
    Hit h;
    if (!closest(S, o, d, h)) {
        Node nd;
        nd.refl = false;
        nd.refr = false;
        nd.hit = false;
        nd.value = sky(d);
        return nd;
    }
    return shade_hit<TREE, COUNT>(S, P, o, d, h, pix, sample, depth, cnt, save, nthr);
}

// TraceRay for scenes where no secondary ray can be spawned.
template <bool COUNT>
__device__ __forceinline__ d3 trace_direct(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                           uint64_t pix, uint32_t sample, Counts& cnt) {
    if (P.max_rec <= 0) return sky(d);
    return shade<false, COUNT>(S, P, o, d, pix, sample, 0, cnt).value;
}

// TraceRay for opaque scenes: a linear reflection chain (Scene.h:131-198 with transparency 0).
// The reference folds it back to front, final_k = value_k + final_{k+1}·rw_k; here it is
// accumulated front to back, acc += W_k·value_k with W_{k+1} = W_k·rw_k, so no level has to wait
// on a stack (the kernel holds four doubles of chain state instead of 4·(max_recursion − 1)).
// Same sum, different rounding order: a relative difference of a few ε per level (every chain
// scene already calls libm pow, so these are held to 1e-12, not to bit equality).
template <bool COUNT>
__device__ __forceinline__ d3 trace_chain(const SceneView& S, const TraceParams& P, d3 o, d3 d,
                                          uint64_t pix, uint32_t sample, Counts& cnt) {
    d3 acc = mk(0.0, 0.0, 0.0);
    double w = 1.0;
    for (int depth = 0;; ++depth) {
        if (depth >= P.max_rec) {  // TraceRay at depth maxRecursion: the sky (Scene.h:132-134)
            acc = acc + sky(d) * w;
            break;
        }
        const Node nd = shade<false, COUNT>(S, P, o, d, pix, sample, depth, cnt);
        acc = acc + nd.value * w;
        if (!nd.hit || !nd.refl) break;
        w = w * nd.rw;
        o = nd.ro;
        d = nd.rd;
    }
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

}  // namespace rtamd
