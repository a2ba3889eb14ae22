// rt_box.hip — reflection chains of scenes made of planes and spheres (no triangles or area
// light): the reference main()'s own scene (RaytracingEngine.cpp:255-291, BASELINE config 1 — a
// box of five axis-aligned mirrored walls lit by two point lights), any box-like room, and rooms
// with up to 64 spheres in them (the SPH instantiations: the mirror scene).
//
// Same TraceRay chain as trace_chain (rt_trace_common.hpp: Scene.h:131-198 with transparency 0,
// accumulated front to back), same shading helpers, so the image is bit-identical to the generic
// chain kernel's.  What changes is how the planes are tested:
//
//  * The planes live in a per-scene table read through the scalar cache (wave-uniform loads into
//    SGPRs), so no plane value occupies a VGPR or an LDS slot, grouped by the axis of their normal
//    (x, y, z, then the rest) so the component a group needs is known at compile time.
//  * A plane whose normal is exactly ±e_k (two zero components, the third ±1 — what the Plane
//    constructor's normalize() makes of an axis direction, Shape.h:142) has, for a ray with finite
//    origin o and direction d, num = (p − o)·n = s·(p_k − o_k) and denom = n·d = s·d_k exactly:
//    the zero terms are signed zeros that cannot change a nonzero sum.  t = num/denom is then
//    (p_k − o_k)/d_k bit for bit (IEEE division is sign-symmetric), i.e. one subtraction and a
//    division through the shared reciprocal of d_k (div_core) instead of two dot products and a
//    division.  p_k − o_k == 0 (a ray starting on the plane: t = ±0, the sign from the literal
//    sum) and values outside div_core's range take the literal expression.
//  * Shadow rays are classified (blocked / clear / undecided) from the same A = num·sign(denom),
//    B = |denom| as the generic occlusion_opaque, which for such a plane are sign(d_k)·(p_k − o_k)
//    and |d_k| exactly; undecided lanes run the exact computeTransmittance march.
//  * Spheres (SPH) are read through the scalar cache as well and tested first, in scene order,
//    with the reference's literal Sphere::Intersect (Shape.h:72-98) — IntersectClosest visits
//    spheres before planes (Scene.h:221-241).
// Closest-hit ties between groups keep the reference's order: the lower scene index wins
// (strict '<' in scene order, Shape.h:36 / Scene.h:233-241), every sphere before every plane.
#include "rt_trace_common.hpp"

#pragma clang fp contract(off)

namespace rtamd {

// Waves per SIMD the single-sample (AA = 1) and the multi-sample instantiations are compiled for.
#ifndef RT_BOX_WAVES
#define RT_BOX_WAVES 4
#endif
#ifndef RT_BOX_MULTI_WAVES
#define RT_BOX_MULTI_WAVES 3
#endif

// The hit's normal and incident direction wait in LDS across the light loop, for the reflection
// ray, and the SPH instantiations (mirror) also read the hit's material at each use: 112 -> 32
// B/lane of scratch at 4 waves/SIMD, mirror 1.326 -> 1.231 ms (profiles/r05_ab_box_spheres.txt;
// the hit point and shading normal parked as well: 1.239 ms).  The planes-only ones keep the
// material in registers (read at use: C1 +1.6 %, at AA = 32 +2.7 %); their park alone: C1 374 ->
// 368.5 µs.  RT_BOX_PARK=0: A/B.
#ifndef RT_BOX_PARK
#define RT_BOX_PARK 1
#endif
constexpr bool kBoxPark = RT_BOX_PARK != 0;
constexpr int kBoxParkStride = 256;  // threads per workgroup of both box kernels
constexpr int kBoxParkSlots = 6;

// wave-uniform reads through the scalar data cache
typedef const __attribute__((address_space(4))) double* cdp;

struct BoxScene {
    cdp pl;           // box table, kBoxRec doubles per plane, in group order
    const double* g;  // the same table for per-lane (vector) reads of the hit plane
    cdp lt;           // point lights (kLtStride)
    cdp sph;          // spheres (kSphStride: cx cy cz r²), SPH instantiations
    const double* sph_v;  // the same for per-lane reads of the hit sphere
    const double* mat;    // material table [spheres | planes] (per-lane reads)
    int n[4];         // planes per group: normal ±e_x, ±e_y, ±e_z, any other
    int nl, ns;
    double* park;     // kBoxPark: this thread's LDS slots (stride kBoxParkStride)
};

struct BoxHit {
    double t;
    int rec;   // the hit plane's record (group order), or −1 − i for sphere i
    int orig;  // its position in IntersectClosest's order: sphere i, then ns + plane index
};

// |o_i| ≤ 2^1000 (with the table's |p_i| ≤ 2^1000 every p_i − o_i is finite, so the shortcut's
// zero terms are signed zeros) and |d_i| ≤ 2^90 (finite; with 2^-900 ≤ |p_k − o_k| ≤ 2^900 and
// |d_k| > 1e-6 every operand is in div_core's range, rt_device.hpp: |n/d| ≥ 2^-1000).  Camera and
// reflection rays are unit vectors; NaN fails both.
__device__ __forceinline__ bool box_ray_ok(d3 o, d3 d) {
    return fabs(o.x) + fabs(o.y) + fabs(o.z) <= 0x1p1000 &&
           fabs(d.x) + fabs(d.y) + fabs(d.z) <= 0x1p90;
}

__device__ __forceinline__ double comp(d3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
// a plane record's position in IntersectClosest's order (after the spheres)
__device__ __forceinline__ int rec_orig(const BoxScene& S, cdp q) { return S.ns + __double2loint(q[15]); }

// The reference's literal Plane::Intersect quotient (Shape.h:149-159); denom checked by the caller.
__device__ __forceinline__ double plane_literal_t(cdp q, d3 o, d3 d) {
    const d3 n = mk(q[3], q[4], q[5]);
    return dot(mk(q[0], q[1], q[2]) - o, n) / dot(n, d);
}

// IntersectClosest's running minimum (Scene.h:233-241): strictly closer, or as close with a
// lower scene index (the reference visits planes in scene order and keeps the first).
__device__ __forceinline__ void box_take(double t, int rec, int orig, bool& found, BoxHit& h) {
    if (t >= 0.0 && (!found || t < h.t || (t == h.t && orig < h.orig))) {
        found = true;
        h.t = t;
        h.rec = rec;
        h.orig = orig;
    }
}

// Group K (normal ±e_K) of the closest-hit search, every lane's ray finite (box_ray_ok).
template <int K>
__device__ __forceinline__ void box_group_closest(const BoxScene& S, int first, d3 o, d3 d,
                                                  bool& found, BoxHit& h) {
    const int n = S.n[K];
    if (n == 0) return;  // uniform
    const double dk = comp(d, K), ok = comp(o, K);
    const bool live = fabs(dk) > 1e-6;  // |denom| > 1e-6 (Shape.h:151)
    const double rk = rcp_refined(dk);
    for (int j = 0; j < n; ++j) {
        cdp q = S.pl + kBoxRec * (first + j);
        const double c = q[6] - ok;  // p_k − o_k
        double t = div_core(c, dk, rk);
        const bool odd = live && !(fabs(c) >= 0x1p-900 && fabs(c) <= 0x1p900);
        if (__ballot(odd)) {  // uniform: some lane needs the literal quotient
            if (odd) t = c == 0.0 ? plane_literal_t(q, o, d) : c / dk;
        }
        if (live) box_take(t, first + j, rec_orig(S, q), found, h);
    }
}

// The reference's literal plane loop over records [first, first + n) (rays that are not finite,
// and planes of no axis).
__device__ __forceinline__ void box_literal_closest(const BoxScene& S, int first, int n, d3 o,
                                                    d3 d, bool& found, BoxHit& h) {
    for (int j = 0; j < n; ++j) {
        cdp q = S.pl + kBoxRec * (first + j);
        const d3 nn = mk(q[3], q[4], q[5]);
        const double denom = dot(nn, d);
        if (fabs(denom) > 1e-6) {
            const double t = dot(mk(q[0], q[1], q[2]) - o, nn) / denom;
            box_take(t, first + j, rec_orig(S, q), found, h);
        }
    }
}

// IntersectClosest's sphere loop (Scene.h:221-232; Sphere::Intersect Shape.h:72-98, literal),
// sphere records through the scalar cache.  (The packet kernel's exact root forms — sqrt /
// division cores with a shared reciprocal of 2a, lazy far root, no-win skip — were 2 % slower
// here: mirror 1.352 vs 1.325 ms, profiles/r05_ab_box_spheres.txt.)
__device__ __forceinline__ void box_spheres_closest(const BoxScene& S, d3 o, d3 d, bool& found,
                                                    BoxHit& h) {
    const double a = dot(d, d);       // Shape.h:75 (same value for every sphere)
    const double two_a = 2.0 * a;     // Shape.h:85-86 denominator
    const double four_a = 4.0 * a;    // Shape.h:79: (4.0 * a) * c
#pragma unroll 2  // mirror 1.227 -> 1.222 ms, at AA = 4 4.607 -> 4.572 ms
    for (int i = 0; i < S.ns; ++i) {
        cdp s = S.sph + kSphStride * i;
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
        if (!found || t < h.t) {
            found = true;
            h.t = t;
            h.rec = -1 - i;
            h.orig = i;
        }
    }
}

// Scene::IntersectClosest (Scene.h:218-257): the spheres (SPH), then the planes (Plane::Intersect
// Shape.h:149-159).
template <bool SPH>
__device__ __forceinline__ bool box_closest(const BoxScene& S, d3 o, d3 d, BoxHit& h) {
    bool found = false;
    h.t = 0.0;
    h.rec = 0;
    h.orig = 0;
    if constexpr (SPH) box_spheres_closest(S, o, d, found, h);
    const int g1 = S.n[0], g2 = g1 + S.n[1], g3 = g2 + S.n[2];
    if (__ballot(!box_ray_ok(o, d)) == 0) {  // uniform
        box_group_closest<0>(S, 0, o, d, found, h);
        box_group_closest<1>(S, g1, o, d, found, h);
        box_group_closest<2>(S, g2, o, d, found, h);
    } else {
        box_literal_closest(S, 0, g3, o, d, found, h);
    }
    box_literal_closest(S, g3, S.n[3], o, d, found, h);
    return found;
}

// Shadow-ray classification of one plane from A = num·sign(denom), B = |denom| (as
// occlusion_opaque): t < 0, beyond the light, blocking, or undecided (near a threshold).
__device__ __forceinline__ void box_classify(double A, double B, double max_dist, double bias,
                                             bool& blocked, bool& undecided) {
    if (A < -1e-300 * B) return;
    if (A >= max_dist * B * (1.0 + 1e-9)) return;
    if (A > bias * B * (1.0 + 1e-9) && A < max_dist * B * (1.0 - 1e-9)) blocked = true;
    else undecided = true;
}

template <int K>
__device__ __forceinline__ void box_group_occlusion(const BoxScene& S, int first, d3 o, d3 d,
                                                    double max_dist, double bias, bool& blocked,
                                                    bool& undecided) {
    const int n = S.n[K];
    if (n == 0) return;  // uniform
    const double dk = comp(d, K), ok = comp(o, K);
    const double B = fabs(dk);
    if (!(B > 1e-6)) return;  // |denom| ≤ 1e-6: no plane of the group can be hit
    for (int j = 0; j < n; ++j) {
        cdp q = S.pl + kBoxRec * (first + j);
        const double c = q[6] - ok;
        box_classify(dk > 0.0 ? c : -c, B, max_dist, bias, blocked, undecided);
    }
}

__device__ __forceinline__ void box_literal_occlusion(const BoxScene& S, int first, int n, d3 o,
                                                      d3 d, double max_dist, double bias,
                                                      bool& blocked, bool& undecided) {
    for (int j = 0; j < n; ++j) {
        cdp q = S.pl + kBoxRec * (first + j);
        const d3 nn = mk(q[3], q[4], q[5]);
        const double denom = dot(nn, d);
        if (!(fabs(denom) > 1e-6)) continue;
        const double num = dot(mk(q[0], q[1], q[2]) - o, nn);
        box_classify(denom > 0.0 ? num : -num, fabs(denom), max_dist, bias, blocked, undecided);
    }
}

// The spheres' part of occlusion_opaque (rt_trace_common.hpp): hit / miss by the reference's FP64
// discriminant, the roots within an explicit error bound from a FP32 square root and one shared
// reciprocal of 2a; anything near a threshold is undecided.
__device__ __forceinline__ void box_spheres_occlusion(const BoxScene& S, d3 o, d3 d,
                                                      double max_dist, double bias, bool& blocked,
                                                      bool& undecided) {
    const double a = dot(d, d);
    const double two_a = 2.0 * a, four_a = 4.0 * a;
    if (!(two_a >= 0x1p-100 && two_a <= 0x1p100)) {
        undecided = true;
        return;
    }
    const double inv2a = rcp_refined(two_a);  // within 1 ulp of 1/2a: far inside the Δ margin
    for (int i = 0; i < S.ns; ++i) {
        cdp s = S.sph + kSphStride * i;
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
        const double sq = static_cast<double>(__builtin_amdgcn_sqrtf(static_cast<float>(disc)));
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
}

// computeTransmittance (Scene.h:35-77) of an opaque scene of planes (and spheres): 1 clear, 0
// blocked, -1 undecided (the exact march decides).
template <bool SPH>
__device__ __forceinline__ int box_occlusion(const BoxScene& S, d3 o, d3 d, double max_dist,
                                             double bias) {
    bool blocked = false, undecided = false;
    if constexpr (SPH) box_spheres_occlusion(S, o, d, max_dist, bias, blocked, undecided);
    const int g1 = S.n[0], g2 = g1 + S.n[1], g3 = g2 + S.n[2];
    if (__ballot(!box_ray_ok(o, d)) == 0) {  // uniform
        box_group_occlusion<0>(S, 0, o, d, max_dist, bias, blocked, undecided);
        box_group_occlusion<1>(S, g1, o, d, max_dist, bias, blocked, undecided);
        box_group_occlusion<2>(S, g2, o, d, max_dist, bias, blocked, undecided);
    } else {
        box_literal_occlusion(S, 0, g3, o, d, max_dist, bias, blocked, undecided);
    }
    box_literal_occlusion(S, g3, S.n[3], o, d, max_dist, bias, blocked, undecided);
    return undecided ? -1 : (blocked ? 0 : 1);
}

// The hit's material record (r g b shininess specular transparency ior).
__device__ __forceinline__ const double* box_material(const BoxScene& S, const BoxHit& h) {
    return h.rec < 0 ? S.mat + kMatStride * (-1 - h.rec) : S.g + kBoxRec * h.rec + 8;
}

// The exact march (transmittance(), rt_trace_common.hpp).
template <bool SPH>
__device__ __forceinline__ double box_transmittance(const BoxScene& S, d3 o, d3 d,
                                                    double max_dist, double bias) {
    double T = 1.0, traveled = 0.0;
    int safety = 64;
    while (safety-- > 0 && T > 1e-4 && traveled < max_dist) {
        BoxHit h;
        if (!box_closest<SPH>(S, o, d, h)) break;
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
        T *= sclamp(box_material(S, h)[5], 0.0, 1.0);
        o = (o + d * t) + d * bias;
        traveled += t + bias;
    }
    return sclamp(T, 0.0, 1.0);
}

// One TraceRay level (shade<false>, rt_trace_common.hpp) for an opaque scene of planes (and
// spheres): the local light of the hit (or the sky) and the reflection ray.
template <bool COUNT, bool SPH>
__device__ __forceinline__ Node box_shade(const BoxScene& S, const TraceParams& P, d3 o, d3 d,
                                          Counts& cnt) {
    Node nd;
    nd.refl = false;
    nd.refr = false;
    if (COUNT) cnt.trace++;
    BoxHit h;
    if (!box_closest<SPH>(S, o, d, h)) {
        nd.hit = false;
        nd.value = sky(d);
        return nd;
    }
    nd.hit = true;
    const double bias = P.bias;
    const d3 hp = o + d * h.t;  // Rayon::pointAtDistance
    d3 gn;
    bool unit_n;
    if (SPH && h.rec < 0) {  // Sphere::GetNormalAt (Shape.h:100-102)
        const double* c = S.sph_v + kSphStride * (-1 - h.rec);
        gn = unit(hp - mk(c[0], c[1], c[2]));
        unit_n = false;
    } else {
        const double* r = S.g + kBoxRec * h.rec;
        gn = mk(r[3], r[4], r[5]);  // Plane::GetNormalAt (Shape.h:161-163)
        unit_n = r[7] != 0.0;       // |n| rounds to exactly 1: normalize() returns n
    }
    // the material record (r g b shininess specular transparency ior): SPH reads it at each use
    // (a copy of its seven values stayed live across the light loop: 14 VGPRs), the planes-only
    // instantiations keep the copy
    const double* mp = box_material(S, h);
    double mc[7];
    if constexpr (!SPH)
        for (int k = 0; k < 7; ++k) mc[k] = mp[k];
    auto mat = [&](int k) -> double {
        if constexpr (SPH) return mp[k];
        else return mc[k];
    };
    const d3 inc = unit(d);
    const bool front = dot(gn, inc) < 0.0;
    const d3 n0 = front ? gn : -gn;
    const d3 view = -inc;
    // directLightning (Scene.h:79-129)
    const d3 n = unit_n ? n0 : unit(n0);
    if constexpr (kBoxPark) {  // n0 and inc wait in LDS for the reflection ray
        S.park[0 * kBoxParkStride] = n0.x;
        S.park[1 * kBoxParkStride] = n0.y;
        S.park[2 * kBoxParkStride] = n0.z;
        S.park[3 * kBoxParkStride] = inc.x;
        S.park[4 * kBoxParkStride] = inc.y;
        S.park[5 * kBoxParkStride] = inc.z;
        __asm__ volatile("" ::: "memory");
    }
    d3 diff = mk(0.0, 0.0, 0.0), spec = mk(0.0, 0.0, 0.0);
    for (int i = 0; i < S.nl; ++i) {
        cdp l = S.lt + kLtStride * i;
        const d3 lpos = mk(l[0], l[1], l[2]), E = mk(l[3], l[4], l[5]);
        double dist, inv_d2;
        d3 L;
        light_dir(lpos - hp, dist, L, inv_d2);
        if (dist <= 0.0) continue;
        const double ndl = smax(0.0, dot(n, L));
        if (ndl <= 0.0) continue;
        if (dist <= bias) continue;
        if (COUNT) cnt.shadow++;
        const d3 so = hp + n * bias;
        const int occ = box_occlusion<SPH>(S, so, L, dist - bias, bias);
        const double T = occ >= 0 ? static_cast<double>(occ)
                                  : box_transmittance<SPH>(S, so, L, dist - bias, bias);
        if (T <= bias) continue;
        diff = diff + ((E * inv_d2) * ndl) * T;
        if (mat(5) <= 0.0 && mat(4) > 0.0) {
            d3 vw = view;
            if constexpr (kBoxPark)
                vw = -mk(S.park[3 * kBoxParkStride], S.park[4 * kBoxParkStride],
                         S.park[5 * kBoxParkStride]);
            const d3 H = unit(L + vw);
            const double ndh = smax(0.0, dot(n, H));
            if (ndh > 0.0) {
                const double sf = pow_bp_t<true>(ndh, mat(3));
                spec = spec + ((E * inv_d2) * sf) * T;
            }
        }
    }
    const d3 local = hmul(mk(mat(0), mat(1), mat(2)), diff) + spec * mat(4);
    const double tr = sclamp(mat(5), 0.0, 1.0);
    d3 fin = mk(0.0, 0.0, 0.0);
    if (tr < 1.0) fin = fin + local * (1.0 - tr);
    nd.value = fin;
    if (mat(4) > bias) {
        d3 inc_c = inc, n0_c = n0;
        if constexpr (kBoxPark) {
            __asm__ volatile("" ::: "memory");
            n0_c = mk(S.park[0 * kBoxParkStride], S.park[1 * kBoxParkStride],
                      S.park[2 * kBoxParkStride]);
            inc_c = mk(S.park[3 * kBoxParkStride], S.park[4 * kBoxParkStride],
                       S.park[5 * kBoxParkStride]);
        }
        const d3 R = unit(reflect(inc_c, n0_c));
        nd.refl = true;
        nd.rd = R;
        nd.ro = hp + R * bias;
        nd.rw = mat(4);
    }
    return nd;
}

// One sample of GeneratePixelAt (Scene.h:283-304): TraceRay as a reflection chain accumulated
// front to back (trace_chain's order, so the image equals the generic chain kernel's bit for bit).
template <bool COUNT, bool SPH>
__device__ __forceinline__ d3 box_sample(const BoxScene& S, const TraceParams& P, d3 cam,
                                         uint32_t x, uint32_t y, uint64_t pix, int s, Counts& cnt) {
    d3 d = camera_dir(P, cam, x, y, pix, s);
    d3 o = cam;
    d3 c = mk(0.0, 0.0, 0.0);
    double w = 1.0;
    for (int depth = 0;; ++depth) {
        if (depth >= P.max_rec) {  // TraceRay at depth maxRecursion: the sky
            c = c + sky(d) * w;
            break;
        }
        const Node nd = box_shade<COUNT, SPH>(S, P, o, d, cnt);
        c = c + nd.value * w;
        if (!nd.hit || !nd.refl) break;
        w = w * nd.rw;
        o = nd.ro;
        d = nd.rd;
    }
    return c;
}

__device__ __forceinline__ BoxScene box_scene(const TraceParams& P) {
    BoxScene S;
    S.pl = (cdp)P.box;
    S.g = P.box;
    S.lt = (cdp)P.lt;
    S.sph = (cdp)P.sph;
    S.sph_v = P.sph;
    S.mat = P.sph_mat;
    for (int k = 0; k < 4; ++k) S.n[k] = P.box ? P.box_n[k] : 0;
    S.nl = P.nl;
    S.ns = P.ns;
    S.park = nullptr;
    return S;
}

template <bool COUNT>
__device__ __forceinline__ void box_count(const Counts& cnt, const TraceParams& P, int tid) {
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

// Multi-sample frames, sample-parallel: thread t of a 256-thread workgroup traces sample
// t mod aa of pixel t div aa (256 / aa consecutive pixels of the row-major frame per workgroup),
// so every thread runs the single-sample code at the single-sample register budget (4
// waves/SIMD, where a per-thread sample loop needs 3) and a wave's rays are the jittered
// samples of one or a few pixels — more coherent than an 8×8 pixel tile.  The colours meet in
// LDS, and one thread per pixel sums them in sample order (acc = acc + c, Scene.h:292-297) and
// divides by the sample count: the same operations in the same order as the per-thread loop.
constexpr int kBoxAaThreads = 256;
constexpr int kBoxAaMax = 128;  // larger sample counts keep the per-thread loop
template <bool COUNT, bool SPH>
__global__ __launch_bounds__(kBoxAaThreads, RT_BOX_WAVES) void box_aa_kernel(TraceParams P) {
    __shared__ double s_c[3 * kBoxAaThreads];
    const int tid = threadIdx.x;
    const int aa = P.aa;                     // 2 ≤ aa ≤ kBoxAaMax (launcher)
    const int ppw = kBoxAaThreads / aa;      // pixels per workgroup
    const int pl = tid / aa, s = tid - pl * aa;
    const uint64_t npx = static_cast<uint64_t>(P.width) * P.rows;
    const uint64_t lin = static_cast<uint64_t>(blockIdx.x) * ppw + pl;
    Counts cnt{0u, 0u};
    BoxScene S = box_scene(P);
    if constexpr (kBoxPark) {
        __shared__ double s_park[kBoxParkSlots * kBoxParkStride];
        S.park = s_park + tid;
    }
    if (pl < ppw && lin < npx) {
        const uint32_t x = static_cast<uint32_t>(lin % P.width);
        const uint32_t y = image_row(P, static_cast<uint32_t>(lin / P.width));
        const uint64_t pix = static_cast<uint64_t>(y) * P.width + x;
        const d3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
        const d3 c = box_sample<COUNT, SPH>(S, P, cam, x, y, pix, s, cnt);
        s_c[tid] = c.x;
        s_c[kBoxAaThreads + tid] = c.y;
        s_c[2 * kBoxAaThreads + tid] = c.z;
    }
    __syncthreads();
    const uint64_t out = static_cast<uint64_t>(blockIdx.x) * ppw + tid;
    if (tid < ppw && out < npx) {
        d3 acc = mk(0.0, 0.0, 0.0);
        for (int k = 0; k < aa; ++k) {
            const int j = tid * aa + k;
            acc = acc + mk(s_c[j], s_c[kBoxAaThreads + j], s_c[2 * kBoxAaThreads + j]);
        }
        store_pixel(P, static_cast<size_t>(out), sdiv(acc, static_cast<double>(aa)));
    }
    if constexpr (COUNT) box_count<COUNT>(cnt, P, tid);
}

// GeneratePixelAt (Scene.h:283-304) with a per-thread sample loop: single-sample frames, and
// sample counts of 0 or above kBoxAaMax.
template <bool COUNT, bool SINGLE, bool SPH>
__global__ __launch_bounds__(kTileW * kTileH, SINGLE ? RT_BOX_WAVES : RT_BOX_MULTI_WAVES) void box_chain_kernel(TraceParams P) {
    const uint32_t x = blockIdx.x * kTileW + threadIdx.x;
    const uint32_t yl = blockIdx.y * kTileH + threadIdx.y;
    Counts cnt{0u, 0u};
    BoxScene S = box_scene(P);
    if constexpr (kBoxPark) {
        __shared__ double s_park[kBoxParkSlots * kBoxParkStride];
        S.park = s_park + threadIdx.y * kTileW + threadIdx.x;
    }
    if (x < P.width && yl < P.rows) {
        const uint32_t y = image_row(P, yl);
        const uint64_t pix = static_cast<uint64_t>(y) * P.width + x;
        const d3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
        d3 acc = mk(0.0, 0.0, 0.0);
        int samples = 0;
        const int nsamples = SINGLE ? 1 : P.aa;
        for (int s = 0; s < nsamples; ++s) {
            acc = acc + box_sample<COUNT, SPH>(S, P, cam, x, y, pix, s, cnt);
            samples += 1;
        }
        const d3 v = samples > 0 ? sdiv(acc, static_cast<double>(samples)) : mk(0.0, 0.0, 0.0);
        store_pixel(P, static_cast<size_t>(yl) * P.width + x, v);
    }
    if constexpr (COUNT) box_count<COUNT>(cnt, P, threadIdx.y * kTileW + threadIdx.x);
}

template <bool SPH>
static hipError_t launch_box(const TraceParams& p, bool count, bool sample_parallel,
                             hipStream_t stream) {
    if (sample_parallel && p.aa >= 2 && p.aa <= kBoxAaMax) {
        const int ppw = kBoxAaThreads / p.aa;
        const uint64_t npx = static_cast<uint64_t>(p.width) * p.rows;
        const dim3 grid(static_cast<unsigned>((npx + ppw - 1) / ppw));
        if (count) hipLaunchKernelGGL((box_aa_kernel<true, SPH>), grid, dim3(kBoxAaThreads), 0, stream, p);
        else hipLaunchKernelGGL((box_aa_kernel<false, SPH>), grid, dim3(kBoxAaThreads), 0, stream, p);
        return hipGetLastError();
    }
    const dim3 block(kTileW, kTileH);
    const dim3 grid((p.width + kTileW - 1) / kTileW, (p.rows + kTileH - 1) / kTileH);
    if (count) {
        if (p.aa == 1) hipLaunchKernelGGL((box_chain_kernel<true, true, SPH>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((box_chain_kernel<true, false, SPH>), grid, block, 0, stream, p);
    } else {
        if (p.aa == 1) hipLaunchKernelGGL((box_chain_kernel<false, true, SPH>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((box_chain_kernel<false, false, SPH>), grid, block, 0, stream, p);
    }
    return hipGetLastError();
}

hipError_t launch_box_chain(const TraceParams& p, bool count, bool sample_parallel,
                            hipStream_t stream) {
    if (p.nt != 0 || p.al_samples != 0 || p.ns > kBoxMaxSpheres || (p.np > 0 && !p.box))
        return hipErrorInvalidValue;  // the launcher's conditions (rt_capi.cpp)
    return p.ns > 0 ? launch_box<true>(p, count, sample_parallel, stream)
                    : launch_box<false>(p, count, sample_parallel, stream);
}

}  // namespace rtamd
