// rt_packet.hip — packet-culled FP64 trace kernel for scenes whose materials spawn no secondary
// rays (every BASELINE synthetic config C2–C5): camera ray + shadow rays per pixel.
//
// Same per-ray arithmetic as the generic kernel (rt_trace_common.hpp), so results stay
// bit-identical to the reference; what changes is WHICH primitives a ray is tested against
// and which divisions are skipped because their outcome is already decided:
//
//  * One wave = an 8×8 pixel tile.  Before each closest-hit search the wave bounds its rays —
//    a direction cone around the camera for camera rays, a capsule from the ball of shadow-ray
//    origins to the light for shadow rays — and each lane tests one sphere against that bound
//    (ballot → a 64-bit candidate mask per 64 spheres, held in SGPRs).  The bounds are reduced
//    across the wave in FP32 with directed rounding (DPP row steps + readlane), so they only
//    ever grow.
//  * The per-sphere test is conservative with a 1e-4 relative radius margin: a sphere outside
//    the bound has, for every ray of the packet, an exact discriminant < 0 by far more than
//    FP64 rounding can flip, so it can never be hit.  Spheres whose |oc|/r exceeds 1e5 (where
//    that argument would need a larger margin) are always kept.  Candidates are visited in
//    ascending index order, so strict-'<' tie-breaking (Shape.h:36) is unchanged.
//  * Camera rays share their origin: oc = cam − C, c = oc·oc − r² (Shape.h:73-77) and each
//    plane's (p − cam)·n (Shape.h:152-153) are the same doubles for every camera ray and are
//    formed once per workgroup into LDS.
//  * A candidate's root (or plane t) is only divided out when it can still win: if
//    numerator > best·denominator·(1+2⁻⁴⁰) the rounded quotient is provably ≥ best and the
//    strict '<' would reject it anyway.  The far root is only formed when the near root is
//    below the 1e-6 epsilon (t0 ≤ t1 holds exactly for 2a > 0, so the reference's swap never
//    fires).
//  * Shadow-ray marches (computeTransmittance, Scene.h:35-77) only move the origin along the
//    segment towards the light, so one capsule mask serves the whole march.
#include <cstdlib>

#include "rt_trace_common.hpp"

#pragma clang fp contract(off)

namespace rtamd {

constexpr int kPkW = 8;             // pixels per wave, x
constexpr int kPkH = 8;             // pixels per wave, y
#ifndef RT_PK_WAVES_X
#define RT_PK_WAVES_X 2
#endif
constexpr int kWgWavesX = RT_PK_WAVES_X;  // waves per workgroup, x
// Waves per workgroup in y (the WGY template parameter): 1 (128 threads, 16×8 px) while ten
// workgroups' LDS images fit the CU's 160 KiB — 20 waves, the 5-waves/SIMD budget — else 2
// (256 threads, 16×16 px: five images, still 20 waves).  Smaller workgroups wait less for their
// slowest wave (C3 -3 %, C5 -2 %); with C4's 27 KiB image they would halve the occupancy.
constexpr size_t kLdsPerCu = 160 * 1024;
constexpr double kCullRel = 1e-4;   // relative inflation of every culling radius
constexpr double kFarRatio = 1e5;   // |oc|/r beyond which a sphere is never culled
constexpr double kNoWin = 1.0 + 0x1.0p-40;  // "quotient provably >= best" factor
// Point-light shadow packets with more candidate spheres than this are split in two (pk_light);
// variants with more than 64 spheres only (MAXC > 1).
#ifndef RT_SHADOW_SPLIT
#define RT_SHADOW_SPLIT 1
#endif
#ifndef RT_SHADOW_SPLIT_MIN
#define RT_SHADOW_SPLIT_MIN 16
#endif
constexpr bool kShadowSplit = RT_SHADOW_SPLIT != 0;
constexpr int kShadowSplitMin = RT_SHADOW_SPLIT_MIN;

// Feature bits of a kernel variant: code for a feature the scene does not use is not compiled
// in, which is what keeps the FP64 register budget (and so the occupancy) down.
constexpr int kFeatSpec = 1;    // some opaque material has specular > 0: Blinn-Phong pow
constexpr int kFeatArea = 2;    // build-defined area light
constexpr int kFeatTris = 4;    // triangles / models
constexpr int kFeatJodie = 8;   // Reinhard-Jodie fused tonemap (log/pow)
constexpr int kFeatPlanes = 16; // ≥ 3 planes: shadow packets also cull planes (cull_capsule)
constexpr int kFeatAll = 31;
// with kFeatArea only: no planes and no point lights (C5: spheres lit by the area light), so the
// plane and point-light code compiles away; the single-sample instantiation then runs at 6
// waves/SIMD (80 VGPRs): C5 508 -> 490 us at 5 waves, -> 482 us at 6 (MI355X)
constexpr int kFeatNoPL = 32;
// Fix-up variant (with no other feature; single sample, ≤ 64 spheres: C2): a lane whose shadow
// ray the classifier leaves undecided does not march (computeTransmittance's exact loop is not
// compiled in, which takes the variant from 80 VGPRs + 44 B/lane of spills at 6 waves/SIMD to 64
// VGPRs + 12 B at 8); its pixel is queued instead and packet_fixup_kernel renders it with the
// exact per-pixel path after the launch (0.08 % of C2's shadow rays are undecided).
constexpr int kFeatFix = 128;
#ifndef RT_PACKET_FIX_WAVES
#define RT_PACKET_FIX_WAVES 8
#endif

// Waves per SIMD of the single-sample variant for <= 64 spheres, point lights and no other
// feature (C2): 6 with its light records read through the scalar cache (80 VGPRs, 48 B/lane of
// scratch): C2 48.1 -> 46.7 us against 5 waves (95 VGPRs + 20 B, lights from LDS), MI355X
constexpr int kPkStack = 64;       // wave-coherent BVH walk: node stack entries per wave (depth ≤ 48)
// A/B options (off): the shading point and normal parked in LDS (6 doubles per lane, structure
// of arrays) across the area light's sample loop (RT_PK_AREA_PARK) or the point-light loop
// (RT_PK_PARK_POINT) of the ≤ 64-sphere variants, instead of in registers.  At 80 VGPRs (6
// waves/SIMD) this cuts C5's spills 116 → 44 B/lane (live scratch 5.6 → 2.2 MB per XCD against a
// 4 MB L2: HBM traffic 5.25 → 2.44× the framebuffer) and C2's 44 → 12 B/lane (1.47 → 1.15×),
// but the reloads cost time: C5 414 → 434 µs, C2 38.3 → 38.9 µs per frame
// (profiles/r04_ab_park.txt, r04_park_traffic.json).
#ifndef RT_PK_AREA_PARK
#define RT_PK_AREA_PARK 0
#endif
#ifndef RT_PK_PARK_POINT
#define RT_PK_PARK_POINT 0
#endif
#ifndef RT_PACKET_SMALL_WAVES
#define RT_PACKET_SMALL_WAVES 6
#endif
// Waves per SIMD of the single-sample area-only variant (C5: spheres lit by the area light)
#ifndef RT_PACKET_AREA_WAVES
#define RT_PACKET_AREA_WAVES 6
#endif
// Waves per SIMD the lean variants are compiled for (4 = at most 128 VGPRs).
#ifndef RT_PACKET_LEAN_WAVES
#define RT_PACKET_LEAN_WAVES 4
#endif
// ... the triangle-only variants (BVH traversal; models without specular materials)
#ifndef RT_PACKET_TRIS_WAVES
#define RT_PACKET_TRIS_WAVES 4
#endif
// ... and the single-sample variants without Blinn-Phong / triangles (5 = at most 96 VGPRs)
#ifndef RT_PACKET_AA1_WAVES
#define RT_PACKET_AA1_WAVES 5
#endif

// This lane's index in the wave, formed where it is used: an opaque (volatile) mbcnt pair the
// compiler cannot hoist and keep live — it spilled the hoisted lane·80 LDS offset of the culls
// in the C2 variant.  C2 46.9 → 46.5 µs per launch, interleaved 3 rounds
// (profiles/r04_ab_c2_march_save_opaque_lane.txt; RT_PK_OPAQUE_LANE=0: threadIdx.x & 63).
#ifndef RT_PK_OPAQUE_LANE
#define RT_PK_OPAQUE_LANE 1
#endif
__device__ __forceinline__ int cull_lane() {
#if RT_PK_OPAQUE_LANE
    int l;
    __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
#else
    return static_cast<int>(threadIdx.x & 63);
#endif
}

// (wave reductions, lane broadcasts: rt_trace_common.hpp)

// A sphere of the packet image (LDS): kPkSph doubles — cx cy cz r², the camera-cone terms as 8
// floats (cone_terms: vx vy vz q | rr dv slack r, r = the culling radius rounded up), the
// camera-ray constant c = oc·oc − r² with oc = cam − C (Shape.h:73,77; the candidates form oc
// again, the same three subtractions), 8 B of padding.  The lane-parallel culls read record `lane` with ds_read_b128: at an 80-B stride the
// 16 lanes of every ds_read_b128 lane group start on distinct 16-B slots of the 256-B bank row
// (20·lane mod 64 distinct), where the former 32-B records (plus a separate radius array) gave
// 2- and 4-way bank conflicts (C3: 1.84 conflict cycles per LDS cycle).
constexpr int kPkSph = 10;

struct PacketScene {
    const double* sph;   // LDS: sphere records (kPkSph doubles, above)
    const double* pl;    // LDS: planes (px py pz nx ny nz (p−cam)·n −)
    const double* lt;    // LDS: point lights
    const double* tri;   // HBM
    const double* mat;   // HBM: material table [spheres | planes | triangles]
    const double* bvh;   // HBM: triangle BVH, or null
    const int32_t* bvh_tri;
    // scenes with >= kSphChunkMin spheres: spheres are in spatial-chunk order (sph, rad, cone,
    // pre), chunk c's bounding sphere is pseudo-sphere ns + c of sph / rad / cone (nb of them),
    // and orig[i] is sorted sphere i's index in the scene (material table, closest-hit ties)
    const int32_t* orig;
    int ns, np, nt, nl, nb;
    int* wstk;  // LDS: this wave's node stack of the wave-coherent BVH walk (kFeatTris variants)
};

// Closest hit of the packet kernel: t and the primitive's index in the material table order
// [spheres | planes | triangles] (one register instead of a kind and a per-kind index).
struct PkHit {
    double t;
    int prim;
};

// Candidate masks: MAXC chunks of 64 spheres.  m[c] is wave-uniform (a ballot result).
template <int MAXC>
struct Masks {
    uint64_t m[MAXC];
    uint64_t pm;  // shadow packets: planes 0..63 that may block (bit set), the rest are clear
};

template <int MAXC>
__device__ __forceinline__ Masks<MAXC> all_candidates(int ns) {
    Masks<MAXC> M;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int left = ns - 64 * c;
        M.m[c] = left >= 64 ? ~0ull : (left <= 0 ? 0ull : ((1ull << left) - 1ull));
    }
    M.pm = ~0ull;
    return M;
}

// ------------------------------------------------------------------ packet culling (FP32)
// The culls only decide which spheres a packet may skip, so they run in FP32 (half the FP64
// issue cost, cheap sqrt) with every rounding error covered by explicit slack: each test keeps a
// sphere unless the FP32 value clears the exact bound by more than kF32Slack times the
// magnitudes involved (≥ 5× the worst-case FP32 error of the expression, derived per test
// below).  Differences of scene coordinates are taken in FP64 first, so large coordinates do not
// cost relative precision; NaN/inf anywhere keeps the sphere (every comparison is negated).
constexpr float kF32Slack = 2e-5f;
constexpr float kF32Up = 1.0f + 1e-6f;  // rounds a positive FP32 conversion up

__device__ __forceinline__ float f32_up(double v) { return static_cast<float>(v) * kF32Up; }
__device__ __forceinline__ float dot3f(float ax, float ay, float az, float bx, float by, float bz) {
    return ax * bx + ay * by + az * bz;
}
// v_sqrt_f32 without the compiler's correct-rounding fix-up (≤ 1 ulp, 1.2e-7 relative): every
// FP32 square root of the culls and classifications carries a margin of ≥ 5e-7 for it.
__device__ __forceinline__ float sqrt_f32(float x) { return __builtin_amdgcn_sqrtf(x); }

// Camera-ray packet: origin `o` shared, directions within the cone (axis, cos_min), cos_min > 0.
// Sphere (C, r) is kept iff angle(C−o, axis) ≤ θ + β, sin β = r'/|C−o| (r' = inflated r),
// evaluated without divisions as  (C−o)·axis ≥ cosθ·√(|C−o|²−r'²) − sinθ·r'.
// Error bound (d = |C−o|): |C−o|² and the dot product carry < 5e-7·d² and 3e-7·d; spheres with
// d ≤ 1.01·r' are kept outright, so |C−o|²−r'² ≥ 0.0199·r'² and its square root is off by at
// most 2.5e-6·d; total < 3e-6·d against a slack of 2e-5·d.
// The cone test's per-sphere terms depend on the camera only (every camera ray starts there),
// so each workgroup forms them once into LDS (8 floats per sphere: vx vy vz q | rr dv slack r),
// with q = NaN for spheres that are always kept; the same FP32 expressions, so the same masks.
__device__ __forceinline__ void cone_terms(const double* s, double radius, d3 o, float* out) {
    const float r = f32_up(radius);
    const float vx = static_cast<float>(s[0] - o.x), vy = static_cast<float>(s[1] - o.y),
                vz = static_cast<float>(s[2] - o.z);
    const float dv2 = dot3f(vx, vy, vz, vx, vy, vz);
    const float rr = r * (1.0f + static_cast<float>(kCullRel));
    const float dv = sqrt_f32(dv2);
    const bool always = !(dv > 1.01f * rr) || !(dv <= static_cast<float>(kFarRatio) * r);
    out[0] = vx;
    out[1] = vy;
    out[2] = vz;
    out[3] = always ? __builtin_nanf("") : sqrt_f32(dv2 - rr * rr);  // |C−o|·cos β
    out[4] = rr;
    out[5] = dv;
    out[6] = kF32Slack * dv;
    out[7] = r;  // the capsule test's radius
}

template <int MAXC>
__device__ __forceinline__ Masks<MAXC> cull_cone(const PacketScene& S, d3 axis, double cos_min) {
    Masks<MAXC> M;
    const int lane = cull_lane();
    const float cs = static_cast<float>(cos_min) * (1.0f - 1e-6f);  // rounded down (cs > 0)
    const float sn = sqrt_f32(fmaxf(0.0f, 1.0f - cs * cs)) * (1.0f + 1e-5f);  // rounded up
    const float ax = static_cast<float>(axis.x), ay = static_cast<float>(axis.y),
                az = static_cast<float>(axis.z);
    auto test = [&](int k) {
        const float4* c4 = reinterpret_cast<const float4*>(S.sph + kPkSph * k + 4);
        const float4 a = c4[0];
        const float4 b = c4[1];
        const float q = a.w, rr = b.x, dv = b.y, slack = b.z;
        // θ + β ≥ π, or the axis is outside the cone around C−o (NaN q: always kept)
        return !(q > -cs * dv + slack) ||
               !(dot3f(a.x, a.y, a.z, ax, ay, az) < cs * q - sn * rr - slack);
    };
    uint64_t live = ~0ull;  // chunks whose bounding sphere the cone may meet
    if constexpr (MAXC > 1)
        if (S.nb > 0) live = __ballot(lane < S.nb && test(S.ns + lane));
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        M.m[c] = 0ull;
        if (!((live >> c) & 1ull)) continue;  // uniform: no sphere of the chunk is in the cone
        const int k = c * 64 + lane;
        M.m[c] = __ballot(k < S.ns && test(k));
    }
    M.pm = ~0ull;
    return M;
}

// Shadow packet: origins inside ball (c, R), every ray aims at a light inside ball (L, RL).
// The segments [so, lpos] lie in the capsule of radius max(R, RL) around [c, L]; the traced
// rays do not quite follow them: directLightning takes the direction from the hit point P
// (L = (lpos − P)/dist) but starts the ray at so = P + n·bias, so the point at parameter t is
// so + (t/dist)·(lpos − so) + (t/dist)·n·bias, within bias·|n| of its segment for every
// t ≤ maxDist = dist − bias.  The capsule radius carries that bias (a sphere grazed by the
// ray but not by the segment is kept).  The squared distance
// from C to the segment carries < 1.5e-6·(|C−c|² + |L−c|²) of FP32 error (any of the three
// branches, including a branch chosen wrongly next to a boundary where they meet
// continuously), against a slack of 2e-5·(|C−c|² + |L−c|²).
template <int MAXC, int FEAT>
__device__ __forceinline__ Masks<MAXC> cull_capsule(const PacketScene& S, d3 c, float R, d3 L,
                                                    double RL, double bias) {
    Masks<MAXC> M;
    const int lane = cull_lane();
    const float sx = static_cast<float>(L.x - c.x), sy = static_cast<float>(L.y - c.y),
                sz = static_cast<float>(L.z - c.z);
    const float sl2 = dot3f(sx, sy, sz, sx, sy, sz);
    const float inv_sl2 = 1.0f / sl2;  // wave-uniform; only read when sl2 > 0
    const float Rc = fmaxf(R, f32_up(RL)) + f32_up(fabs(bias)) * 1.001f;  // |n| ≤ 1 + 2ε
    auto test = [&](int k) {
        const double2* s2 = reinterpret_cast<const double2*>(S.sph + kPkSph * k);
        const double2 sxy = s2[0], szr = s2[1];  // cx cy | cz r² (two ds_read_b128)
        const float r = reinterpret_cast<const float4*>(s2 + 2)[1].w;  // f32_up(radius)
        const float vx = static_cast<float>(sxy.x - c.x), vy = static_cast<float>(sxy.y - c.y),
                    vz = static_cast<float>(szr.x - c.z);
        const float vs = dot3f(vx, vy, vz, sx, sy, sz);
        const float vv = dot3f(vx, vy, vz, vx, vy, vz);
        float d2;
        if (!(vs > 0.0f) || !(sl2 > 0.0f)) {
            d2 = vv;
        } else if (!(vs < sl2)) {
            const float wx = vx - sx, wy = vy - sy, wz = vz - sz;
            d2 = dot3f(wx, wy, wz, wx, wy, wz);
        } else {
            d2 = vv - (vs * vs) * inv_sl2;  // one more rounding than a division: ≪ slack
        }
        const float lim = (r + Rc) * (1.0f + static_cast<float>(kCullRel));
        const float far = static_cast<float>(kFarRatio) * r - Rc;
        return !(d2 > lim * lim + kF32Slack * (vv + sl2)) || !(far > 0.0f) || !(vv <= far * far);
    };
    uint64_t live = ~0ull;  // chunks whose bounding sphere the capsule may meet
    if constexpr (MAXC > 1)
        if (S.nb > 0) live = __ballot(lane < S.nb && test(S.ns + lane));
#pragma unroll
    for (int ch = 0; ch < MAXC; ++ch) {
        M.m[ch] = 0ull;
        if (!((live >> ch) & 1ull)) continue;  // uniform: the capsule misses the whole chunk
        const int k = ch * 64 + lane;
        M.m[ch] = __ballot(k < S.ns && test(k));
    }
    // Planes (feature kFeatPlanes, scenes with three or more, where one lane-parallel test costs
    // less than the per-lane plane tests it saves): a plane with the capsule strictly on one
    // side — the origin ball and the light ball on the same side by their radii, the rays' bias
    // offset and 1e-8 of the magnitudes (FP64 rounding, and pk_occlusion's 1e-9 relative
    // "beyond the light" margin) — meets no ray of the packet within [0, maxDist], so
    // pk_occlusion would classify it clear for every lane.  |n|₁ bounds |n|₂.  The exact march
    // (pk_transmittance) still tests every plane.
    M.pm = ~0ull;
    if constexpr ((FEAT & kFeatPlanes) != 0) {
        if (S.np <= 64) {
            bool keep = true;
            if (lane < S.np) {
                const double* q = S.pl + kPlStride * lane;
                const d3 pn = mk(q[3], q[4], q[5]);
                const d3 p0 = mk(q[0], q[1], q[2]);
                const d3 vc = c - p0, vl = L - p0;
                const double nn = fabs(pn.x) + fabs(pn.y) + fabs(pn.z);
                const double sc = dot(vc, pn), sl = dot(vl, pn);
                const double mag = (fabs(vc.x) + fabs(vc.y) + fabs(vc.z) + fabs(vl.x) +
                                    fabs(vl.y) + fabs(vl.z) + static_cast<double>(R) + RL) * nn;
                const double off = fabs(bias) * 1.01 * nn + 1e-8 * mag;
                const double mc = static_cast<double>(R) * 1.001 * nn + off;
                const double ml = RL * 1.001 * nn + off;
                keep = !((sc > mc && sl > ml) || (sc < -mc && sl < -ml));
            }
            M.pm = __ballot(keep);
        }
    }
    return M;
}

// The running closest hit takes candidate i at t when the reference's in-order loop with strict
// '<' (Shape.h:36) would end on it: t < best, or — when the spheres are in spatial-chunk order
// (ORD, orig[] = scene indices) — t == best with a lower scene index.
template <bool ORD>
__device__ __forceinline__ void take_closest(double t, int i, const int32_t* orig, bool& found,
                                             double& best, int& prim) {
    bool take = !found || t < best;
    if constexpr (ORD) take = take || (t == best && orig[i] < orig[prim]);
    if (take) {
        found = true;
        best = t;
        prim = i;
    }
}

// Root selection of Sphere::Intersect (Shape.h:84-97) folded into the running closest.
// Requires two_a > 0 (then t0 ≤ t1 exactly); divisions are skipped when the candidate
// provably cannot be strictly closer than `best`.
template <bool ORD>
__device__ __forceinline__ void sphere_roots(double b, double disc, double two_a, int i,
                                             const int32_t* orig, bool& found, double& best,
                                             int& prim) {
    if (disc < 0.0) return;
    const double sq = sqrt(disc);
    const double n0 = -b - sq;
    if (found && n0 > (best * two_a) * kNoWin) return;  // t1 >= t0 > best (strictly)
    double t = n0 / two_a;
    if (t < 1e-6) {
        t = (-b + sq) / two_a;
        if (t < 1e-6) return;
    }
    take_closest<ORD>(t, i, orig, found, best, prim);
}

// sphere_roots through the sqrt/division cores (rt_device.hpp), r2a = rcp_refined(two_a) with
// two_a in [2^-100, 2^100].  A finite disc ≥ 2^-767 keeps b, √disc and both numerators finite;
// a numerator |n| ≥ 2^-900 divides exactly, and a smaller one gives |t| < 2^-790 both exactly
// and through the core, so the 1e-6 test (the only use of such a root) decides alike.  Other
// discriminants take the literal path.  t0 ≤ t1 as in sphere_roots.
template <bool ORD>
__device__ __forceinline__ void sphere_roots_core(double b, double disc, double two_a, double r2a,
                                                  int i, const int32_t* orig, bool& found,
                                                  double& best, int& prim) {
    if (disc < 0.0) return;
    double t;
    if (disc >= 0x1p-767 && disc <= 0x1.fffffffffffffp+1023) {
        const double sq = sqrt_core(disc);
        t = div_core(-b - sq, two_a, r2a);
        if (t < 1e-6) {
            t = div_core(-b + sq, two_a, r2a);
            if (t < 1e-6) return;
        }
    } else {
        const double sq = sqrt(disc);
        t = (-b - sq) / two_a;
        if (t < 1e-6) {
            t = (-b + sq) / two_a;
            if (t < 1e-6) return;
        }
    }
    take_closest<ORD>(t, i, orig, found, best, prim);
}

// The reference's literal root selection, for degenerate directions (2a not > 0).
template <bool ORD>
__device__ __forceinline__ void sphere_roots_literal(double b, double disc, double two_a, int i,
                                                     const int32_t* orig, bool& found,
                                                     double& best, int& prim) {
    if (disc < 0.0) return;
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
        if (t < 1e-6) return;
    }
    take_closest<ORD>(t, i, orig, found, best, prim);
}

// Plane::Intersect (Shape.h:149-159) given num = (p − o)·n and denom = n·d.
__device__ __forceinline__ void plane_t(double num, double denom, int p, bool& found,
                                        double& best, int& prim) {
    if (!(fabs(denom) > 1e-6)) return;
    if (found && best >= 0x1p-900) {  // skip the division when t = num/denom is provably >= best
        const double lim = (best * denom) * kNoWin;  // (a normal product: |denom| > 1e-6)
        if (denom > 0.0 ? num > lim : num < lim) return;
    }
    const double t = num / denom;
    if (t >= 0.0 && (!found || t < best)) {
        found = true;
        best = t;
        prim = p;
    }
}

// plane_t through the division core for a camera-ray plane whose numerator passed the
// prologue's test (2^-900 ≤ |num| ≤ 2^400, |n|₁ ≤ 2^90): with 1e-6 < |denom| ≤ 2^91 every
// operand is inside div_core's range, so t has the bits of num / denom.
__device__ __forceinline__ void plane_t_core(double num, double denom, int p, bool& found,
                                             double& best, int& prim) {
    if (!(fabs(denom) > 1e-6)) return;
    // opposite signs: t = num/denom is negative and nonzero (|num| ≥ 2^-900), so the
    // reference's t >= 0 rejects it — a whole wave looking away from the plane skips the division
    if ((num < 0.0) != (denom < 0.0)) return;
    const double t = div_core(num, denom, rcp_refined(denom));
    if (t >= 0.0 && (!found || t < best)) {
        found = true;
        best = t;
        prim = p;
    }
}

// The triangles' part of IntersectClosest over the BVH, walked once per WAVE (the packet
// kernel's rays of an 8x8 tile, or the lanes of a shadow march, go through the same nodes):
// the node stack is wave-uniform in LDS, node boxes, leaf triangle ids and triangle records
// are read through the scalar cache (wave-uniform addresses: SGPRs, no per-lane loads), and
// each lane tests the popped node's box against its own current best (the per-lane walk's
// test, bvh_triangles in rt_trace_common.hpp, with the same 1e-9 margin), so a lane only tests
// the triangles of leaves its ray reaches and is not closer than.  A lane may see nodes its
// own walk would not visit (another lane hit them); every triangle it tests in a leaf is a real
// intersection test, so it still returns exactly the (t, index) minimum among the triangles
// the reference tests (the leaf of the winning triangle is always entered: every ancestor box
// contains the hit, and no box whose entry exceeds the winner's t is needed).  Children are
// pushed nearer-first along the node's split axis by the lanes' majority direction.
typedef const __attribute__((address_space(4))) int32_t* pk_cip;
typedef const __attribute__((address_space(4))) double* pk_cdp;
__device__ __forceinline__ void bvh_wave(const PacketScene& S, d3 o, d3 d, bool& found,
                                         double& best, int& kind, int& idx) {
    const d3 inv = mk(d.x != 0.0 ? 1.0 / d.x : 0.0, d.y != 0.0 ? 1.0 / d.y : 0.0,
                      d.z != 0.0 ? 1.0 / d.z : 0.0);
    const pk_cdp bvh = (pk_cdp)S.bvh;
    const pk_cdp tri = (pk_cdp)S.tri;
    const pk_cip ord = (pk_cip)S.bvh_tri;
    int* stk = S.wstk;
    bool tf = false;
    double tb = 0.0;
    int ti = 0;
    int sp = 0;
    stk[sp++] = 0;  // every active lane writes the same value
    while (sp > 0) {
        const int node = __builtin_amdgcn_readfirstlane(stk[--sp]);
        const pk_cdp nd = bvh + kBvhNodeStride * node;
        const double bound = tf ? (found ? fmin(tb, best) : tb) : (found ? best : INFINITY);
        double tn;
        const bool in = bvh_box_v(mk(nd[0], nd[1], nd[2]), mk(nd[3], nd[4], nd[5]), o, d, inv, tn) &&
                        !(tn > bound * (1.0 + 1e-9));
        if (__ballot(in) == 0) continue;  // uniform
        const double w = nd[6];
        const int first = __double2loint(w), count = __double2hiint(w);
        if (count > 0) {
            if (in) {
                for (int j = first; j < first + count; ++j) {
                    const int i = ord[j];
                    const pk_cdp q = tri + kTriStride * i;
                    double t;
                    if (tri_hit_v(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]),
                                  o, d, t) &&
                        (!tf || t < tb || (t == tb && i < ti))) {
                        tf = true;
                        tb = t;
                        ti = i;
                    }
                }
            }
            continue;
        }
        const int axis = __double2loint(nd[7]);
        const double da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
        const int pos = __builtin_popcountll(__ballot(in && da > 0.0));
        const int neg = __builtin_popcountll(__ballot(in && da < 0.0));
        const bool low_first = pos >= neg;  // the lower child is nearer for rays going up
        stk[sp++] = low_first ? first + 1 : first;
        stk[sp++] = low_first ? first : first + 1;
    }
    if (tf && (!found || tb < best)) {
        found = true;
        best = tb;
        kind = 3;
        idx = ti;
    }
}

template <int FEAT>
__device__ __forceinline__ void triangles(const PacketScene& S, d3 o, d3 d, bool& found,
                                          double& best, int& prim) {
    if (!(FEAT & kFeatTris)) return;
    const int base = S.ns + S.np;
    if (S.bvh) {
        int kind = 0, ti = -1;
        bvh_wave(S, o, d, found, best, kind, ti);
        if (kind == 3) prim = base + ti;
        return;
    }
    for (int i = 0; i < S.nt; ++i) {
        double t;
        if (tri_hit(S.tri, i, o, d, t) && (!found || t < best)) {
            found = true;
            best = t;
            prim = base + i;
        }
    }
}

// IntersectClosest for a camera ray (origin = the camera) over the candidate spheres.
template <int MAXC, int FEAT>
__device__ __forceinline__ bool closest_camera(const PacketScene& S, const Masks<MAXC>& M,
                                               int nchunks, d3 o, d3 d, PkHit& h) {
    bool found = false;
    double best = 0.0;
    int prim = -1;
    const double a = dot(d, d);
    const double two_a = 2.0 * a, four_a = 4.0 * a;
    const bool regular = two_a > 0.0;
    const bool core = two_a >= 0x1p-100 && two_a <= 0x1p100;  // camera rays are unit vectors
    if (__ballot(!core) == 0) {  // uniform: the whole wave divides through the shared reciprocal
        const double r2a = rcp_refined(two_a);
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            if (c >= nchunks) break;
            uint64_t m = M.m[c];
            while (m) {
                const int i = c * 64 + __builtin_ctzll(m);
                m &= m - 1;
                const double* q = S.sph + kPkSph * i;
                const double b = 2.0 * dot(o - mk(q[0], q[1], q[2]), d);  // oc = cam − C
                const double disc = b * b - four_a * q[8];
                sphere_roots_core<(MAXC > 1)>(b, disc, two_a, r2a, i, S.orig, found, best, prim);
            }
        }
    } else {
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            if (c >= nchunks) break;
            uint64_t m = M.m[c];
            while (m) {
                const int i = c * 64 + __builtin_ctzll(m);
                m &= m - 1;
                const double* q = S.sph + kPkSph * i;
                const double b = 2.0 * dot(o - mk(q[0], q[1], q[2]), d);  // oc = cam − C
                const double disc = b * b - four_a * q[8];
                if (regular) sphere_roots<(MAXC > 1)>(b, disc, two_a, i, S.orig, found, best, prim);
                else sphere_roots_literal<(MAXC > 1)>(b, disc, two_a, i, S.orig, found, best, prim);
            }
        }
    }
    for (int i = 0; i < S.np; ++i) {
        const double* p = S.pl + kPlStride * i;
        const double denom = dot(mk(p[3], p[4], p[5]), d);
        if (p[7] != 0.0) plane_t_core(p[6], denom, S.ns + i, found, best, prim);  // uniform
        else plane_t(p[6], denom, S.ns + i, found, best, prim);
    }
    triangles<FEAT>(S, o, d, found, best, prim);
    h.t = best;
    h.prim = prim;
    return found;
}

// IntersectClosest for an arbitrary ray over the candidate spheres.
template <int MAXC, int FEAT>
__device__ __forceinline__ bool closest_masked(const PacketScene& S, const Masks<MAXC>& M,
                                               int nchunks, d3 o, d3 d, PkHit& h) {
    bool found = false;
    double best = 0.0;
    int prim = -1;
    const double a = dot(d, d);
    const double two_a = 2.0 * a, four_a = 4.0 * a;
    const bool regular = two_a > 0.0;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c >= nchunks) break;
        uint64_t m = M.m[c];
        while (m) {
            const int i = c * 64 + __builtin_ctzll(m);
            m &= m - 1;
            const double* s = S.sph + kPkSph * i;
            const d3 oc = o - mk(s[0], s[1], s[2]);
            const double b = 2.0 * dot(oc, d);
            const double cc = dot(oc, oc) - s[3];
            const double disc = b * b - four_a * cc;
            if (regular) sphere_roots<(MAXC > 1)>(b, disc, two_a, i, S.orig, found, best, prim);
            else sphere_roots_literal<(MAXC > 1)>(b, disc, two_a, i, S.orig, found, best, prim);
        }
    }
    for (int i = 0; i < S.np; ++i) {
        const double* p = S.pl + kPlStride * i;
        const d3 n = mk(p[3], p[4], p[5]);
        plane_t(dot(mk(p[0], p[1], p[2]) - o, n), dot(n, d), S.ns + i, found, best, prim);
    }
    triangles<FEAT>(S, o, d, found, best, prim);
    h.t = best;
    h.prim = prim;
    return found;
}

template <int MAXC>
__device__ __forceinline__ const double* pk_material(const PacketScene& S, const PkHit& h) {
    // the table is [spheres | planes | triangles] in scene order; spheres in chunk order (MAXC
    // > 1: > 64 spheres) map back to it
    int m = h.prim;
    if constexpr (MAXC > 1) m = h.prim < S.ns ? S.orig[h.prim] : h.prim;
    return S.mat + kMatStride * m;
}

__device__ __forceinline__ d3 pk_normal(const PacketScene& S, const PkHit& h, d3 p) {
    if (h.prim < S.ns) {
        const double* s = S.sph + kPkSph * h.prim;
        return unit(p - mk(s[0], s[1], s[2]));
    }
    if (h.prim < S.ns + S.np) {
        const double* q = S.pl + kPlStride * (h.prim - S.ns);
        return mk(q[3], q[4], q[5]);
    }
    const double* q = S.tri + kTriStride * (h.prim - S.ns - S.np);
    return mk(q[9], q[10], q[11]);
}

// computeTransmittance (Scene.h:35-77) over the candidate spheres of the shadow packet.
template <int MAXC, int FEAT>
__device__ __forceinline__ double pk_transmittance(const PacketScene& S, const Masks<MAXC>& M,
                                                   int nchunks, d3 o, d3 d, double max_dist,
                                                   double bias) {
    double T = 1.0, traveled = 0.0;
    int safety = 64;
    while (safety-- > 0 && T > 1e-4 && traveled < max_dist) {
        PkHit h;
        if (!closest_masked<MAXC, FEAT>(S, M, nchunks, o, d, h)) break;
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
        T *= sclamp(pk_material<MAXC>(S, h)[5], 0.0, 1.0);
        o = (o + d * t) + d * bias;
        traveled += t + bias;
    }
    return sclamp(T, 0.0, 1.0);
}

// Occlusion test for an all-opaque scene (the only kind this kernel renders: any material with
// transparency > 0 goes to the tree kernel), where computeTransmittance (Scene.h:35-77) can only
// return 1 (clear) or 0 (blocked): its first closest hit t* decides — t* in (bias, maxDist)
// blocks, t* >= maxDist or no hit is clear, t* <= bias starts the march over near hits.  Each
// candidate is classified with a FP32 square root and one shared FP64 reciprocal instead of the
// reference's sqrt and division, with an explicit error bound Δ on every root; any root within
// Δ of a threshold (1e-6, bias, maxDist), any near hit, or any value out of the fast ranges makes
// the lane undecided, and undecided lanes run the exact march.  Returns 0 clear, 1 blocked,
// 2 undecided.  The discriminant (and with it hit/miss) is the reference's FP64 expression.
template <int MAXC, int FEAT>
__device__ __forceinline__ int pk_occlusion(const PacketScene& S, const Masks<MAXC>& M,
                                            int nchunks, d3 o, d3 d, double max_dist,
                                            double bias) {
    if constexpr ((FEAT & kFeatTris) != 0) return 2;
    const double a = dot(d, d);
    const double two_a = 2.0 * a, four_a = 4.0 * a;
    if (!(two_a >= 0x1p-100 && two_a <= 0x1p100)) return 2;
    const double inv2a = rcp_refined(two_a);  // within 1 ulp of 1/2a: far inside the Δ margin
    bool blocked = false, undecided = false;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c >= nchunks) break;
        uint64_t m = M.m[c];
        while (m) {
            const int i = c * 64 + __builtin_ctzll(m);
            m &= m - 1;
            const double* s = S.sph + kPkSph * i;
            const d3 oc = o - mk(s[0], s[1], s[2]);
            const double b = 2.0 * dot(oc, d);
            const double cc = dot(oc, oc) - s[3];
            const double disc = b * b - four_a * cc;
            if (disc < 0.0) continue;  // miss, exactly as the reference decides it
            if (!(disc == 0.0 || (disc > 1e-30 && disc < 1e30))) {
                undecided = true;
                continue;
            }
            // |sq − fl(√disc)| ≤ 5e-7·√disc (FP32 conversion + sqrt_f32), so both roots are within
            // Δ = 2e-6·(|b| + sq)/2a of the reference's fl(fl(−b ∓ sq)/2a) (2× margin)
            const double sq = static_cast<double>(sqrt_f32(static_cast<float>(disc)));
            const double delta = 2e-6 * (fabs(b) + sq) * inv2a;
            double t = (-b - sq) * inv2a;
            if (!(t >= 1e-6 + delta)) {
                if (!(t < 1e-6 - delta)) {
                    undecided = true;
                    continue;
                }
                t = (-b + sq) * inv2a;
                if (t < 1e-6 - delta) continue;  // both roots behind: no hit
                if (!(t >= 1e-6 + delta)) {
                    undecided = true;
                    continue;
                }
            }
            if (t >= max_dist + delta) continue;              // beyond the light
            if (t > bias + delta && t < max_dist - delta) blocked = true;
            else undecided = true;                            // near hit or on a boundary
        }
    }
    for (int i = 0; i < S.np; ++i) {
        if (i < 64 && ((M.pm >> i) & 1ull) == 0) continue;  // clear for the whole packet (uniform)
        // Plane::Intersect (Shape.h:149-159): t = num / denom, decided without the division:
        // with A = num·sign(denom), B = |denom|, t lies on the side of x that A lies of x·B
        // (1e-9 relative margin ≫ the FP64 rounding of the quotient and the product)
        const double* p = S.pl + kPlStride * i;
        const d3 n = mk(p[3], p[4], p[5]);
        const double denom = dot(n, d);
        if (!(fabs(denom) > 1e-6)) continue;
        const double num = dot(mk(p[0], p[1], p[2]) - o, n);
        const double A = denom > 0.0 ? num : -num, B = fabs(denom);
        if (A < -1e-300 * B) continue;                        // t < 0 (no underflow to −0)
        if (A >= max_dist * B * (1.0 + 1e-9)) continue;       // beyond the light
        if (A > bias * B * (1.0 + 1e-9) && A < max_dist * B * (1.0 - 1e-9)) blocked = true;
        else undecided = true;
    }
    return undecided ? 2 : (blocked ? 1 : 0);
}

// Shadow-packet candidates: the origins `so` of the lanes in `casting_lanes` lie in a ball around
// the first such lane's origin (exact), radius = the wave maximum of the distances in FP32
// rounded up; every segment ends in the light's ball (lcenter, lrad); non-finite origins or
// radius keep every sphere.
struct OriginBall {
    d3 c;
    float R;
    bool ok;  // wave-uniform: some lane casts, every origin finite, R finite
};
__device__ __forceinline__ OriginBall origin_ball(bool casting_lane, d3 so) {
    OriginBall B;
    const uint64_t casting = __ballot(casting_lane);
    B.c = mk(0.0, 0.0, 0.0);
    B.R = 0.0f;
    B.ok = false;
    if (!casting) return B;
    const bool bad = casting_lane && !(isfinite(so.x) && isfinite(so.y) && isfinite(so.z));
    B.c = lane_d3(so, __builtin_ctzll(casting));
    float r_lane = 0.0f;
    if (casting_lane) {  // |so − c| in FP32, rounded up (FP64 differences, 5e-7 rel. error)
        const float dx = static_cast<float>(so.x - B.c.x), dy = static_cast<float>(so.y - B.c.y),
                    dz = static_cast<float>(so.z - B.c.z);
        r_lane = sqrt_f32(dot3f(dx, dy, dz, dx, dy, dz)) * (1.0f + 1e-5f);
    }
    B.R = wave_red<1>(r_lane);
    B.ok = !__ballot(bad) && isfinite(B.R);
    return B;
}

template <int MAXC, int FEAT>
__device__ __forceinline__ Masks<MAXC> shadow_masks(const PacketScene& S, bool casting_lane, d3 so,
                                                    d3 lcenter, double lrad, double bias) {
    const OriginBall B = origin_ball(casting_lane, so);
    return B.ok ? cull_capsule<MAXC, FEAT>(S, B.c, B.R, lcenter, lrad, bias)
                : all_candidates<MAXC>(S.ns);
}

// One light of directLightning (Scene.h:86-124) for the whole wave: every lane calls it
// (uniform control flow for the packet reductions); `active` lanes shade.
template <int MAXC, int FEAT, bool COUNT>
__device__ __forceinline__ void pk_light(const PacketScene& S, bool active, d3 P, d3 n, d3 view,
                                         const PkHit& h, d3 lpos, d3 E, d3 lcenter, double lrad,
                                         double bias, int nchunks, d3& diff, d3& spec,
                                         Counts& cnt, const Masks<MAXC>* pre = nullptr,
                                         bool* fix = nullptr) {
    double dist = 0.0, inv_d2 = 0.0;
    d3 L = mk(0.0, 0.0, 0.0);
    if (active) light_dir(lpos - P, dist, L, inv_d2);  // skipped by waves with no hit lane
    const bool reach = active && !(dist <= 0.0);
    if (!reach) L = mk(0.0, 0.0, 0.0);
    const double ndl = smax(0.0, dot(n, L));
    const bool need = reach && !(ndl <= 0.0) && !(dist <= bias);
    const d3 so = P + n * bias;
    const uint64_t casting = __ballot(need);
    if (!casting) return;  // no lane casts this shadow ray (uniform)
    // every lane stays in the code below until the march mask is formed (wave reductions);
    // lanes that cast no ray only take part in them
    int occ = 0;
    Masks<MAXC> M;
    if (pre) {
        M = *pre;
        if (need) occ = pk_occlusion<MAXC, FEAT>(S, M, nchunks, so, L, dist - bias, bias);
    } else {
        const OriginBall B = origin_ball(need, so);
        M = B.ok ? cull_capsule<MAXC, FEAT>(S, B.c, B.R, lcenter, lrad, bias)
                 : all_candidates<MAXC>(S.ns);
        bool split = false;
        if constexpr (kShadowSplit && MAXC > 1) {
            // A wide packet (origins straddling a depth edge: a sphere in front of a wall) gets a
            // fat capsule that keeps much of the scene, and every lane then classifies every
            // candidate: these waves run 10-35x the median and set the tail of a launch.  Such
            // a packet is split in two — the lanes within R/2 of the ball's centre and the rest —
            // each with its own ball and capsule (ANDed with the shared mask), and each group
            // walks only its own candidates.  Masks only shrink by provable misses, so every
            // lane's classification is unchanged.  The groups' capsules skip the plane cull
            // (they keep the shared one's plane mask: C3 -0.7 %).  8-rank row splits: slowest
            // rank C4 0.30 → 0.20 ms, C3 0.11 → 0.09 ms (with the march mask below); one whole
            // frame: C4 -1 %, C3 +1.2 %, C2/C5 ±0.5 % (tools/gpu_ab.sh, 3 interleaved rounds).
            int cand = 0;
#pragma unroll
            for (int c = 0; c < MAXC; ++c) cand += __builtin_popcountll(M.m[c]);
            split = B.ok && cand > kShadowSplitMin;  // uniform
            if (split) {
                float r_lane = 0.0f;
                if (need) {
                    const float dx = static_cast<float>(so.x - B.c.x),
                                dy = static_cast<float>(so.y - B.c.y),
                                dz = static_cast<float>(so.z - B.c.z);
                    r_lane = sqrt_f32(dot3f(dx, dy, dz, dx, dy, dz));
                }
                const bool near = r_lane <= 0.5f * B.R;
                Masks<MAXC> Mn = M, Mf = M;
                const OriginBall Bn = origin_ball(need && near, so);
                const OriginBall Bf = origin_ball(need && !near, so);
                if (Bn.ok) {
                    const Masks<MAXC> t =
                        cull_capsule<MAXC, (FEAT & ~kFeatPlanes)>(S, Bn.c, Bn.R, lcenter, lrad, bias);
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) Mn.m[c] &= t.m[c];
                    Mn.pm &= t.pm;
                }
                if (Bf.ok) {
                    const Masks<MAXC> t =
                        cull_capsule<MAXC, (FEAT & ~kFeatPlanes)>(S, Bf.c, Bf.R, lcenter, lrad, bias);
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) Mf.m[c] &= t.m[c];
                    Mf.pm &= t.pm;
                }
#pragma unroll 1
                for (int g = 0; g < 2; ++g) {  // uniform: one group after the other
                    Masks<MAXC> Mg;
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) Mg.m[c] = g == 0 ? Mn.m[c] : Mf.m[c];
                    Mg.pm = g == 0 ? Mn.pm : Mf.pm;
                    if (need && near == (g == 0))
                        occ = pk_occlusion<MAXC, FEAT>(S, Mg, nchunks, so, L, dist - bias, bias);
                }
            }
        }
        if (!split && need) occ = pk_occlusion<MAXC, FEAT>(S, M, nchunks, so, L, dist - bias, bias);
    }
    // The exact march (computeTransmittance) for the undecided lanes: a handful of lanes whose
    // shadow ray starts on or next to a surface, marching up to 64 closest-hit steps.  Over the
    // whole packet's mask such a march visits every candidate of a wide capsule at every step
    // (the slowest waves of C3 spend > 90 % of their time here), so it gets a capsule of its
    // own around the marching lanes' origins: every origin of the march lies on the segment
    // from its shadow-ray origin towards the light, inside that capsule, so the mask still
    // holds every sphere the march can hit.  C3's slowest waves 240 → 85 µs; its 8-rank
    // row split went from 1.37-1.45× the mean rank to 1.02-1.04× (profiles/r02_*).
    const bool undecided = need && occ == 2;
    double T = occ == 1 ? 0.0 : 1.0;
    if constexpr ((FEAT & kFeatFix) != 0) {
        // no march here: the pixel is queued for packet_fixup_kernel (its output is rewritten)
        if (undecided) *fix = true;
    } else if (__ballot(undecided)) {  // uniform
        Masks<MAXC> Mu = M;
        const OriginBall Bu = origin_ball(undecided, so);
        if (Bu.ok) {
            const Masks<MAXC> t = cull_capsule<MAXC, FEAT>(S, Bu.c, Bu.R, lcenter, lrad, bias);
#pragma unroll
            for (int c = 0; c < MAXC; ++c) Mu.m[c] &= t.m[c];
            Mu.pm &= t.pm;
        }
        if (undecided) T = pk_transmittance<MAXC, FEAT>(S, Mu, nchunks, so, L, dist - bias, bias);
    }
    if (!need) return;
    if (COUNT) cnt.shadow++;
    if (T <= bias) return;
    diff = diff + ((E * inv_d2) * ndl) * T;
    if constexpr ((FEAT & kFeatSpec) != 0) {
        const double* m = pk_material<MAXC>(S, h);
        if (m[5] <= 0.0 && m[4] > 0.0) {
            const d3 H = unit(L + view);
            const double ndh = smax(0.0, dot(n, H));
            if (ndh > 0.0) {
                const double sf = pow_bp(ndh, m[3]);
                spec = spec + ((E * inv_d2) * sf) * T;
            }
        }
    }
}

// Point light l's position and E = colour·intensity.  With <= 64 spheres (MAXC == 1) the record
// is read through the scalar cache: wave-uniform, so SGPRs instead of VGPRs, which is what lets
// C2's variant run at 6 waves/SIMD (RT_PACKET_SMALL_WAVES).  More spheres keep the LDS copy
// (C3 +1.2 % through the scalar cache: the chunk masks need those SGPRs).
template <int MAXC>
__device__ __forceinline__ void pk_light_record(const PacketScene& S, const TraceParams& P, int l,
                                                d3& L, d3& E) {
    if constexpr (MAXC == 1) {
        const pk_cdp q = (pk_cdp)P.lt + kLtStride * l;
        L = mk(q[0], q[1], q[2]);
        E = mk(q[3], q[4], q[5]);
    } else {
        const double* q = S.lt + kLtStride * l;
        L = mk(q[0], q[1], q[2]);
        E = mk(q[3], q[4], q[5]);
    }
}

// The packet kernel's LDS image of a scene seen from one camera (layout below, 16-byte
// aligned arrays): spheres, camera-cone terms, culling radii, camera-ray sphere constants,
// planes with their camera numerators, point lights, camera-ray plane normals.  Formed by each
// workgroup into LDS, or once per (scene, camera) into HBM by packet_image_kernel and copied.
// With >= kSphChunkMin spheres the spheres are in spatial-chunk order, each chunk's bounding
// sphere follows them as a pseudo-sphere in the sphere / cone / radius arrays, and the scene
// index of every sorted sphere closes the image.
__host__ __device__ inline int pk_chunk_bounds(int ns) { return ns >= kSphChunkMin ? (ns + 63) / 64 : 0; }
__host__ __device__ inline size_t pk_image_bytes(int ns, int np, int nl) {
    const size_t nsb = static_cast<size_t>(ns) + pk_chunk_bounds(ns);
    const size_t b = sizeof(double) * (static_cast<size_t>(kPkSph) * nsb +
                                       static_cast<size_t>(kPlStride + 4) * np +
                                       static_cast<size_t>(kLtStride) * nl) +
                     (pk_chunk_bounds(ns) ? sizeof(int32_t) * ns : 0);
    return (b + 15) / 16 * 16;
}

__device__ __forceinline__ void pk_build_image(const TraceParams& P, const double* camp,
                                               double* img, int tid, int nthreads) {
    const int ns = P.ns, np = P.np, nl = P.nl, nb = pk_chunk_bounds(ns), nsb = ns + nb;
    double* s_sph = img;                                          // 80·nsb bytes
    double* s_pl = s_sph + kPkSph * nsb;
    double* s_lt = s_pl + kPlStride * np;
    double* s_pln = s_lt + kLtStride * nl;                        // 4·np doubles
    int32_t* s_orig = reinterpret_cast<int32_t*>(s_pln + 4 * np);  // nb > 0 only
    const d3 cam = mk(camp[0], camp[1], camp[2]);
    const int32_t* perm = nb ? P.sph_perm : nullptr;
    for (int i = tid; i < nb; i += nthreads) {  // chunk bounds as pseudo-spheres ns + c
        const double* q = P.sph_bnd + 4 * i;
        double* o = s_sph + kPkSph * (ns + i);
        o[0] = q[0];
        o[1] = q[1];
        o[2] = q[2];
        o[3] = q[3] * q[3];
        o[8] = 0.0;
        o[9] = 0.0;
        cone_terms(o, q[3], cam, reinterpret_cast<float*>(o + 4));
    }
    for (int i = tid; i < ns; i += nthreads) {
        const int si = perm ? perm[i] : i;
        if (perm) s_orig[i] = si;
        const double* s = P.sph + kSphStride * si;
        double* o = s_sph + kPkSph * i;
        o[0] = s[0];
        o[1] = s[1];
        o[2] = s[2];
        o[3] = s[3];
        o[9] = 0.0;
        // culling radius (only ever used with a margin, rounded up to FP32 in cone_terms)
        cone_terms(s, sqrt(s[3]), cam, reinterpret_cast<float*>(o + 4));
        // camera-ray constant of Sphere::Intersect (Shape.h:73,77)
        const d3 oc = cam - mk(s[0], s[1], s[2]);
        o[8] = dot(oc, oc) - s[3];
    }
    for (int i = tid; i < np; i += nthreads) {
        const double* p = P.pl + kPlStride * i;
        double* o = s_pl + kPlStride * i;
        for (int k = 0; k < 6; ++k) o[k] = p[k];
        // camera-ray numerator of Plane::Intersect (Shape.h:152-153)
        o[6] = dot(mk(p[0], p[1], p[2]) - cam, mk(p[3], p[4], p[5]));
        // 1 when camera rays may divide it through the core (plane_t_core)
        const double n1 = fabs(p[3]) + fabs(p[4]) + fabs(p[5]);
        o[7] = fabs(o[6]) >= 0x1p-900 && fabs(o[6]) <= 0x1p400 && n1 <= 0x1p90 ? 1.0 : 0.0;
        // Shading normal of a camera-ray hit on this plane (Scene.h:147-154 then directLightning's
        // normalize, Scene.h:81).  A hit has t = num/denom ≥ 0 with 2^-900 ≤ |num| (no underflow
        // to ±0) and |denom| > 1e-6, so sign(denom) = sign(num); with |n|₁ ≤ 2 both n·d and the
        // reference's n·normalize(d) are within 5ε·|n|₁ ≪ 1e-6 of the exact n·d, so frontFace
        // (n·normalize(d) < 0) is num < 0 for every camera ray that hits the plane, and the
        // normal is unit(num < 0 ? n : −n): the same for the whole frame.
        const d3 pn = mk(p[3], p[4], p[5]);
        const d3 un = unit(o[6] < 0.0 ? pn : -pn);
        double* q = s_pln + 4 * i;
        q[0] = un.x;
        q[1] = un.y;
        q[2] = un.z;
        q[3] = o[7] != 0.0 && n1 <= 2.0 ? 1.0 : 0.0;
    }
    for (int i = tid; i < kLtStride * nl; i += nthreads) s_lt[i] = P.lt[i];

}

// Waves per SIMD of a variant (its register budget).
constexpr int pk_waves(int MAXC, int FEAT, bool COUNT, bool MULTI) {
    return (FEAT == kFeatFix && MAXC == 1 && !MULTI && !COUNT) ? RT_PACKET_FIX_WAVES
         : (FEAT == 0 && MAXC == 1 && !MULTI && !COUNT) ? RT_PACKET_SMALL_WAVES
         : (FEAT == (kFeatArea | kFeatNoPL) && !MULTI && !COUNT) ? RT_PACKET_AREA_WAVES
         : FEAT == kFeatTris ? RT_PACKET_TRIS_WAVES
         : (((FEAT == 0 || (FEAT & ~kFeatNoPL) == kFeatArea || FEAT == kFeatPlanes) && MAXC <= 4)
                ? (MULTI ? (FEAT == 0 ? RT_PACKET_LEAN_WAVES : 1) : RT_PACKET_AA1_WAVES)
                : 1);
}
template <int MAXC, int FEAT, bool COUNT, bool MULTI, int WGY>  // MULTI = false: one sample (AA = 1)
__global__ __launch_bounds__(64 * kWgWavesX * WGY, pk_waves(MAXC, FEAT, COUNT, MULTI)) void packet_direct_kernel(TraceParams P) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int tid = threadIdx.x;
    constexpr bool kNoPL = (FEAT & kFeatNoPL) != 0;  // the launcher checked P.np == P.nl == 0
    // The tile this workgroup renders.  Results do not depend on the order; the tail of the
    // launch does.  Default: rows bottom-up (scenes lit from above put the shadow-ray work on
    // the floor and little on the sky / back wall, so the cheap top rows fill the partly idle
    // end: C3 -9 %, C5 -1 %, C2/C4 within ±1 %; centre-out and edges-in orders measured worse).
    // With a tile order (costliest first, from the wave durations of an earlier launch of this
    // scene, camera and shape: packet_order_kernel) the cheapest tiles fill the end instead.
    const uint32_t lin = blockIdx.y * gridDim.x + blockIdx.x;  // dispatch position
    uint32_t tbx = blockIdx.x, tby = gridDim.y - 1 - blockIdx.y;
    if (P.tile_order) {
        const uint32_t t = P.tile_order[lin];
        tbx = t % gridDim.x;
        tby = t / gridDim.x;
    }
    // the recording launch (the general variant, rt_capi.cpp tile_order): each wave's start
    uint64_t t_start = 0;
    if constexpr (MULTI)
        if (P.tile_cost) t_start = __builtin_amdgcn_s_memrealtime();
    const int ns = P.ns, np = kNoPL ? 0 : P.np, nl = kNoPL ? 0 : P.nl, nb = pk_chunk_bounds(ns),
              nsb = ns + nb;
    double* s_sph = smem;                                         // 80·nsb bytes
    double* s_pl = s_sph + kPkSph * nsb;
    double* s_lt = s_pl + kPlStride * np;
    double* s_pln = s_lt + kLtStride * nl;                        // 4·np doubles
    const int32_t* s_orig = reinterpret_cast<const int32_t*>(s_pln + 4 * np);
    // The frame: one per launch, or frame blockIdx.z of a batch (rt_render_batch) with its own
    // camera and image source (scalar loads from the kernel arguments).
    const double* camp = P.cam_pos;
    const double* pk_img = P.pk_image;
    unsigned long long* pk_pub = P.pk_pub;
    uint32_t pk_epoch = P.pk_epoch;
    uint64_t frame_off = 0;
    if (P.nframes) {
        const PkFrame& F = P.fr[blockIdx.z];
        camp = F.cam;
        pk_img = F.img;
        pk_pub = F.pub;
        pk_epoch = F.epoch;
        frame_off = static_cast<uint64_t>(blockIdx.z) * P.frame_px;
    }
    const d3 cam = mk(camp[0], camp[1], camp[2]);
    constexpr int kThreads = 64 * kWgWavesX * WGY;
    if (pk_img) {  // the image of this scene and camera, formed once (packet_image_kernel)
        const float4* src = reinterpret_cast<const float4*>(pk_img);
        float4* dst = reinterpret_cast<float4*>(smem);
        const int nv = static_cast<int>(pk_image_bytes(ns, np, nl) / 16);
        for (int i = tid; i < nv; i += kThreads) dst[i] = src[i];
        __syncthreads();
    } else if (pk_pub) {
        // A camera without a cached image: the launch's first workgroup forms the image and
        // publishes it as {epoch, word} granules (8-byte agent-scope atomic stores, written
        // through to memory: the tag travels with its word, so no flag and no fence).  The
        // workgroups of the first resident round (linear index < pk_pub_first) form their own
        // and never read the slot, so no XCD's L2 holds a line of it from before the publish;
        // a later workgroup reads the granules with relaxed agent-scope 8-byte atomic loads
        // (each {epoch, word} read whole, as written) and copies them when every tag is this
        // launch's epoch.  A granule with this epoch can only hold this launch's word, so a
        // stale or half-published slot just means "form it".
        uint32_t* dst = reinterpret_cast<uint32_t*>(smem);
        const int nw = static_cast<int>(pk_image_bytes(ns, np, nl) / 4);  // a multiple of 4
        const uint32_t ep = pk_epoch;
        const uint32_t wg = lin;  // in its frame: a batch's frames dispatch one after another
        bool have = false;
        if (wg >= P.pk_pub_first) {
            int ok = 1;
            for (int i = tid; i < nw / 2; i += kThreads) {
                const unsigned long long gx = __hip_atomic_load(
                    pk_pub + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long gy = __hip_atomic_load(
                    pk_pub + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok &= static_cast<uint32_t>(gx >> 32) == ep && static_cast<uint32_t>(gy >> 32) == ep;
                dst[2 * i] = static_cast<uint32_t>(gx);
                dst[2 * i + 1] = static_cast<uint32_t>(gy);
            }
            have = __syncthreads_and(ok) != 0;
        }
        if (!have) {
            pk_build_image(P, camp, smem, tid, kThreads);
            __syncthreads();
            if (wg == 0) {
                const unsigned long long tag = static_cast<unsigned long long>(ep) << 32;
                for (int i = tid; i < nw; i += kThreads)
                    __hip_atomic_store(pk_pub + i, tag | dst[i], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    } else {
        pk_build_image(P, camp, smem, tid, kThreads);
        __syncthreads();
    }

    PacketScene S;
    S.sph = s_sph;
    S.pl = s_pl;
    S.lt = s_lt;
    S.tri = P.tri;
    S.mat = P.sph_mat;
    S.bvh = P.bvh;
    S.bvh_tri = P.bvh_tri;
    S.ns = ns;
    S.np = np;
    S.nt = P.nt;
    S.nl = nl;
    S.nb = nb;
    S.orig = nb ? s_orig : nullptr;
    S.wstk = nullptr;
    if constexpr ((FEAT & kFeatTris) != 0)  // after the image: 64 ints per wave
        S.wstk = reinterpret_cast<int*>(smem + pk_image_bytes(ns, np, nl) / 8) +
                 kPkStack * (tid >> 6);
    constexpr bool kPark = RT_PK_AREA_PARK && (FEAT & kFeatArea) != 0 && MAXC == 1;
    constexpr bool kParkPoint = RT_PK_PARK_POINT && MAXC == 1;
    double* park = nullptr;  // then 6 doubles per lane (stride kThreads)
    if constexpr (kPark || kParkPoint)
        park = smem + pk_image_bytes(ns, np, nl) / 8 +
               ((FEAT & kFeatTris) != 0 ? kPkStack * kThreads / 128 : 0) + tid;
    const int nchunks = (ns + 63) / 64;

    const int lane = tid & 63, wave = tid >> 6;
    const uint32_t x = tbx * (kPkW * kWgWavesX) + (wave % kWgWavesX) * kPkW + (lane % kPkW);
    const uint32_t yl = tby * (kPkH * WGY) + (wave / kWgWavesX) * kPkH + (lane / kPkW);
    const bool valid = x < P.width && yl < P.rows;
    // lanes past the image edge trace a clamped in-image ray: they take part in the packet
    // reductions (a superset bound is still conservative) and write nothing.
    const uint32_t xc = x < P.width ? x : P.width - 1;
    const uint32_t y = image_row(P, yl < P.rows ? yl : P.rows - 1);
    const uint64_t pix = static_cast<uint64_t>(y) * P.width + xc;
    const double bias = P.bias;
    d3 al_c = mk(0.0, 0.0, 0.0);
    double al_r = 0.0;
    if constexpr ((FEAT & kFeatArea) != 0) {
        const d3 eu = mk(P.al_u[0], P.al_u[1], P.al_u[2]);
        const d3 ev = mk(P.al_v[0], P.al_v[1], P.al_v[2]);
        al_c = (mk(P.al_corner[0], P.al_corner[1], P.al_corner[2]) + eu * 0.5) + ev * 0.5;
        al_r = (0.5 * (length(eu) + length(ev))) * (1.0 + kCullRel);
    }
    Counts cnt{0u, 0u};
    bool fix = false;  // kFeatFix: an undecided shadow ray, the pixel goes to the fix-up

    d3 acc = mk(0.0, 0.0, 0.0);
    int samples = 0;
    const int nsamples = MULTI ? P.aa : 1;
    for (int s = 0; s < nsamples; ++s) {
        // Camera::getRay (Math.h:99-121)
        double sx = static_cast<double>(xc) - static_cast<double>(P.width) / 2.0;
        double sy = static_cast<double>(P.height) / 2.0 - static_cast<double>(y);
        double jx = 0.0, jy = 0.0;
        if (s > 0 && P.aa > 1) {
            jx = u01(P.seed, pix, static_cast<uint32_t>(s), 0u);
            jy = u01(P.seed, pix, static_cast<uint32_t>(s), 1u);
        }
        sx += jx;
        sy += jy;
        const d3 d = unit(mk(sx, sy, cam.z + P.focal) - cam);

        d3 col;
        if (P.max_rec <= 0) {
            col = sky(d);  // TraceRay at depth >= maxRecursion (Scene.h:132-134)
        } else {
            if (COUNT && valid) cnt.trace++;
            // camera cone: axis = the tile's centre-lane direction (exact copy), half-angle
            // from the wave minimum of the per-lane cosines in FP32 (|cos| ≤ 1 + 2ε, so the
            // conversion is off by ≤ 6e-8, inside the 1e-7 taken off)
            const d3 axis = lane_d3(d, (kPkH / 2) * kPkW + kPkW / 2);
            const double cos_min =
                static_cast<double>(wave_red<0>(static_cast<float>(dot(d, axis)))) - 1e-7;
            const bool ok = isfinite(cos_min) && cos_min > 0.0;  // cones narrower than 90°
            const Masks<MAXC> M = ok ? cull_cone<MAXC>(S, axis, cos_min)
                                     : all_candidates<MAXC>(ns);
            PkHit h;
            h.t = 0.0;
            h.prim = 0;
            const bool hit = valid && closest_camera<MAXC, FEAT>(S, M, nchunks, cam, d, h);
            // shading inputs (Scene.h:147-154); misses carry harmless placeholders
            const d3 hp = cam + d * h.t;
            // `view` is only read by the Blinn-Phong term.
            d3 view = mk(0.0, 0.0, 0.0);
            d3 inc = mk(0.0, 0.0, 0.0);
            if constexpr ((FEAT & kFeatSpec) != 0) {
                inc = unit(d);
                view = -inc;
            }
            // planes: the frame-constant oriented normal of the prologue (s_pln); misses: unused
            d3 n = mk(0.0, 1.0, 0.0);
            bool known = !hit;
            if (hit && h.prim >= ns && h.prim < ns + np) {
                const double* q = s_pln + 4 * (h.prim - ns);
                if (q[3] != 0.0) {
                    n = mk(q[0], q[1], q[2]);
                    known = true;
                }
            }
            if (!known) {
                const d3 gn = pk_normal(S, h, hp);
                // frontFace = n·normalize(d) < 0 (Scene.h:148-150).  d is a unit vector (or
                // zero), so normalize(d) = d/l·(1+δ) with l = 1 ± 4ε and |δ| ≤ ε; both dot
                // products are within 5ε·S of their exact values, S = Σ|n_i·d_i| — when
                // |n·d| > 1e-14·S they have the same sign, and the second normalize (3
                // divisions) is only needed otherwise.
                bool front;
                if constexpr ((FEAT & kFeatSpec) != 0) {
                    front = dot(gn, inc) < 0.0;
                } else {
                    const double nd = dot(gn, d);
                    const double sabs = fabs(gn.x * d.x) + fabs(gn.y * d.y) + fabs(gn.z * d.z);
                    if (fabs(nd) > 1e-14 * sabs && sabs > 1e-200) front = nd < 0.0;
                    else front = dot(gn, unit(d)) < 0.0;
                }
                const d3 n0 = front ? gn : -gn;
                n = unit(n0);  // directLightning's own normalize (Scene.h:81)
            }
            d3 diff = mk(0.0, 0.0, 0.0), spec = mk(0.0, 0.0, 0.0);
            if constexpr (kParkPoint) {
                park[0 * kThreads] = hp.x;
                park[1 * kThreads] = hp.y;
                park[2 * kThreads] = hp.z;
                park[3 * kThreads] = n.x;
                park[4 * kThreads] = n.y;
                park[5 * kThreads] = n.z;
                __asm__ volatile("" ::: "memory");
            }
            for (int l = 0; l < nl; ++l) {
                d3 L, E;
                pk_light_record<MAXC>(S, P, l, L, E);
                d3 hl = hp, nl_ = n;
                if constexpr (kParkPoint) {
                    __asm__ volatile("" ::: "memory");
                    hl = mk(park[0 * kThreads], park[1 * kThreads], park[2 * kThreads]);
                    nl_ = mk(park[3 * kThreads], park[4 * kThreads], park[5 * kThreads]);
                }
                pk_light<MAXC, FEAT, COUNT>(S, hit, hl, nl_, view, h, L, E, L, 0.0, bias, nchunks,
                                            diff, spec, cnt, nullptr, &fix);
            }
            if constexpr ((FEAT & kFeatArea) != 0) {
                if (P.al_samples > 0) {
                    const uint32_t stream = 0x10000u + (static_cast<uint32_t>(s) << 6);
                    const double k = static_cast<double>(P.al_k);
                    const d3 corner = mk(P.al_corner[0], P.al_corner[1], P.al_corner[2]);
                    const d3 eu = mk(P.al_u[0], P.al_u[1], P.al_u[2]);
                    const d3 ev = mk(P.al_v[0], P.al_v[1], P.al_v[2]);
                    const d3 E = mk(P.al_E[0], P.al_E[1], P.al_E[2]);
                    // one packet cull for all samples: every sample's casting lanes are hit
                    // lanes with this origin, and every sample point is in (al_c, al_r)
                    const OriginBall B = origin_ball(hit, hp + n * bias);
                    if constexpr (kPark) {
                        park[0 * kThreads] = hp.x;
                        park[1 * kThreads] = hp.y;
                        park[2 * kThreads] = hp.z;
                        park[3 * kThreads] = n.x;
                        park[4 * kThreads] = n.y;
                        park[5 * kThreads] = n.z;
                        __asm__ volatile("" ::: "memory");  // no forwarding of the stored values
                    }
                    const Masks<MAXC> Ma = B.ok ? cull_capsule<MAXC, FEAT>(S, B.c, B.R, al_c, al_r, bias)
                                                : all_candidates<MAXC>(ns);
                    // When that leaves many candidates (a wide light seen past many spheres),
                    // each sample gets its own capsule: sample q lies in stratum cell
                    // (q mod k, q div k), a parallelogram of half-diagonal ≤ (|u|+|v|)/2k
                    // around the cell centre (plus an absolute term for the rounding of the
                    // sample and centre positions); its mask is ANDed with the shared one.
                    int cand = 0;
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) cand += __builtin_popcountll(Ma.m[c]);
                    const bool per_cell = B.ok && cand > 4;
                    const double cell_r =
                        ((0.5 * (length(eu) + length(ev))) / k) * (1.0 + kCullRel) +
                        1e-12 * (fabs(corner.x) + fabs(corner.y) + fabs(corner.z) + fabs(eu.x) +
                                 fabs(eu.y) + fabs(eu.z) + fabs(ev.x) + fabs(ev.y) + fabs(ev.z));
                    // the stratum coordinates x / k as div_core with k's refined reciprocal (the
                    // correctly rounded quotient, rt_device.hpp: 0 ≤ x < k + 1, k ≤ 2^31)
                    const double rk = rcp_refined(k);
                    for (int q = 0; q < P.al_samples; ++q) {
                        const double r1 = u01(P.seed, pix, stream, 2u * static_cast<uint32_t>(q));
                        const double r2 =
                            u01(P.seed, pix, stream, 2u * static_cast<uint32_t>(q) + 1u);
                        const double fu = div_core(static_cast<double>(q % P.al_k) + r1, k, rk);
                        const double fv = div_core(static_cast<double>(q / P.al_k) + r2, k, rk);
                        const d3 lpos = (corner + eu * fu) + ev * fv;
                        Masks<MAXC> Mq = Ma;
                        if (per_cell) {  // uniform
                            const double cu = div_core(static_cast<double>(q % P.al_k) + 0.5, k, rk);
                            const double cv = div_core(static_cast<double>(q / P.al_k) + 0.5, k, rk);
                            const Masks<MAXC> Mc = cull_capsule<MAXC, FEAT>(
                                S, B.c, B.R, (corner + eu * cu) + ev * cv, cell_r, bias);
#pragma unroll
                            for (int c = 0; c < MAXC; ++c) Mq.m[c] &= Mc.m[c];
                            Mq.pm &= Mc.pm;
                        }
                        d3 hq = hp, nq = n;
                        if constexpr (kPark) {
                            __asm__ volatile("" ::: "memory");  // read back every sample
                            hq = mk(park[0 * kThreads], park[1 * kThreads], park[2 * kThreads]);
                            nq = mk(park[3 * kThreads], park[4 * kThreads], park[5 * kThreads]);
                        }
                        pk_light<MAXC, FEAT, COUNT>(S, hit, hq, nq, view, h, lpos, E, al_c, al_r,
                                                    bias, nchunks, diff, spec, cnt, &Mq);
                    }
                }
            }
            if (hit) {
                const double* m = pk_material<MAXC>(S, h);
                const d3 local = hmul(mk(m[0], m[1], m[2]), diff) + spec * m[4];
                const double tr = sclamp(m[5], 0.0, 1.0);
                d3 fin = mk(0.0, 0.0, 0.0);
                if (tr < 1.0) fin = fin + local * (1.0 - tr);
                col = fin;
            } else {
                col = sky(d);
            }
        }
        acc = acc + col;
        samples += 1;
    }
    // The pixel again, from the lane id (mbcnt) and the workgroup's tile (scalars): keeping x /
    // yl live across the trace cost the single-sample variants a spilled dword per lane, whose
    // scratch write-back was most of C2's HBM traffic beyond the framebuffer (12 MB per frame).
    const uint32_t lane_e = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const uint32_t wave_e = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(wave));
    const uint32_t x_e = tbx * (kPkW * kWgWavesX) + (wave_e % kWgWavesX) * kPkW + (lane_e % kPkW);
    const uint32_t yl_e = tby * (kPkH * WGY) + (wave_e / kWgWavesX) * kPkH + (lane_e / kPkW);
    bool store = x_e < P.width && yl_e < P.rows;
    if constexpr ((FEAT & kFeatFix) != 0) {
        // the pixels with an undecided shadow ray: appended to the fix-up list (one atomic per
        // wave), rendered by packet_fixup_kernel after this launch instead of stored here
        const bool q = fix && store;
        const uint64_t bq = __ballot(q);
        if (bq) {
            uint32_t base = 0;
            if (lane_e == static_cast<uint32_t>(__builtin_ctzll(bq)))
                base = atomicAdd(P.fix_ctl, static_cast<uint32_t>(__builtin_popcountll(bq)));
            base = __shfl(base, __builtin_ctzll(bq), 64);
            if (q)
                P.fix_list[base + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bq >> 32),
                                                            __builtin_amdgcn_mbcnt_lo(
                                                                static_cast<uint32_t>(bq), 0u))] =
                    static_cast<uint32_t>(frame_off + static_cast<size_t>(yl_e) * P.width + x_e);
        }
        store = store && !fix;
    }
    if (store) {
        // accumulated / samples (Scene.h:298-300); x / 1.0 == x, so AA=1 skips the division
        const d3 v = samples == 1 ? acc
                   : (samples > 0 ? sdiv(acc, static_cast<double>(samples)) : mk(0.0, 0.0, 0.0));
        const size_t o = frame_off + static_cast<size_t>(yl_e) * P.width + x_e;
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
            if (P.tonemap == 1) {  // uniform: Reinhard, through the FP32 byte decision
                r = reinhard_byte(v.x);
                g = reinhard_byte(v.y);
                b = reinhard_byte(v.z);
            } else if constexpr ((FEAT & kFeatJodie) != 0) {
                to_color(tonemap_op(v, P.tonemap), r, g, b);
            } else {
                to_color(tonemap_op_nolog(v, P.tonemap), r, g, b);
            }
            P.ldr[3 * o + 0] = r;
            P.ldr[3 * o + 1] = g;
            P.ldr[3 * o + 2] = b;
        }
    }
    if constexpr (COUNT) {
        uint32_t t = cnt.trace, sh = cnt.shadow;
        for (int off = 32; off > 0; off >>= 1) {
            t += __shfl_xor(t, off, 64);
            sh += __shfl_xor(sh, off, 64);
        }
        if (lane == 0) {
            atomicAdd(P.counters + 0, static_cast<unsigned long long>(t));
            atomicAdd(P.counters + 1, static_cast<unsigned long long>(sh));
        }
    }
    if constexpr (MULTI) {
        // this wave's duration (100 MHz wall clock), per tile (a batch records its first frame)
        if (P.tile_cost && lane == 0 && blockIdx.z == 0) {
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
            P.tile_cost[(tby * gridDim.x + tbx) * (kWgWavesX * WGY) + wave] =
                static_cast<uint32_t>(t_end - t_start);
        }
    }
}

#ifdef RT_PACKET_PROBE
// tools/isa/probe.sh: one instantiation only (register / ISA studies of a single variant)
template __global__ void packet_direct_kernel<RT_PACKET_PROBE>(TraceParams);
#else
#ifndef RT_PACKET_AREA_TU
size_t packet_lds_bytes(int ns, int np, int nl) { return pk_image_bytes(ns, np, nl); }

__global__ __launch_bounds__(256) void packet_image_kernel(TraceParams P, double* img) {
    pk_build_image(P, P.cam_pos, img, static_cast<int>(threadIdx.x), 256);
}

hipError_t launch_packet_image(const TraceParams& p, double* img, hipStream_t stream) {
    hipLaunchKernelGGL(packet_image_kernel, dim3(1), dim3(256), 0, stream, p, img);
    return hipGetLastError();
}

// The images of a frame batch's uncached cameras, one workgroup per job (pk_build_image: the
// same words a workgroup of the batch launch would form for itself), each written where the
// host put it: a new cache entry (a camera seen before) or the batch's ring slot.
__global__ __launch_bounds__(256) void packet_image_batch_kernel(TraceParams P, PkImageJobs J) {
    const int f = J.frame[blockIdx.x];
    pk_build_image(P, P.fr[f].cam, J.dst[blockIdx.x], static_cast<int>(threadIdx.x), 256);
}

hipError_t launch_packet_image_batch(const TraceParams& p, const PkImageJobs& jobs,
                                     hipStream_t stream) {
    if (jobs.n <= 0) return hipSuccess;
    if (jobs.n > kPkMaxBatch) return hipErrorInvalidValue;
    for (int j = 0; j < jobs.n; ++j)
        if (!jobs.dst[j] || jobs.frame[j] < 0 || jobs.frame[j] >= static_cast<int>(p.nframes))
            return hipErrorInvalidValue;
    hipLaunchKernelGGL(packet_image_batch_kernel, dim3(static_cast<unsigned>(jobs.n)),
                       dim3(256), 0, stream, p, jobs);
    return hipGetLastError();
}

// The pixels a fix-up variant queued (TraceParams.fix_list: output index frame · frame_px + row-
// local pixel): GeneratePixelAt (Scene.h:283-304) with one sample through the per-pixel path —
// generic closest hit over every primitive, occlusion_opaque and the exact computeTransmittance
// march (rt_trace_common.hpp trace_direct) — the same image bits as the packet kernel, stored
// like it.  A persistent grid over the device-side count; it zeroes the count the next
// fix-variant launch uses (the two alternate, no memset on the stream), and workgroups past
// the list return before staging.  The scene records are staged into LDS when
// they fit.  Its cost is per wave, ~2 300 VALU + 1 100 SALU (~45k cycles) each: one wave per
// 64 queued pixels is the fastest arrangement — 16, 8 or 4 pixels per wave (more waves per SIMD)
// took 75 / 152 / 334 µs against 26 µs per 32-frame C2 batch, lanes of a group sharing one
// pixel's sphere loops 42 µs, a per-ray capsule mask for the marches no change
// (profiles/r05_ab_fixup.txt).
constexpr int kFixThreads = 256;
constexpr int kFixBlocks = 256;
template <bool LDS>
__global__ __launch_bounds__(kFixThreads) void packet_fixup_kernel(TraceParams P) {
    extern __shared__ double smem[];
    const uint32_t n = *P.fix_ctl;  // the packet launch before this one on the stream appended
    // the count the context's next fix-variant launch appends to: zeroed here, where nothing
    // reads it (the launch before this one's fix-up read it, and the next packet launch is
    // ordered after this one) — round 6: replaces 256 same-address completion atomics and
    // fences (the launch's floor, profiles/r06_fixup_ab.txt)
    if (blockIdx.x == 0 && threadIdx.x == 0) *P.fix_next = 0u;
    // workgroups past the list skip the scene staging (uniform per workgroup)
    if (blockIdx.x * kFixThreads >= n) return;
    // the fix-up variants' scenes: spheres, planes and point lights, no specular material, so
    // no triangle, BVH, area-light or pow code is compiled in (229 -> 167 VGPRs, 288 -> 40 B of
    // scratch: 27.5 -> 26 µs per 32-frame batch)
    SceneView S = stage_scene<LDS>(P, smem, threadIdx.x, kFixThreads);
    S.nt = 0;
    S.al = 0;
    S.spec = false;
    S.tri = S.tri_mat = S.bvh = nullptr;
    S.bvh_tri = nullptr;
    Counts cnt{0u, 0u};
    // (list entries are 32-bit output indices: the launch's pixels are < 2^32, fixup_buffers)
    const uint32_t fpx = P.nframes ? static_cast<uint32_t>(P.frame_px) : 0u;
    for (uint32_t i = blockIdx.x * kFixThreads + threadIdx.x; i < n; i += gridDim.x * kFixThreads) {
        const uint32_t o = P.fix_list[i];
        const uint32_t z = fpx ? o / fpx : 0u;
        const uint32_t pl = o - z * fpx;
        const uint32_t yl = pl / P.width;
        const uint32_t x = pl - yl * P.width;
        const double* cp = P.nframes ? P.fr[z].cam : P.cam_pos;
        const d3 cam = mk(cp[0], cp[1], cp[2]);
        const uint32_t y = image_row(P, yl);
        const uint64_t pix = static_cast<uint64_t>(y) * P.width + x;
        const d3 d = camera_dir(P, cam, x, y, pix, 0);
        d3 acc = mk(0.0, 0.0, 0.0);
        acc = acc + trace_direct<false>(S, P, cam, d, pix, 0u, cnt);  // one sample (AA = 1)
        store_pixel(P, static_cast<size_t>(o), acc);
    }
}

hipError_t launch_packet_fixup(const TraceParams& p, hipStream_t stream) {
    if (!p.fix_list || !p.fix_ctl || !p.fix_next) return hipErrorInvalidValue;
    if (p.nt != 0 || p.al_samples != 0) return hipErrorInvalidValue;  // the lean scene view
    const size_t lds = sizeof(double) * scene_doubles(p);
    if (lds <= 32 * 1024)
        hipLaunchKernelGGL(packet_fixup_kernel<true>, dim3(kFixBlocks), dim3(kFixThreads), lds,
                           stream, p);
    else
        hipLaunchKernelGGL(packet_fixup_kernel<false>, dim3(kFixBlocks), dim3(kFixThreads), 0,
                           stream, p);
    return hipGetLastError();
}

int packet_max_spheres() { return 16 * 64; }

void packet_grid(const TraceParams& p, uint32_t& gx, uint32_t& gy, uint32_t& waves) {
    const size_t lds = pk_image_bytes(p.ns, p.np, p.nl);
    const uint32_t wgy = 10 * lds <= kLdsPerCu ? 1u : 2u;  // launch_packet_variant's choice
    gx = (p.width + kPkW * kWgWavesX - 1) / (kPkW * kWgWavesX);
    gy = (p.rows + kPkH * wgy - 1) / (kPkH * wgy);
    waves = kWgWavesX * wgy;
}

// Costliest tiles first: the tile order of the next launches from the wave durations one launch
// recorded (tile_cost, `waves` per tile).  One workgroup: a tile's cost is its slowest wave's
// (a workgroup holds its slots until then), binned into 16 levels of the largest cost; the bins
// are dispatched costliest first, and inside a bin the tiles keep the default (bottom-up) order,
// so tiles of similar cost stay spatially together (a fully cost-sorted order was 3.6 % slower on
// C2, whose tiles cost nearly the same).  Every key is read once and kept (`keys`), so the
// output is a permutation of the tiles even if another launch rewrites the costs meanwhile.
constexpr int kOrderBins = 16;
__global__ __launch_bounds__(1024) void packet_order_kernel(const uint32_t* cost, uint32_t gx,
                                                            uint32_t gy, uint32_t waves,
                                                            uint32_t* keys, uint32_t* order,
                                                            uint32_t* verdict) {
    __shared__ uint32_t s_max, s_cnt[kOrderBins];
    const uint32_t tid = threadIdx.x, tiles = gx * gy;
    if (tid == 0) s_max = 0;
    if (tid < kOrderBins) s_cnt[tid] = 0;
    __syncthreads();
    uint32_t m = 0;
    for (uint32_t i = tid; i < tiles; i += blockDim.x) {
        uint32_t c = 0;
        for (uint32_t w = 0; w < waves; ++w) c = max(c, cost[i * waves + w]);
        keys[i] = c;
        m = max(m, c);
    }
    atomicMax(&s_max, m);
    __syncthreads();
    const uint64_t top = static_cast<uint64_t>(s_max) + 1;
    for (uint32_t i = tid; i < tiles; i += blockDim.x) {
        const uint64_t bin = static_cast<uint64_t>(keys[i]) * kOrderBins / top;  // < kOrderBins
        const uint32_t key = kOrderBins - 1 - static_cast<uint32_t>(bin);        // 0: costliest
        keys[i] = key;
        atomicAdd(&s_cnt[key], 1u);
    }
    __syncthreads();
    if (tid >= 64) return;
    // Narrow distributions keep the default order: when the median tile costs at least a
    // quarter of the costliest (C2: ~0.4), costliest-first was slower (C2 +3 %, MI355X); wide
    // ones (C3-C5: a few tiles at 10-35x the median) gain 4-10 %.
    uint32_t acc = 0;
    int median_bin = 0;  // cost bin (0 cheapest) holding the median tile
    for (int b = kOrderBins - 1; b >= 0; --b) {  // keys from cheapest (kOrderBins - 1) up
        acc += s_cnt[b];
        if (2 * acc >= tiles) {
            median_bin = kOrderBins - 1 - b;
            break;
        }
    }
    const bool narrow = median_bin >= kOrderBins / 4;
    // for the host (pinned memory): 1 = narrow, launches keep the default order without even
    // reading the table (its per-workgroup load cost C2 3 %); 2 = dispatch by the table
    if (tid == 0 && verdict) __hip_atomic_store(verdict, narrow ? 1u : 2u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_SYSTEM);
    // one wave scatters the tiles in default dispatch order (bottom-up rows), stably per bin:
    // lane b < kOrderBins holds bin b's cursor
    uint32_t cur = 0;
    for (int b = 0; b < kOrderBins; ++b)
        if (static_cast<int>(tid) > b) cur += s_cnt[b];
    if (narrow) {
        for (uint32_t lin = tid; lin < tiles; lin += 64) order[lin] = (gy - 1 - lin / gx) * gx + lin % gx;
        return;
    }
    const uint64_t below = (1ull << tid) - 1ull;
    for (uint32_t c0 = 0; c0 < tiles; c0 += 64) {
        const uint32_t lin = c0 + tid;
        const bool ok = lin < tiles;
        uint32_t tile = 0, key = kOrderBins;
        if (ok) {
            tile = (gy - 1 - lin / gx) * gx + lin % gx;
            key = keys[tile];
        }
        for (int b = 0; b < kOrderBins; ++b) {
            const uint64_t mk_ = __ballot(key == static_cast<uint32_t>(b));
            if (!mk_) continue;  // uniform
            const uint32_t base = __builtin_amdgcn_readlane(cur, b);
            if (key == static_cast<uint32_t>(b))
                order[base + __builtin_popcountll(mk_ & below)] = tile;
            if (static_cast<int>(tid) == b) cur += __builtin_popcountll(mk_);
        }
    }
}

hipError_t launch_packet_order(const uint32_t* cost, uint32_t gx, uint32_t gy, uint32_t waves,
                               uint32_t* keys, uint32_t* order, uint32_t* verdict,
                               hipStream_t stream) {
    hipLaunchKernelGGL(packet_order_kernel, dim3(1), dim3(1024), 0, stream, cost, gx, gy, waves,
                       keys, order, verdict);
    return hipGetLastError();
}
#endif


template <int MAXC, int FEAT, int WGY>
static void launch_packet_shape(const TraceParams& p, bool count, size_t lds, hipStream_t stream) {
    const dim3 block(64 * kWgWavesX * WGY);
    const dim3 grid((p.width + kPkW * kWgWavesX - 1) / (kPkW * kWgWavesX),
                    (p.rows + kPkH * WGY - 1) / (kPkH * WGY), p.nframes ? p.nframes : 1u);
    // the single-sample variant keeps no accumulator live across the trace (AA = 1, the
    // reference default for a preview and the bench's configuration); counting passes use the
    // general one
    // (a launch that records its wave durations for the tile order takes the general variant:
    // the single-sample one carries no recording code)
    if constexpr ((FEAT & kFeatTris) != 0) lds += sizeof(int) * kPkStack * (block.x / 64);
    if constexpr ((RT_PK_AREA_PARK && (FEAT & kFeatArea) != 0 && MAXC == 1) ||
                  (RT_PK_PARK_POINT && MAXC == 1))
        lds += 6 * sizeof(double) * block.x;
    if (count) hipLaunchKernelGGL((packet_direct_kernel<MAXC, FEAT, true, true, WGY>), grid, block, lds, stream, p);
    else if (p.aa == 1 && !p.tile_cost) hipLaunchKernelGGL((packet_direct_kernel<MAXC, FEAT, false, false, WGY>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((packet_direct_kernel<MAXC, FEAT, false, true, WGY>), grid, block, lds, stream, p);
}

template <int MAXC, int FEAT>
static void launch_packet_variant(const TraceParams& p, bool count, size_t lds, hipStream_t stream) {
    if (10 * lds <= kLdsPerCu) launch_packet_shape<MAXC, FEAT, 1>(p, count, lds, stream);
    else launch_packet_shape<MAXC, FEAT, 2>(p, count, lds, stream);
}

#ifdef RT_PACKET_AREA_TU
// rt_packet_area.hip: the area-light variants, in their own translation unit so that they are
// scheduled with the compiler's default strategy (C5 -2 % against max-ilp, which the other
// variants keep).
hipError_t launch_packet_area(const TraceParams& p, bool count, size_t lds, int chunks,
                              hipStream_t stream) {
    if (p.np == 0 && p.nl == 0 && chunks <= 1)
        launch_packet_variant<1, kFeatArea | kFeatNoPL>(p, count, lds, stream);
    else if (chunks <= 1) launch_packet_variant<1, kFeatArea>(p, count, lds, stream);
    else if (chunks <= 4) launch_packet_variant<4, kFeatArea>(p, count, lds, stream);
    else launch_packet_variant<16, kFeatArea>(p, count, lds, stream);
    return hipGetLastError();
}
#else
hipError_t launch_packet_area(const TraceParams& p, bool count, size_t lds, int chunks,
                              hipStream_t stream);

template <int MAXC>
static void launch_packet_maxc(const TraceParams& p, bool count, size_t lds, int feat,
                               hipStream_t stream) {
    // compiled feature sets: lean (the BASELINE C2-C4 shape), lean + plane culls (C3), lean +
    // area light (C5, rt_packet_area.hip), triangles / models only (no Blinn-Phong, area light
    // or Reinhard-Jodie), and everything
    if (feat == kFeatFix) launch_packet_variant<1, kFeatFix>(p, count, lds, stream);
    else if (feat == 0) launch_packet_variant<MAXC, 0>(p, count, lds, stream);
    else if (feat == kFeatPlanes) launch_packet_variant<MAXC, kFeatPlanes>(p, count, lds, stream);
    else if (feat == kFeatTris) launch_packet_variant<MAXC, kFeatTris>(p, count, lds, stream);
    else launch_packet_variant<MAXC, kFeatAll>(p, count, lds, stream);
}

static int packet_features(const TraceParams& p, bool any_specular) {
    int feat = 0;
    if (any_specular) feat |= kFeatSpec;
    if (p.al_samples > 0) feat |= kFeatArea;
    if (p.nt > 0) feat |= kFeatTris;
    if (p.ldr && p.tonemap == 4) feat |= kFeatJodie;
    // the plane cull has its own lean variant; combined with other features the general one
    if (p.np >= 3 && feat == 0) feat = kFeatPlanes;
    return feat;
}

// The fix-up variant serves the single-sample, ≤ 64-sphere, no-feature launches (C2) of frame
// batches that neither count rays nor record tile costs, when the launch is large enough to pay
// for its fix-up launch: that launch costs ~25 µs whatever it holds (one wave's serial generic
// pixel), the march-free packet kernel saves ~1 ns per pixel (C2: 37.8 → 35.7 µs per 1080p
// frame), so the break-even is ~25 M pixels per launch — kPkFixMinPixels (≈ 15 1080p frames)
// leaves a margin: a 32-frame batch takes it, an 8-frame one or one rank's rows of a 4- or
// 8-rank split keep the marching variant (profiles/r05_ab_fixup.txt).  RTAMD_PK_FIX=0: the
// marching variant everywhere, =1: the fix-up variant for every eligible batch (tests, A/B).
constexpr uint64_t kPkFixMinPixels = 32ull << 20;
bool packet_uses_fixup(const TraceParams& p, bool count, bool any_specular) {
    const char* e = std::getenv("RTAMD_PK_FIX");  // read per launch (tests switch it)
    const int mode = e ? std::atoi(e) : -1;
    if (mode == 0) return false;
    const bool eligible = !count && p.aa == 1 && !p.tile_cost && p.nframes >= 1 &&
                          (p.ns + 63) / 64 <= 1 && packet_features(p, any_specular) == 0;
    const uint64_t px = static_cast<uint64_t>(p.nframes) * p.rows * p.width;
    return eligible && (mode == 1 || px >= kPkFixMinPixels);
}

hipError_t launch_packet_direct(const TraceParams& p, bool count, bool any_specular,
                                hipStream_t stream) {
    const size_t lds = packet_lds_bytes(p.ns, p.np, p.nl);
    const int chunks = (p.ns + 63) / 64;
    int feat = packet_features(p, any_specular);
    if (packet_uses_fixup(p, count, any_specular)) {
        if (!p.fix_list || !p.fix_ctl || !p.fix_next) return hipErrorInvalidValue;
        feat = kFeatFix;
    }
    // the area-light variants live in rt_packet_area.hip (compiled with the default scheduler)
    if (feat == kFeatArea) return launch_packet_area(p, count, lds, chunks, stream);
    if (chunks <= 1) launch_packet_maxc<1>(p, count, lds, feat, stream);
    else if (chunks <= 4) launch_packet_maxc<4>(p, count, lds, feat, stream);
    else launch_packet_maxc<16>(p, count, lds, feat, stream);
    return hipGetLastError();
}

#endif  // RT_PACKET_AREA_TU
#endif  // RT_PACKET_PROBE
}  // namespace rtamd
