// rt_device.hpp — gfx950 device-side FP64 vector math for the trace kernels.
//
// Every helper evaluates in the same operation order as the reference's Vec3
// (/root/reference/RaytracingEngine/Math.h:9-71), and the whole library is compiled with
// -ffp-contract=off (and the pragma below), so no multiply-add is fused and every rounding
// matches the reference's x86-64 SSE2 build.  Device double division and sqrt lower to the
// correctly rounded gfx950 sequences (pinned by tests/test_gpu_parity.py::test_device_libm).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace rtamd {

struct d3 {
    double x, y, z;
};

__device__ __forceinline__ d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ d3 operator+(d3 a, d3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ d3 operator-(d3 a, d3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ d3 operator*(d3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ d3 operator-(d3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ d3 hmul(d3 a, d3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ d3 hdiv(d3 a, d3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
__device__ __forceinline__ d3 sdiv(d3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ d3 sadd(d3 a, double s) { return {a.x + s, a.y + s, a.z + s}; }
__device__ __forceinline__ d3 ssub(d3 a, double s) { return {a.x - s, a.y - s, a.z - s}; }
// Vec3::dot — ((x*x' + y*y') + z*z')
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ d3 cross(d3 a, d3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double length(d3 a) { return sqrt(dot(a, a)); }

// ------------------------------------------------------------------ exact sqrt / division cores
// gfx950 lowers the correctly rounded FP64 sqrt and division to Newton-Raphson cores wrapped in
// range scaling and special-case fix-ups:
//   sqrt(x): x < 2^-767 ? scale by 2^256; v_rsq r; g = x·r; h = r·0.5; e = fma(−h, g, 0.5);
//            g = fma(g, e, g); h = fma(h, e, h); 2× { e = fma(−g, g, x); g = fma(e, h, g) };
//            unscale by 2^-128; x ∈ {±0, +inf} ? x : g                       (17 VALU)
//   n / d:   v_div_scale (d), v_div_scale (n); v_rcp r; 2× { e = fma(−d, r, 1); r = fma(r, e, r) };
//            q = n·r; e = fma(−d, q, n); v_div_fmas(e, r, q); v_div_fixup       (11 VALU)
// For operands inside the ranges below every scale step is the identity (v_div_scale returns
// its operand with VCC = 0, so v_div_fmas is a plain FMA) and every fix-up returns the core's
// value, so the cores alone are the same instructions on the same values: the same bits, in
// 10 and 8 VALU.  The reciprocal refinement depends on d only, so a vector divided by one
// scalar shares it (3 VALU per further component).  Ranges (V_DIV_SCALE_F64 scales when
// exp(n) ≤ 53 biased, i.e. |n| < 2^-969, when d or 1/d or n/d is subnormal, or when
// exp(n) − exp(d) ≥ 768; the sqrt lowering scales below 2^-767):
//   sqrt_core(x):          finite x ≥ 2^-767
//   div_core(n, d, r(d)):  2^-900 ≤ |n|, 2^-400 ≤ |d| ≤ 2^400, |n/d| ≥ 2^-1000, all finite
// Every caller checks its operands and takes the compiler's exact lowering otherwise; the
// equality is pinned bit for bit by tests/test_gpu_parity.py::test_fast_exact_cores.
__device__ __forceinline__ double sqrt_core(double x) {
    double r = __builtin_amdgcn_rsq(x);
    double g = x * r;
    double h = r * 0.5;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    g = fma(d, h, g);
    return g;
}
__device__ __forceinline__ double rcp_refined(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    return r;
}
__device__ __forceinline__ double div_core(double n, double d, double r) {
    const double q = n * r;
    const double e = fma(-d, q, n);
    return fma(e, r, q);
}
// sqrt(dot(a, a)) with the dot product in the normalize range [2^-78, 2^120]: the length is in
// [2^-39, 2^60] (> 1e-12), and components with |c| ≥ 2^-900 divide by it exactly in div_core.
constexpr double kUnitLo = 0x1p-78, kUnitHi = 0x1p120, kNumLo = 0x1p-900;
__device__ __forceinline__ bool unit_fast_ok(d3 a, double x) {
    return x >= kUnitLo && x <= kUnitHi && fabs(a.x) >= kNumLo && fabs(a.y) >= kNumLo &&
           fabs(a.z) >= kNumLo;
}

// Vec3::normalize: zero vector below 1e-12, otherwise three true divisions.
// x / 1.0 == x exactly (IEEE), so an already-unit vector skips its three divisions.
__device__ __forceinline__ d3 unit_exact(d3 a) {
    const double l = length(a);
    if (l <= 1e-12) return {0.0, 0.0, 0.0};
    if (l == 1.0) return a;
    return sdiv(a, l);
}
// The same bits through the cores when the operands allow it (zero components, e.g. axis-
// aligned normals, take the exact path unless the length is exactly 1).
__device__ __forceinline__ d3 unit(d3 a) {
    const double x = dot(a, a);
    d3 out;
    if (x >= kUnitLo && x <= kUnitHi) {
        const double l = sqrt_core(x);
        if (l == 1.0) {
            out = a;
        } else if (fabs(a.x) >= kNumLo && fabs(a.y) >= kNumLo && fabs(a.z) >= kNumLo) {
            const double r = rcp_refined(l);
            out = mk(div_core(a.x, l, r), div_core(a.y, l, r), div_core(a.z, l, r));
        } else {
            out = sdiv(a, l);
        }
    } else {
        const double l = sqrt(x);
        out = l <= 1e-12 ? mk(0.0, 0.0, 0.0) : (l == 1.0 ? a : sdiv(a, l));
    }
    return out;
}
// directLightning's light vector (Scene.h:87-90, 110): dist = v.length(), L = v / dist and
// 1 / (dist·dist), through the cores when the operands allow it.  L is only meaningful for
// dist > 0 (the reference skips the light otherwise).
__device__ __forceinline__ void light_dir(d3 v, double& dist, d3& L, double& inv_d2) {
    const double x = dot(v, v);
    if (unit_fast_ok(v, x)) {
        dist = sqrt_core(x);
        const double r = rcp_refined(dist);
        L = mk(div_core(v.x, dist, r), div_core(v.y, dist, r), div_core(v.z, dist, r));
        const double dd = dist * dist;  // in [2^-78, 2^120]
        inv_d2 = div_core(1.0, dd, rcp_refined(dd));
    } else {
        dist = sqrt(x);
        L = sdiv(v, dist);
        inv_d2 = 1.0 / (dist * dist);
    }
}

// std::pow for the Blinn-Phong factor (Scene.h:119: pow(N·H, shininess), N·H in (0, 1]).  The
// libm pow (ocml) carries log and exp in double-double to be within 1 ulp for every input: 214
// VALU, and inlined into the light loop it raises the trace kernels' register budget by ~60
// VGPRs.  Here ln(x) = e·ln2 + 2·atanh(s), s = (m−1)/(m+1) with m in [√½, √2) (series to s^23),
// exp by k·ln2 + r reduction and a degree-13 Taylor polynomial, explicit FMAs: ~90 VALU, with an
// ABSOLUTE error ≤ 2e-16 on results in [0, 1] (the relative error grows like |y·ln x|·ε on
// results that shrink like e^(y·ln x)); images move by ≤ 1e-15, inside the 1e-12 bar the parity
// tests hold libm-pow scenes to.  Inputs outside x ∈ (0, 1.5), |y| ≤ 2^60 (none in a trace: N·H
// is in (0, 1 + 4ε]) call the libm pow out of line.
__device__ __noinline__ double pow_libm(double x, double y) { return pow(x, y); }

// An FP64 constant materialized into an SGPR pair at its point of use (two s_mov_b32 that the
// compiler may not hoist).  gfx950 VALU instructions take no 64-bit literal, so the compiler
// keeps every FP64 constant of a loop body in registers for the whole loop; in a reflection
// chain that is pow_bp's 26 polynomial constants, 36 VGPRs held across every level (rt_box.hip:
// 167 -> 131 VGPRs).  Same value, same bits: only where it is formed changes.
template <uint64_t B>
__device__ __forceinline__ double kc_bits() {
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3"
                 : "=s"(lo), "=s"(hi)
                 : "i"(static_cast<uint32_t>(B)), "i"(static_cast<uint32_t>(B >> 32)));
    return __hiloint2double(static_cast<int>(hi), static_cast<int>(lo));
}
#define RT_KC(x) ::rtamd::kc_bits<__builtin_bit_cast(uint64_t, static_cast<double>(x))>()

// KC: form the polynomial constants at their use (kc_bits) instead of as hoistable literals.
template <bool KC = false>
__device__ __forceinline__ double pow_bp_t(double x, double y) {
#define RT_PC(v) (KC ? RT_KC(v) : static_cast<double>(v))
    if (!(x > 0.0 && x < 1.5 && fabs(y) <= 0x1p60)) return pow_libm(x, y);
    int e;
    double m = frexp(x, &e);
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e -= 1;
    }
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    double p = RT_PC(1.0 / 23.0);
    p = fma(p, s2, RT_PC(1.0 / 21.0));
    p = fma(p, s2, RT_PC(1.0 / 19.0));
    p = fma(p, s2, RT_PC(1.0 / 17.0));
    p = fma(p, s2, RT_PC(1.0 / 15.0));
    p = fma(p, s2, RT_PC(1.0 / 13.0));
    p = fma(p, s2, RT_PC(1.0 / 11.0));
    p = fma(p, s2, RT_PC(1.0 / 9.0));
    p = fma(p, s2, RT_PC(1.0 / 7.0));
    p = fma(p, s2, RT_PC(1.0 / 5.0));
    p = fma(p, s2, RT_PC(1.0 / 3.0));
    const double ln_m = fma(2.0 * (s * s2), p, 2.0 * s);
    const double ed = static_cast<double>(e);
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double ln_x = fma(ed, RT_PC(kLn2Hi), fma(ed, RT_PC(kLn2Lo), ln_m));
    const double z = y * ln_x;
    if (z < -1500.0) return 0.0;  // e^z below the subnormal range (and k fits an int below)
    if (z > 1500.0) return INFINITY;
    const double kd = rint(z * RT_PC(0x1.71547652b82fep0));
    double r = fma(-kd, RT_PC(kLn2Hi), z);
    r = fma(-kd, RT_PC(kLn2Lo), r);
    double q = RT_PC(1.0 / 6227020800.0);
    q = fma(q, r, RT_PC(1.0 / 479001600.0));
    q = fma(q, r, RT_PC(1.0 / 39916800.0));
    q = fma(q, r, RT_PC(1.0 / 3628800.0));
    q = fma(q, r, RT_PC(1.0 / 362880.0));
    q = fma(q, r, RT_PC(1.0 / 40320.0));
    q = fma(q, r, RT_PC(1.0 / 5040.0));
    q = fma(q, r, RT_PC(1.0 / 720.0));
    q = fma(q, r, RT_PC(1.0 / 120.0));
    q = fma(q, r, RT_PC(1.0 / 24.0));
    q = fma(q, r, RT_PC(1.0 / 6.0));
    q = fma(q, r, 0.5);
    q = fma(q, r, 1.0);
    q = fma(q, r, 1.0);
    return ldexp(q, static_cast<int>(kd));
#undef RT_PC
}
__device__ __forceinline__ double pow_bp(double x, double y) { return pow_bp_t<true>(x, y); }

// std::max / std::min / std::clamp with libstdc++'s comparison order (NaN handling).
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }
__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double sclamp(double v, double lo, double hi) {
    return (v < lo) ? lo : (hi < v) ? hi : v;
}
// Vec3::reflect: this - (n * 2.0) * dot(this, n)
__device__ __forceinline__ d3 reflect(d3 i, d3 n) { return i - (n * 2.0) * dot(i, n); }
// Vec3::refract (Math.h:43-52)
__device__ __forceinline__ d3 refract(d3 v, d3 n, double eta) {
    const d3 I = unit(v);
    const d3 N = unit(n);
    const double cosi = sclamp(dot(I, N), -1.0, 1.0);
    const double k = 1.0 - eta * eta * (1.0 - cosi * cosi);
    if (k < 0.0) return {0.0, 0.0, 0.0};
    return I * eta - N * (eta * cosi + sqrt(k));
}

// Build-defined counter RNG (the reference's jitter is an unseeded mt19937, Math.h:109-112).
// Identical integer arithmetic to oracle_u01 (oracle/rt_oracle.c) and rtamd::jitter_u01
// (api/rtamd/math.hpp), so AA>1 and area-light renders are reproducible.  Per pixel one 64-bit
// splitmix64 finalizer of (seed, pixel) folded to a 32-bit key; per (key, stream) and per draw
// one 32-bit finalizer each (lowbias32: x ^= x >> 16, ×0x7feb352d, x ^= x >> 15, ×0x846ca68b,
// x ^= x >> 16 — a bijection of 2^32 with full avalanche).  A draw is h·2^-32 ∈ [0, 1) (32-bit
// resolution).  Round 6: this replaced two 64-bit finalizers per draw (eight 64-bit multiplies,
// 32 quarter-rate 32-bit multiplies on the VALU): the key and the stream's key are loop
// invariants of a pixel's sample loops, so a draw costs two 32-bit multiplies.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t pixel_key(uint64_t seed, uint64_t pixel) {
    const uint64_t k = mix64(seed ^ (0x9E3779B97F4A7C15ULL * (pixel + 1ULL)));
    return static_cast<uint32_t>(k ^ (k >> 32));
}
__device__ __forceinline__ uint32_t stream_key(uint32_t key, uint32_t stream) {
    return hash32(key ^ (stream * 0x9E3779B9U));
}
__device__ __forceinline__ double u01_skey(uint32_t skey, uint32_t index) {
    return static_cast<double>(hash32(skey + index * 0x85EBCA6BU)) * 0x1.0p-32;
}
__device__ __forceinline__ double u01(uint64_t seed, uint64_t pixel, uint32_t stream,
                                      uint32_t index) {
    return u01_skey(stream_key(pixel_key(seed, pixel), stream), index);
}

// Sky colour, Scene::backgroundColor (Scene.h:30-33), in two steps: its blend weight (the only
// thing it needs of the direction) and the colour from it.
__device__ __forceinline__ double sky_weight(d3 dir) { return 0.5 * (unit(dir).y + 1.0); }
__device__ __forceinline__ d3 sky_color(double t) {
    return mk(1.0, 1.0, 1.0) * (1.0 - t) + mk(0.5, 0.7, 1.0) * t;
}
__device__ __forceinline__ d3 sky(d3 dir) { return sky_color(sky_weight(dir)); }

// ------------------------------------------------------------------ tonemap operators
// RaytracingEngine.cpp:70-174.  Float literals are float-rounded then promoted, and the
// products/quotients of two float constants are formed in float, exactly as the reference.
__device__ __forceinline__ d3 clamp3(d3 v, double lo, double hi) {
    return {smin(hi, smax(lo, v.x)), smin(hi, smax(lo, v.y)), smin(hi, smax(lo, v.z))};
}
__device__ __forceinline__ d3 uncharted2_partial(d3 x) {
    const float A = 0.15f, B = 0.50f, C = 0.10f, D = 0.20f, E = 0.02f, F = 0.30f;
    const float CB = C * B, DE = D * E, DF = D * F, EF = E / F;
    const d3 num = sadd(hmul(x, sadd(x * static_cast<double>(A), static_cast<double>(CB))),
                        static_cast<double>(DE));
    const d3 den = sadd(hmul(x, sadd(x * static_cast<double>(A), static_cast<double>(B))),
                        static_cast<double>(DF));
    return ssub(hdiv(num, den), static_cast<double>(EF));
}
__device__ __forceinline__ double luminance(d3 c) { return dot(c, mk(0.2126, 0.7152, 0.0722)); }
__device__ __forceinline__ d3 change_luminance(d3 c, double l_out) {
    return c * (l_out / luminance(c));
}
__device__ __forceinline__ d3 tonemap_op(d3 c, int op) {
    switch (op) {
    case 0:  // simple
        return {smin(1.0, smax(0.0, c.x)), smin(1.0, smax(0.0, c.y)), smin(1.0, smax(0.0, c.z))};
    case 1:  // reinhardSimple: c / (c + 1)
        return hdiv(c, sadd(c, 1.0));
    case 2: {  // reinhardExtended(c, 5.0)
        const double ws = 5.0 * 5.0;
        return hdiv(hmul(c, sadd(hdiv(c, mk(ws, ws, ws)), 1.0)), sadd(c, 1.0));
    }
    case 3: {  // reinhardExtendedLuminance(c, 5.0)
        const double lo = luminance(c);
        const double num = lo * (1.0 + (lo / (5.0 * 5.0)));
        return change_luminance(c, num / (1.0 + lo));
    }
    case 4: {  // reinhardJodie(c, 0.18)
        const double L = luminance(c);
        const double lm = (0.18 / log(2.0 + pow((L / 0.85), 1.7))) * log(1.0 + L);
        return change_luminance(c, lm);
    }
    case 5: {  // uncharted2
        const double exposure = static_cast<double>(2.0f);
        const d3 cur = uncharted2_partial(c * exposure);
        const d3 ws = hdiv(mk(1.0, 1.0, 1.0), uncharted2_partial(mk(11.2, 11.2, 11.2)));
        return hmul(cur, ws);
    }
    default: {  // aces_approx
        const d3 v = c * static_cast<double>(0.6f);
        const float a = 2.51f, b = 0.03f, cc = 2.43f, d = 0.59f, e = 0.14f;
        const d3 num = hmul(v, sadd(v * static_cast<double>(a), static_cast<double>(b)));
        const d3 den = sadd(hmul(v, sadd(v * static_cast<double>(cc), static_cast<double>(d))),
                            static_cast<double>(e));
        return clamp3(hdiv(num, den), static_cast<double>(0.0f), static_cast<double>(1.0f));
    }
    }
}
// The operators without libm calls (all but Reinhard-Jodie, op 4): lean kernels fuse only
// these; a Jodie request selects the kernel variant that compiles tonemap_op in full.
__device__ __forceinline__ d3 tonemap_op_nolog(d3 c, int op) {
    switch (op) {
    case 0: case 1: case 2: case 3: case 5: return tonemap_op(c, op);
    default: return tonemap_op(c, 6);
    }
}
// toColor (RaytracingEngine.cpp:113-121): clamp to [0,1], truncating cast of x*255.
__device__ __forceinline__ void to_color(d3 v, uint8_t& r, uint8_t& g, uint8_t& b) {
    const d3 c = clamp3(v, 0.0, 1.0);
    r = static_cast<uint8_t>(c.x * 255.0);
    g = static_cast<uint8_t>(c.y * 255.0);
    b = static_cast<uint8_t>(c.z * 255.0);
}

// toColor(reinhardSimple(c)) for one component (RaytracingEngine.cpp:70-72, 113-121): the byte
// is trunc(fl(fl(c / (c + 1)) · 255)) after the clamp to [0, 1].  For 0 ≤ c ≤ 2^20 an FP32
// estimate f of 255·c/(c+1) — conversion, add, v_rcp_f32 (1 ulp), two products: relative error
// ≤ 6·2^-24 + 2^-23 < 5e-7, so |f − 255·c/(c+1)| < 1.3e-4 — decides the truncation whenever its
// fraction is more than 5e-4 from an integer: the exact value (and the reference's FP64 result,
// within 1e-13 of it) then has the same integer part.  Otherwise, and for c outside that range
// (negative, NaN, huge), the reference's FP64 expression.
__device__ __forceinline__ uint8_t reinhard_byte(double c) {
    if (c >= 0.0 && c <= 0x1p20) {
        const float cf = static_cast<float>(c);
        const float f = (255.0f * cf) * __builtin_amdgcn_rcpf(cf + 1.0f);
        const float fl = __builtin_floorf(f);
        const float fr = f - fl;  // exact (f < 256)
        if (fr > 5e-4f && fr < 1.0f - 5e-4f) return static_cast<uint8_t>(static_cast<int>(fl));
    }
    const double y = c / (c + 1.0);
    return static_cast<uint8_t>(smin(1.0, smax(0.0, y)) * 255.0);
}

}  // namespace rtamd
