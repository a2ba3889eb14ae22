// Microbenchmark: issue cost of the non-arithmetic VALU instructions the packet kernel is full of
// (FP64 compares, conversions, selects, lane reads, 64-bit shifts, 32-bit integer multiplies) next
// to FP64 FMA / add and FP32 add, on gfx950 (dev tool; tools/micro/fp64_rates.hip measures the
// FP64 arithmetic and transcendental ops).  Eight independent instructions per loop iteration, in
// inline asm so that exactly that instruction is issued; cycles per wave-instruction per SIMD
// at 2.4 GHz with 1, 4 and 8 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/valu_rates.hip -o tools/micro/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int N = 4096;

__global__ void k_fma_f64(double* out, double s) {
    double a = s + threadIdx.x * 1e-9, b = a * 1.1, c = a * 1.3, d = a * 1.7;
    double e = a * 1.9, f = a * 2.3, g = a * 2.9, h = a * 3.1;
    for (int i = 0; i < N; ++i) {
        asm volatile(
            "v_fma_f64 %0, %0, %0, %1\n v_fma_f64 %1, %1, %1, %2\n v_fma_f64 %2, %2, %2, %3\n"
            "v_fma_f64 %3, %3, %3, %4\n v_fma_f64 %4, %4, %4, %5\n v_fma_f64 %5, %5, %5, %6\n"
            "v_fma_f64 %6, %6, %6, %7\n v_fma_f64 %7, %7, %7, %0\n"
            : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
}

// independent ops (no chain): each writes its own register from fixed inputs
#define INDEP_KERNEL(name, body)                                                             \
    __global__ void name(double* out, double s) {                                             \
        double a = s + threadIdx.x * 1e-9, b = a * 1.1;                                       \
        float fa = (float)a, fb = (float)b;                                                   \
        unsigned ia = __double2loint(a), ib = __double2hiint(a);                              \
        double r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;               \
        float g0 = 0, g1 = 0, g2 = 0, g3 = 0;                                                 \
        unsigned u0 = 0, u1 = 0, u2 = 0, u3 = 0;                                              \
        for (int i = 0; i < N; ++i) { body }                                                  \
        out[blockIdx.x * blockDim.x + threadIdx.x] =                                          \
            r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7 + g0 + g1 + g2 + g3 + u0 + u1 + u2 + u3;   \
    }

INDEP_KERNEL(k_add_f64, asm volatile(
    "v_add_f64 %0, %8, %9\n v_add_f64 %1, %8, %9\n v_add_f64 %2, %8, %9\n v_add_f64 %3, %8, %9\n"
    "v_add_f64 %4, %8, %9\n v_add_f64 %5, %8, %9\n v_add_f64 %6, %8, %9\n v_add_f64 %7, %8, %9\n"
    : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3), "=v"(r4), "=v"(r5), "=v"(r6), "=v"(r7) : "v"(a), "v"(b));)
INDEP_KERNEL(k_cmp_f64, asm volatile(
    "v_cmp_lt_f64 vcc, %0, %1\n v_cmp_lt_f64 vcc, %1, %0\n v_cmp_gt_f64 vcc, %0, %1\n"
    "v_cmp_gt_f64 vcc, %1, %0\n v_cmp_le_f64 vcc, %0, %1\n v_cmp_le_f64 vcc, %1, %0\n"
    "v_cmp_ge_f64 vcc, %0, %1\n v_cmp_ge_f64 vcc, %1, %0\n" :: "v"(a), "v"(b) : "vcc");)
INDEP_KERNEL(k_cvt_f32_f64, asm volatile(
    "v_cvt_f32_f64 %0, %8\n v_cvt_f32_f64 %1, %9\n v_cvt_f32_f64 %2, %8\n v_cvt_f32_f64 %3, %9\n"
    "v_cvt_f32_f64 %4, %8\n v_cvt_f32_f64 %5, %9\n v_cvt_f32_f64 %6, %8\n v_cvt_f32_f64 %7, %9\n"
    : "=v"(g0), "=v"(g1), "=v"(g2), "=v"(g3), "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3) : "v"(a), "v"(b));)
INDEP_KERNEL(k_cvt_f64_f32, asm volatile(
    "v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %5\n v_cvt_f64_f32 %2, %4\n v_cvt_f64_f32 %3, %5\n"
    "v_cvt_f64_f32 %0, %5\n v_cvt_f64_f32 %1, %4\n v_cvt_f64_f32 %2, %5\n v_cvt_f64_f32 %3, %4\n"
    : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(fa), "v"(fb));)
INDEP_KERNEL(k_cndmask, asm volatile(
    "v_cmp_lt_f32 vcc, %8, %9\n"
    "v_cndmask_b32 %0, %10, %11, vcc\n v_cndmask_b32 %1, %11, %10, vcc\n"
    "v_cndmask_b32 %2, %10, %11, vcc\n v_cndmask_b32 %3, %11, %10, vcc\n"
    "v_cndmask_b32 %4, %10, %11, vcc\n v_cndmask_b32 %5, %11, %10, vcc\n"
    "v_cndmask_b32 %6, %10, %11, vcc\n v_cndmask_b32 %7, %11, %10, vcc\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(g0), "=v"(g1), "=v"(g2), "=v"(g3)
    : "v"(fa), "v"(fb), "v"(ia), "v"(ib) : "vcc");)
// the mask written once before the loop: v_cndmask throughput alone (VCC, and an SGPR pair)
#define MASK_KERNEL(name, setup, body)                                                        \
    __global__ void name(double* out, double s) {                                             \
        double a = s + threadIdx.x * 1e-9, b = a * 1.1;                                       \
        float fa = (float)a, fb = (float)b;                                                   \
        unsigned ia = __double2loint(a), ib = __double2hiint(a);                              \
        unsigned u0 = 0, u1 = 0, u2 = 0, u3 = 0, u4 = 0, u5 = 0, u6 = 0, u7 = 0;              \
        setup                                                                                 \
        for (int i = 0; i < N; ++i) { body }                                                  \
        out[blockIdx.x * blockDim.x + threadIdx.x] = u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7;  \
    }
MASK_KERNEL(k_cndmask_vcc,
    asm volatile("v_cmp_lt_f32 vcc, %0, %1" :: "v"(fa), "v"(fb) : "vcc");,
    asm volatile(
    "v_cndmask_b32 %0, %8, %9, vcc\n v_cndmask_b32 %1, %9, %8, vcc\n"
    "v_cndmask_b32 %2, %8, %9, vcc\n v_cndmask_b32 %3, %9, %8, vcc\n"
    "v_cndmask_b32 %4, %8, %9, vcc\n v_cndmask_b32 %5, %9, %8, vcc\n"
    "v_cndmask_b32 %6, %8, %9, vcc\n v_cndmask_b32 %7, %9, %8, vcc\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
    : "v"(ia), "v"(ib) : "vcc");)
MASK_KERNEL(k_cndmask_sgpr,
    asm volatile("v_cmp_lt_f32_e64 s[40:41], %0, %1" :: "v"(fa), "v"(fb) : "s40", "s41");,
    asm volatile(
    "v_cndmask_b32_e64 %0, %8, %9, s[40:41]\n v_cndmask_b32_e64 %1, %9, %8, s[40:41]\n"
    "v_cndmask_b32_e64 %2, %8, %9, s[40:41]\n v_cndmask_b32_e64 %3, %9, %8, s[40:41]\n"
    "v_cndmask_b32_e64 %4, %8, %9, s[40:41]\n v_cndmask_b32_e64 %5, %9, %8, s[40:41]\n"
    "v_cndmask_b32_e64 %6, %8, %9, s[40:41]\n v_cndmask_b32_e64 %7, %9, %8, s[40:41]\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
    : "v"(ia), "v"(ib) : "s40", "s41");)
MASK_KERNEL(k_cndmask_vcc_e64,
    asm volatile("v_cmp_lt_f32 vcc, %0, %1" :: "v"(fa), "v"(fb) : "vcc");,
    asm volatile(
    "v_cndmask_b32_e64 %0, %8, %9, vcc\n v_cndmask_b32_e64 %1, %9, %8, vcc\n"
    "v_cndmask_b32_e64 %2, %8, %9, vcc\n v_cndmask_b32_e64 %3, %9, %8, vcc\n"
    "v_cndmask_b32_e64 %4, %8, %9, vcc\n v_cndmask_b32_e64 %5, %9, %8, vcc\n"
    "v_cndmask_b32_e64 %6, %8, %9, vcc\n v_cndmask_b32_e64 %7, %9, %8, vcc\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
    : "v"(ia), "v"(ib) : "vcc");)
// the VOP2 form with VCC, its operands in other registers than the VOP3 test (v_addc-style
// VCC reads for comparison)
MASK_KERNEL(k_addc_vcc,
    asm volatile("v_cmp_lt_f32 vcc, %0, %1" :: "v"(fa), "v"(fb) : "vcc");,
    asm volatile(
    "v_addc_co_u32 %0, s[42:43], %8, %9, vcc\n v_addc_co_u32 %1, s[42:43], %9, %8, vcc\n"
    "v_addc_co_u32 %2, s[42:43], %8, %9, vcc\n v_addc_co_u32 %3, s[42:43], %9, %8, vcc\n"
    "v_addc_co_u32 %4, s[42:43], %8, %9, vcc\n v_addc_co_u32 %5, s[42:43], %9, %8, vcc\n"
    "v_addc_co_u32 %6, s[42:43], %8, %9, vcc\n v_addc_co_u32 %7, s[42:43], %9, %8, vcc\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
    : "v"(ia), "v"(ib) : "vcc", "s42", "s43");)
// the compiler's select pattern: a compare into the mask, then two selects (a double's halves);
// four per iteration, counted as 12 instructions per 4... (reported per instruction: x8/12)
MASK_KERNEL(k_sel_vop2, ,
    asm volatile(
    "v_cmp_lt_f32 vcc, %8, %9\n v_cndmask_b32 %0, %8, %9, vcc\n v_cndmask_b32 %1, %9, %8, vcc\n"
    "v_cmp_gt_f32 vcc, %8, %9\n v_cndmask_b32 %2, %8, %9, vcc\n v_cndmask_b32 %3, %9, %8, vcc\n"
    "v_cmp_le_f32 vcc, %8, %9\n v_cndmask_b32 %4, %8, %9, vcc\n v_cndmask_b32 %5, %9, %8, vcc\n"
    "v_cmp_ge_f32 vcc, %8, %9\n v_cndmask_b32 %6, %8, %9, vcc\n v_cndmask_b32 %7, %9, %8, vcc\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
    : "v"(ia), "v"(ib) : "vcc");)
MASK_KERNEL(k_sel_vop3, ,
    asm volatile(
    "v_cmp_lt_f32_e64 s[40:41], %8, %9\n v_cndmask_b32_e64 %0, %8, %9, s[40:41]\n v_cndmask_b32_e64 %1, %9, %8, s[40:41]\n"
    "v_cmp_gt_f32_e64 s[40:41], %8, %9\n v_cndmask_b32_e64 %2, %8, %9, s[40:41]\n v_cndmask_b32_e64 %3, %9, %8, s[40:41]\n"
    "v_cmp_le_f32_e64 s[40:41], %8, %9\n v_cndmask_b32_e64 %4, %8, %9, s[40:41]\n v_cndmask_b32_e64 %5, %9, %8, s[40:41]\n"
    "v_cmp_ge_f32_e64 s[40:41], %8, %9\n v_cndmask_b32_e64 %6, %8, %9, s[40:41]\n v_cndmask_b32_e64 %7, %9, %8, s[40:41]\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
    : "v"(ia), "v"(ib) : "s40", "s41");)
MASK_KERNEL(k_sel_vop3_vcc, ,
    asm volatile(
    "v_cmp_lt_f32 vcc, %8, %9\n v_cndmask_b32_e64 %0, %8, %9, vcc\n v_cndmask_b32_e64 %1, %9, %8, vcc\n"
    "v_cmp_gt_f32 vcc, %8, %9\n v_cndmask_b32_e64 %2, %8, %9, vcc\n v_cndmask_b32_e64 %3, %9, %8, vcc\n"
    "v_cmp_le_f32 vcc, %8, %9\n v_cndmask_b32_e64 %4, %8, %9, vcc\n v_cndmask_b32_e64 %5, %9, %8, vcc\n"
    "v_cmp_ge_f32 vcc, %8, %9\n v_cndmask_b32_e64 %6, %8, %9, vcc\n v_cndmask_b32_e64 %7, %9, %8, vcc\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7)
    : "v"(ia), "v"(ib) : "vcc");)
INDEP_KERNEL(k_add_f32, asm volatile(
    "v_add_f32 %0, %8, %9\n v_add_f32 %1, %8, %9\n v_add_f32 %2, %8, %9\n v_add_f32 %3, %8, %9\n"
    "v_add_f32 %4, %8, %9\n v_add_f32 %5, %8, %9\n v_add_f32 %6, %8, %9\n v_add_f32 %7, %8, %9\n"
    : "=v"(g0), "=v"(g1), "=v"(g2), "=v"(g3), "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3) : "v"(fa), "v"(fb));)
INDEP_KERNEL(k_mul_lo_u32, asm volatile(
    "v_mul_lo_u32 %0, %8, %9\n v_mul_lo_u32 %1, %8, %9\n v_mul_lo_u32 %2, %8, %9\n v_mul_lo_u32 %3, %8, %9\n"
    "v_mul_lo_u32 %4, %8, %9\n v_mul_lo_u32 %5, %8, %9\n v_mul_lo_u32 %6, %8, %9\n v_mul_lo_u32 %7, %8, %9\n"
    : "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(g0), "=v"(g1), "=v"(g2), "=v"(g3) : "v"(ia), "v"(ib));)
INDEP_KERNEL(k_lshl_b64, asm volatile(
    "v_lshlrev_b64 %0, 3, %4\n v_lshlrev_b64 %1, 5, %4\n v_lshlrev_b64 %2, 7, %4\n v_lshlrev_b64 %3, 9, %4\n"
    "v_lshlrev_b64 %0, 4, %5\n v_lshlrev_b64 %1, 6, %5\n v_lshlrev_b64 %2, 8, %5\n v_lshlrev_b64 %3, 10, %5\n"
    : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(a), "v"(b));)
INDEP_KERNEL(k_readlane, asm volatile(
    "v_readlane_b32 s40, %0, 1\n v_readlane_b32 s41, %0, 5\n v_readlane_b32 s42, %0, 9\n"
    "v_readlane_b32 s43, %0, 13\n v_readlane_b32 s44, %1, 17\n v_readlane_b32 s45, %1, 21\n"
    "v_readlane_b32 s46, %1, 25\n v_readlane_b32 s47, %1, 29\n"
    :: "v"(ia), "v"(ib) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");)

template <class F>
void run(const char* name, F k, double* out, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd;  // one 256-thread block = 4 waves = 1 per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = 5.0 * blocks * 4 * (double)N * 8 / 1024.0;  // wave-instructions
    printf("%-14s waves/SIMD=%d  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name,
           waves_per_simd, ms * 1e6 * 2.4 / per_simd);
}

int main() {
    double* out;
    hipMalloc(&out, 256 * 8 * 256 * sizeof(double));
    for (int w : {1, 4, 8}) {
        run("v_fma_f64 (chain)", k_fma_f64, out, w);
        run("v_add_f64", k_add_f64, out, w);
        run("v_cmp_*_f64", k_cmp_f64, out, w);
        run("v_cvt_f32_f64", k_cvt_f32_f64, out, w);
        run("v_cvt_f64_f32", k_cvt_f64_f32, out, w);
        run("v_cmp_f32+8 cndmask", k_cndmask, out, w);
        run("v_cndmask vcc", k_cndmask_vcc, out, w);
        run("v_cndmask sgpr", k_cndmask_sgpr, out, w);
        run("v_cndmask_e64 vcc", k_cndmask_vcc_e64, out, w);
        run("v_addc vcc", k_addc_vcc, out, w);
        run("sel vop2 (x12/8)", k_sel_vop2, out, w);
        run("sel vop3 sgpr (x12/8)", k_sel_vop3, out, w);
        run("sel vop3 vcc (x12/8)", k_sel_vop3_vcc, out, w);
        run("v_add_f32", k_add_f32, out, w);
        run("v_mul_lo_u32", k_mul_lo_u32, out, w);
        run("v_lshlrev_b64", k_lshl_b64, out, w);
        run("v_readlane_b32", k_readlane, out, w);
    }
    return 0;
}
