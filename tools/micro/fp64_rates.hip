// Microbenchmark: FP64 VALU instruction throughput / latency on gfx950 (dev tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
constexpr int N = 2048;
#define KERNEL(name, init, body)                                                          \
__global__ void name(double* out, double s) {                                               \
    double a = s + threadIdx.x * 1e-9, b = a * 1.1, c = a * 1.3, d = a * 1.7;              \
    init;                                                                                   \
    for (int i = 0; i < N; ++i) { body; }                                                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;                            \
}
KERNEL(k_fma4, , a = __builtin_fma(a, 1.0000001, 1e-9); b = __builtin_fma(b, 1.0000001, 1e-9); c = __builtin_fma(c, 1.0000001, 1e-9); d = __builtin_fma(d, 1.0000001, 1e-9))
KERNEL(k_fma1, , a = __builtin_fma(a, 1.0000001, 1e-9))
KERNEL(k_rcp4, , a = __builtin_amdgcn_rcp(a); b = __builtin_amdgcn_rcp(b); c = __builtin_amdgcn_rcp(c); d = __builtin_amdgcn_rcp(d))
KERNEL(k_rsq4, , a = __builtin_amdgcn_rsq(a); b = __builtin_amdgcn_rsq(b); c = __builtin_amdgcn_rsq(c); d = __builtin_amdgcn_rsq(d))
KERNEL(k_div4, double e = s + 1.5, a = e / a; b = e / b; c = e / c; d = e / d)
KERNEL(k_div1, double e = s + 1.5, a = e / a)
KERNEL(k_sqrt4, , a = sqrt(a) + 0.5; b = sqrt(b) + 0.5; c = sqrt(c) + 0.5; d = sqrt(d) + 0.5)
KERNEL(k_sqrt1, , a = sqrt(a) + 0.5)
KERNEL(k_fma32x4, float fa = a; float fb = b; float fc = c; float fd = d, fa = __builtin_fmaf(fa, 1.0000001f, 1e-9f); fb = __builtin_fmaf(fb, 1.0000001f, 1e-9f); fc = __builtin_fmaf(fc, 1.0000001f, 1e-9f); fd = __builtin_fmaf(fd, 1.0000001f, 1e-9f); a = fa; b = fb; c = fc; d = fd)

template <class F>
void run(const char* name, F k, int ops_per_iter, double* out, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd;  // one 256-thread block = 4 waves = 1 per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr = 5.0 * blocks * 4 * (double)N * ops_per_iter;
    const double per_simd = wave_instr / 1024.0;
    const double ns = ms * 1e6;
    printf("%-10s waves/SIMD=%d  %.2f cycles per wave-op per SIMD (at 2.4 GHz)\n", name,
           waves_per_simd, ns * 2.4 / per_simd);
}

int main() {
    double* out;
    hipMalloc(&out, 256 * 8 * 256 * sizeof(double));
    for (int w : {1, 4}) {
        run("fma x4", k_fma4, 4, out, w);
        run("fma x1", k_fma1, 1, out, w);
        run("rcp x4", k_rcp4, 4, out, w);
        run("rsq x4", k_rsq4, 4, out, w);
        run("div x4", k_div4, 4, out, w);
        run("div x1", k_div1, 1, out, w);
        run("sqrt x4", k_sqrt4, 4, out, w);
        run("sqrt x1", k_sqrt1, 1, out, w);
        run("f32fma x4", k_fma32x4, 4, out, w);
    }
    return 0;
}
