// Microbenchmark (dev tool): cost of a dynamic tile queue for a persistent packet kernel.
// 32400 "tiles" (the C2 frame's 8x8 waves) of synthetic FP64 work, taken by 5120 resident
// waves (256 CUs x 4 SIMDs x 5) through
//   static    : no atomics, tile = wave + k * nwaves
//   global    : one device-scope atomicAdd counter
//   part8     : 8 counters (partition = blockIdx % 8, 256 B apart), each over 1/8 of the tiles
//   launch    : one wave per tile, a plain grid of 8100 workgroups (today's launch shape)
// and the same with no work per tile (raw queue rate).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kTiles = 32400;

__device__ __forceinline__ double work(unsigned tile, int lane, int iters) {
    double a = tile * 1e-3 + lane, b = a * 0.5, c = a * 0.25, d = a * 0.125;
    for (int i = 0; i < iters; ++i) {
        a = fma(a, 0.999, 1e-3);
        b = fma(b, 0.999, 2e-3);
        c = fma(c, 0.999, 3e-3);
        d = fma(d, 0.999, 4e-3);
    }
    return a + b + c + d;
}

template <int MODE>
__global__ __launch_bounds__(256) void persist(unsigned* ctr, double* out, int iters, int nwaves) {
    const int lane = threadIdx.x & 63;
    const unsigned wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (MODE == 0) {
        for (unsigned t = wid; t < kTiles; t += nwaves) out[t * 64 + lane] = work(t, lane, iters);
    } else if (MODE == 1) {
        for (;;) {
            unsigned t = 0;
            if (lane == 0) t = atomicAdd(ctr, 1u);
            t = __builtin_amdgcn_readfirstlane(t);
            if (t >= kTiles) break;
            out[t * 64 + lane] = work(t, lane, iters);
        }
    } else if (MODE == 3) {
        // partition = the XCD this wave runs on; L2 (workgroup-scope) atomics, coherent
        // among the CUs of one XCD
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const unsigned part = xcc & 7;
        const unsigned lo = part * kTiles / 8, hi = (part + 1) * kTiles / 8;
        for (;;) {
            unsigned t = 0;
            if (lane == 0)
                t = __hip_atomic_fetch_add(ctr + 64 * part, 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
            t = __builtin_amdgcn_readfirstlane(t) + lo;
            if (t >= hi) break;
            out[t * 64 + lane] = work(t, lane, iters);
        }
    } else {
        const unsigned part = blockIdx.x % 8;
        const unsigned lo = part * kTiles / 8, hi = (part + 1) * kTiles / 8;
        for (;;) {
            unsigned t = 0;
            if (lane == 0) t = atomicAdd(ctr + 64 * part, 1u);
            t = __builtin_amdgcn_readfirstlane(t) + lo;
            if (t >= hi) break;
            out[t * 64 + lane] = work(t, lane, iters);
        }
    }
}

__global__ __launch_bounds__(256) void launch_shape(double* out, int iters) {
    const int lane = threadIdx.x & 63;
    const unsigned t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t < kTiles) out[t * 64 + lane] = work(t, lane, iters);
}

int main() {
    unsigned* ctr;
    double* out;
    hipMalloc(&ctr, 8 * 256);
    hipMalloc(&out, sizeof(double) * 64 * kTiles);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int nwg = 1280, nwaves = nwg * 4;
    const char* names[5] = {"static", "global", "part8", "launch", "xccL2"};
    for (int iters : {0, 45, 90, 180}) {
        for (int mode = 0; mode < 5; ++mode) {
            float best = 1e9;
            for (int rep = 0; rep < 20; ++rep) {
                hipMemset(ctr, 0, 8 * 256);
                hipEventRecord(e0);
                if (mode == 0) persist<0><<<nwg, 256>>>(ctr, out, iters, nwaves);
                else if (mode == 1) persist<1><<<nwg, 256>>>(ctr, out, iters, nwaves);
                else if (mode == 2) persist<2><<<nwg, 256>>>(ctr, out, iters, nwaves);
                else if (mode == 4) persist<3><<<nwg, 256>>>(ctr, out, iters, nwaves);
                else launch_shape<<<(kTiles + 3) / 4, 256>>>(out, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("iters %4d  %-7s %8.1f us\n", iters, names[mode], best * 1e3);
        }
    }
    return 0;
}
