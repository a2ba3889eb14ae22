// rt_assemble.hip — rank 0's step of a row-tiled multi-GPU frame batch (rt_multi.cpp): the
// gathered per-rank buffers [n][frames][max_rows][row_bytes] (each rank's block-cyclic rows of
// every frame, packed in render order, one ncclGather of the whole batch) are written into image
// row order, frame after frame.  Pure data movement, HBM bound: each image row is
// read once and written once, 16 B per lane where the row pitch allows.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "rt_internal.hpp"

namespace rtamd {

namespace {

// Source row (in the gathered buffer) of frame z's image row y: block b = y / B belongs to rank
// b % n, as its (b / n)-th block (rt_render_opts row_block / row_cycle with row_begin = rank*B),
// in that rank's frame z.
__device__ __forceinline__ size_t gathered_row(uint32_t y, uint32_t z, uint32_t frames,
                                               uint32_t block, uint32_t n, uint32_t max_rows) {
    const uint32_t b = y / block;
    const uint32_t rank = b % n;
    const uint32_t local = (b / n) * block + (y - b * block);
    return (static_cast<size_t>(rank) * frames + z) * max_rows + local;
}

template <typename V>
__global__ __launch_bounds__(256) void assemble_rows_kernel(const V* __restrict__ src,
                                                            V* __restrict__ dst,
                                                            uint32_t words_per_row,
                                                            uint32_t height, uint32_t block,
                                                            uint32_t n, uint32_t max_rows) {
    // frame blockIdx.z of a batch: height image rows out
    dst += static_cast<size_t>(blockIdx.z) * height * words_per_row;
    // one workgroup row-strip: blockIdx.y walks image rows, x covers the row's words
    for (uint32_t y = blockIdx.y; y < height; y += gridDim.y) {
        const V* s =
            src + gathered_row(y, blockIdx.z, gridDim.z, block, n, max_rows) * words_per_row;
        V* d = dst + static_cast<size_t>(y) * words_per_row;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < words_per_row;
             i += gridDim.x * blockDim.x)
            d[i] = s[i];
    }
}

template <typename V>
hipError_t launch_as(const void* src, void* dst, size_t row_bytes, uint32_t height,
                     uint32_t block, uint32_t n, uint32_t max_rows, uint32_t frames,
                     hipStream_t stream) {
    const uint32_t words = static_cast<uint32_t>(row_bytes / sizeof(V));
    const uint32_t gx = (words + 255) / 256;
    // enough rows in flight to fill 256 CUs several times over; rows loop inside
    const uint32_t gy = height < 4096u ? height : 4096u;
    hipLaunchKernelGGL(assemble_rows_kernel<V>, dim3(gx, gy, frames), dim3(256), 0, stream,
                       static_cast<const V*>(src), static_cast<V*>(dst), words, height, block,
                       n, max_rows);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_assemble_rows(const void* gathered, void* image, size_t row_bytes,
                                uint32_t height, uint32_t block, uint32_t n, uint32_t max_rows,
                                uint32_t frames, hipStream_t stream) {
    if (height == 0 || row_bytes == 0 || frames == 0) return hipSuccess;
    const uintptr_t align = reinterpret_cast<uintptr_t>(gathered) |
                            reinterpret_cast<uintptr_t>(image) | row_bytes |
                            static_cast<uintptr_t>(max_rows * row_bytes);
    if (align % 16 == 0)
        return launch_as<uint4>(gathered, image, row_bytes, height, block, n, max_rows, frames,
                                  stream);
    if (align % 4 == 0)
        return launch_as<uint32_t>(gathered, image, row_bytes, height, block, n, max_rows, frames,
                                  stream);
    return launch_as<uint8_t>(gathered, image, row_bytes, height, block, n, max_rows, frames,
                                  stream);
}

}  // namespace rtamd
