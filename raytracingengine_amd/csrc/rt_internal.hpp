// rt_internal.hpp — what the C-ABI layer (rt_capi.cpp) and the kernels (rt_trace.hip) share.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace rtamd {

// Device scene records (doubles per record).  Layout in HBM is one allocation, record arrays
// back to back; the per-ray geometry arrays (sphere/plane/light) are staged into LDS.
constexpr int kSphStride = 4;   // cx cy cz r²            (r² = radius*radius, as Shape.h:77)
constexpr int kPlStride = 8;    // px py pz nx ny nz - -  (normal as stored, Shape.h:142)
constexpr int kTriStride = 12;  // a0(3) e1(3) e2(3) n(3) (translated v0 and edges, Shape.h:204-206;
                                //                         untranslated normal, Shape.h:222-227)
constexpr int kLtStride = 8;    // px py pz Ex Ey Ez - -  (E = color*intensity, Scene.h:110)
constexpr int kMatStride = 8;   // r g b shininess specular transparency ior -
// Planes-only chain kernel (rt_box.hip): one record per plane, in axis-group order —
// p xyz | n xyz | p[k] (k = the group's axis) | 1 when |n| rounds to exactly 1 |
// material (kMatStride - 1 doubles: r g b shininess specular transparency ior) | scene index (int)
constexpr int kBoxRec = 16;
constexpr int kBoxMaxSpheres = 64;  // reflection chains with spheres take rt_box.hip up to this

constexpr int kBvhNodeStride = 8;  // triangle BVH node: lo xyz, hi xyz, {first, count}
constexpr int kBvhMinTris = 32;    // scenes with fewer triangles test them all (no BVH)
constexpr int kBvhStack = 64;      // traversal stack entries (build depth <= 48)
constexpr int kMaxDepth = 16;   // deepest recursion the CHAIN/TREE kernels keep a stack for
// Generic kernels: 256-thread workgroups of 8×32 pixels, so each wave is an 8×8 tile — the
// rays of a square tile stay together down a reflection chain longer than those of a 64-pixel
// row (C1 0.52 → 0.49 ms, mirror -2 %, mesh -4 %; 16×4 waves: C1 0.50 ms).
constexpr int kTileW = 8;       // pixels per workgroup row
constexpr int kTileH = 32;      // rows per workgroup (256 threads: 4 waves of 8×8)

enum PathKind : int {
    kPathDirect = 0,  // no material can spawn a secondary ray: primary + shadow rays only
    kPathChain = 1,   // opaque, some specular > bias: linear reflection chain (≤ maxRecursion)
    kPathTree = 2     // some transparency > 0: refraction + reflection binary tree
};

// Packet kernel frame batches (rt_render_batch): frames of one scene and launch shape, one per
// blockIdx.z, each with its own camera position and the camera-dependent packet-image source.
constexpr int kPkMaxBatch = 32;
struct PkFrame {
    double cam[3];
    const double* img;         // cached LDS image of this camera, or null
    unsigned long long* pub;   // else: the in-launch hand-off slot, or null (form per workgroup)
    uint32_t epoch;
    uint32_t _pad;
};

struct TraceParams {
    // scene (device pointers into the scene allocation)
    const double* sph;
    const double* sph_mat;
    const double* pl;
    const double* pl_mat;
    const double* tri;
    const double* tri_mat;
    const double* lt;
    int32_t ns, np, nt, nl;
    // build-defined area light (samples == 0: none)
    double al_corner[3];
    double al_u[3];
    double al_v[3];
    double al_E[3];        // color * (intensity / samples)
    int32_t al_samples;
    int32_t al_k;          // sqrt(samples)
    // camera
    double cam_pos[3];
    double focal;
    uint32_t width, height;
    int32_t aa;
    int32_t max_rec;
    double bias;
    uint64_t seed;
    // tile
    uint32_t row0, rows;
    uint32_t row_block, row_stride;  // block-cyclic rows (row_block 0: contiguous from row0)
    // outputs (device; any may be null)
    double* out64;
    float* out32;
    uint8_t* ldr;
    int32_t tonemap;
    int32_t _pad;
    unsigned long long* counters;  // [trace, shadow] — only written by the counting variant
    const uint8_t* redo;  // generic kernels: when set, only pixels with a flagged sample run
    const double* bvh;       // triangle BVH nodes (rt_bvh.cpp), or null: test every triangle
    const int32_t* bvh_tri;  // triangle ids in leaf order
    const double* pk_image;  // packet kernel: LDS image of this scene + camera, or null
    // packet kernel, camera without a cached image: the slot the launch's first workgroup
    // publishes its image to ({epoch, word} granules, one per 32-bit image word), or null
    unsigned long long* pk_pub;
    uint32_t pk_epoch;       // this launch's tag (never 0)
    uint32_t pk_pub_first;   // workgroups below this linear index form the image themselves
    // packet kernel, ns >= kSphChunkMin: spatial sphere order and chunk bounds (build_sphere_chunks)
    const int32_t* sph_perm;
    const double* sph_bnd;
    // generic kernels with `redo`: 0 here means no sample overflowed, every workgroup leaves
    const uint32_t* redo_any;
    // packet kernel: the tile each workgroup renders, by dispatch position (costliest first,
    // packet_order_kernel), or null for the default bottom-up order; and, when set, where each
    // wave records its duration (per tile and wave) for the next order
    const uint32_t* tile_order;
    uint32_t* tile_cost;
    // planes-only chain kernel: the box table (kBoxRec doubles per plane) and its group sizes —
    // normal ±e_x, ±e_y, ±e_z, any other
    const double* box;
    int32_t box_n[4];
    // packet kernel, fix-up variants (kFeatFix): undecided shadow rays are not marched; the
    // pixel's output index (frame · frame_px + row-local pixel) is appended to fix_list and
    // packet_fixup_kernel renders it with the exact per-pixel path.  fix_ctl: the list's count
    // for this launch; fix_next: the count the context's NEXT fix-variant launch appends to (the
    // two alternate launch by launch; the fix-up launch zeroes fix_next — nothing reads it until
    // that next launch, ordered after this one — so no completion atomic is needed)
    uint32_t* fix_list;
    uint32_t* fix_ctl;
    uint32_t* fix_next;
    // packet kernel frame batch: nframes > 0 replaces cam_pos / pk_image / pk_pub / pk_epoch
    // by fr[blockIdx.z]; frame z writes its outputs frame_px pixels after frame z - 1's
    uint32_t nframes;
    uint32_t _pad2;
    uint64_t frame_px;
    PkFrame fr[kPkMaxBatch];
};

// Host: the spatial sphere chunks of the packet kernel's culls (rt_bvh.cpp): perm[sorted] =
// original index, bounds = one bounding sphere (cx cy cz R) per 64 sorted spheres.
constexpr int kSphChunkMin = 65;  // scenes with fewer spheres have a single chunk (no order)
void build_sphere_chunks(const double* sph, int ns, std::vector<int32_t>& perm,
                         std::vector<double>& bounds);

// Host: builds the triangle BVH over the uploaded triangle records (kTriStride doubles each).
void build_triangle_bvh(const double* tri, int nt, std::vector<double>& nodes,
                        std::vector<int32_t>& order);

// Doubles of the scene image the generic kernels stage into LDS (spheres, planes, lights).
__host__ __device__ inline size_t scene_doubles(const TraceParams& p) {
    return static_cast<size_t>(kSphStride) * p.ns + static_cast<size_t>(kPlStride) * p.np +
           static_cast<size_t>(kLtStride) * p.nl;
}

// sample_parallel: multi-sample frames (2 ≤ aa ≤ kAaParallelMax) of the direct and chain paths
// trace one sample per thread (rt_trace.hip), the same image as the per-thread sample loop
constexpr int kAaParallelMax = 128;
hipError_t launch_trace(const TraceParams& p, int path, bool count, bool lds, size_t lds_bytes,
                        hipStream_t stream, bool sample_parallel = false);
namespace lean {  // rt_trace_lean.hip: the same kernels for scenes without triangles / area light
hipError_t launch_trace(const TraceParams& p, int path, bool count, bool lds, size_t lds_bytes,
                        hipStream_t stream, bool sample_parallel = false);
}
hipError_t launch_box_chain(const TraceParams& p, bool count, bool sample_parallel,
                            hipStream_t stream);
hipError_t launch_packet_direct(const TraceParams& p, bool count, bool any_specular,
                                hipStream_t stream);
size_t packet_lds_bytes(int ns, int np, int nl);
hipError_t launch_packet_image(const TraceParams& p, double* img, hipStream_t stream);
// Whether launch_packet_direct takes a fix-up variant for p (then p.fix_list / p.fix_ctl must be
// set, with room for every output pixel of the launch), and the fix-up launch that follows it.
bool packet_uses_fixup(const TraceParams& p, bool count, bool any_specular);
hipError_t launch_packet_fixup(const TraceParams& p, hipStream_t stream);
// The images a frame batch forms before its launch: job j forms frame frame[j]'s image
// (camera p.fr[frame[j]].cam) at dst[j] — a cache entry of the scene or a slot of its ring.
struct PkImageJobs {
    double* dst[kPkMaxBatch];
    int32_t frame[kPkMaxBatch];
    int32_t n;
};
hipError_t launch_packet_image_batch(const TraceParams& p, const PkImageJobs& jobs,
                                     hipStream_t stream);
// The packet kernel's launch shape for p (grid of workgroups, waves per workgroup), and the
// costliest-first tile order built from the wave durations a launch of that shape recorded.
void packet_grid(const TraceParams& p, uint32_t& gx, uint32_t& gy, uint32_t& waves);
hipError_t launch_packet_order(const uint32_t* cost, uint32_t gx, uint32_t gy, uint32_t waves,
                               uint32_t* keys, uint32_t* order, uint32_t* verdict,
                               hipStream_t stream);
int packet_max_spheres();
hipError_t launch_trace_rays(const TraceParams& p, int path, bool count, const double* rays,
                             size_t n, double* out, hipStream_t stream);
hipError_t launch_intersect_rays(const TraceParams& p, const double* rays, size_t n, double* out,
                                 hipStream_t stream);
hipError_t launch_tonemap(const double* hdr, size_t n, int op, uint8_t* out, hipStream_t stream);
hipError_t launch_debug_f64(const double* x, const double* y, size_t n, double* out,
                            hipStream_t stream);
hipError_t launch_debug_vec(const double* v, size_t n, double* out, hipStream_t stream);

}  // namespace rtamd
