// rt_context.hpp — the C-ABI objects (rt_context, rt_scene) and the helpers the C-ABI
// translation units share (rt_capi.cpp: single device; rt_multi.cpp: RCCL multi-GPU frames).
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <string>
#include <utility>
#include <vector>

#include "rt_capi.h"
#include "rt_internal.hpp"

namespace rtamd {

// Sets the calling thread's rt_last_error() message and returns st.
rt_status fail(rt_status st, const std::string& msg);
rt_status hip_fail(hipError_t e, const char* what);

#define RT_HIP(call)                                    \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return rtamd::hip_fail(e_, #call); \
    } while (0)

struct DeviceBuffer {
    void* ptr = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&ptr, need);
        if (e == hipSuccess) bytes = need;
        return e;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace rtamd

struct rt_comm;

struct rt_context {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    size_t lds_limit = 0;
    rtamd::DeviceBuffer out64, out32, ldr, tm_in, tm_out, dbg, rays;
    rtamd::DeviceBuffer counters;  // 2 x u64
    rtamd::DeviceBuffer wf, wf_ctl;  // breadth-first TraceRay arena + its control block
    // The arena and the counters are one per context: a render that uses them waits for the
    // previous one that did, on whatever stream it ran (scratch_wait / scratch_done).
    hipEvent_t scratch_event = nullptr;
    bool scratch_used = false;
    hipStream_t scratch_stream = nullptr;  // the stream of the latest scratch user
    // the packet kernel's fix-up list (TraceParams.fix_list) and its control words, one per
    // context like the counters (ordered across streams by scratch_wait / scratch_done)
    rtamd::DeviceBuffer fix_list, fix_ctl;
    int fix_parity = 0;  // which of the two counts of fix_ctl the next fix-variant launch uses
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> free_events;
    double timed_ms = 0.0;
    uint64_t launches = 0;
    // rt_render_multi: RCCL communicators over the devices of the last context list this
    // context led (rt_multi.cpp); destroyed with the context
    std::vector<rt_context*> group_ctxs;
    std::vector<rt_comm*> group_comms;
    // the contexts whose cached group includes this one (released when this one is destroyed)
    std::vector<rt_context*> group_roots;
};

struct rt_scene {
    rt_context* ctx = nullptr;
    rtamd::DeviceBuffer buf;
    int32_t ns = 0, np = 0, nt = 0, nl = 0;
    size_t off_sph = 0, off_sph_mat = 0, off_pl = 0, off_pl_mat = 0, off_tri = 0, off_tri_mat = 0,
           off_lt = 0;
    bool any_transparent = false;
    double max_specular = 0.0;  // NaN-aware: stored as +inf when a NaN specular exists
    bool has_area = false;
    rt_area_light area{};
    size_t off_bvh = 0, off_bvh_tri = 0;  // triangle BVH, when bvh_nodes > 0
    int32_t bvh_nodes = 0;
    size_t off_sperm = 0, off_sbnd = 0;   // sphere chunks, when ns >= kSphChunkMin
    size_t off_box = 0;                   // planes-only chain table (rt_box.hip), when np > 0
    int32_t box_n[4] = {0, 0, 0, 0};
    // Packet-kernel LDS images, one per camera position this scene was rendered from more than
    // once (the image depends on the spheres, planes, point lights and camera position only).  An
    // entry is written once, by packet_image_kernel on the stream of the render that created
    // it; renders on other streams wait for its event until it has completed.  Never rewritten
    // or freed before the scene, so a launch in flight never sees it change.
    struct PkImage {
        double cam[3];
        rtamd::DeviceBuffer buf;
        hipEvent_t ready = nullptr;
        hipStream_t stream = nullptr;
        bool done = false;
        // Costliest-first tile order of the packet kernel for this camera (rt_capi.cpp
        // tile_order): the wave durations one launch records, then the order built from them,
        // for launches of the same shape (grid, rows) — state 1 recorded, 2 ordered.  One entry
        // per launch shape (up to kMaxTileOrders), each written once and never rewritten, so a
        // launch of one shape in flight on any stream never sees another shape's table.
        struct TileOrder {
            uint32_t key[8] = {};  // gx gy waves width height rows row0 row_block|row_stride
            int state = 0;
            rtamd::DeviceBuffer cost, keys, order;
            hipEvent_t recorded = nullptr, built = nullptr;
            // pinned host word the order kernel fills: 0 not yet, 1 narrow (keep the default
            // order, no table), 2 dispatch by the table
            uint32_t* verdict = nullptr;
        };
        std::vector<TileOrder> ords;
        int last_ord = -1;  // the entry of the latest launch (rt_debug_tile_order)
    };
    mutable std::vector<PkImage> pk_images;
    mutable std::vector<std::array<double, 3>> pk_seen;  // cameras rendered once, no image yet
    // Cameras without an image: a ring of kPkPubSlots publish slots (rt_packet.hip, in-launch
    // image hand-off), each launch tagged with its own epoch; zeroed once at allocation.
    mutable rtamd::DeviceBuffer pk_pub;
    // Frame batches with cameras that have no cached image (a moving camera): one small launch
    // forms every frame's image into a ring entry of kPkBatchRing × kPkMaxBatch images before
    // the batch launch, which copies them like cached ones; an entry is reused only after the
    // batch that read it (its event) has completed.
    static constexpr int kPkBatchRing = 4;
    mutable rtamd::DeviceBuffer pk_batch;
    mutable hipEvent_t pk_batch_done[kPkBatchRing] = {nullptr, nullptr, nullptr, nullptr};
    mutable bool pk_batch_used[kPkBatchRing] = {false, false, false, false};
    mutable int pk_batch_next = 0;
};

namespace rtamd {

// Rows a render call produces: [row_begin, row_end), or with row_cycle > 1 the row_block-row
// blocks starting at row_begin + k*row_cycle*row_block inside it (rt_render_opts).
uint32_t rendered_rows(const rt_render_opts& o, uint32_t height);
rt_status validate_camera(const rt_camera* cam);
// Enqueues one render (plus the counting pass with RT_FLAG_COUNT_RAYS) on ctx's stream into
// device outputs in the packed row order of opts.  The caller holds a DeviceGuard.
rt_status enqueue_render(rt_context* ctx, const rt_scene* sc, const rt_camera* cam,
                         const rt_render_opts* opts, double* d64, float* d32, uint8_t* dldr);
// The same for a batch of nframes cameras (same width / height / focal / aa_samples): frame f
// writes its rows f·stride·width pixels into each output, stride = frame_rows (0: the rows the
// render produces; larger pads every frame, as the row-split gather's send buffers are laid out).
// Packet-kernel scenes render up to kPkMaxBatch frames per launch (blockIdx.z = frame), other
// scenes one launch per frame.
rt_status enqueue_frames(rt_context* ctx, const rt_scene* sc, const rt_camera* cams, int nframes,
                         const rt_render_opts* opts, double* d64, float* d32, uint8_t* dldr,
                         uint32_t frame_rows = 0);
rt_status check_batch(const rt_camera* cams, int nframes);
// Whether a render takes the breadth-first TraceRay path, whose arena is one per context (as are
// the ray counters): renders that use them are ordered across streams (scratch_wait/_done).
bool uses_wavefront_arena(int path, int flags);
// Orders work on ctx->stream after the last render that used the context's scratch (any
// stream), and marks ctx->stream's work so far as the latest such user.
rt_status scratch_wait(rt_context* ctx);
rt_status scratch_done(rt_context* ctx);
// Adds the elapsed time of completed RT_FLAG_TIME_KERNEL event pairs to the context totals.
rt_status harvest_events(rt_context* ctx, bool all);
// rt_multi.cpp: releases the communicators rt_render_multi cached in ctx.
void release_group(rt_context* ctx);
// rt_multi.cpp: releases ctx's own group and every group that includes ctx (context teardown).
void leave_groups(rt_context* ctx);

}  // namespace rtamd
