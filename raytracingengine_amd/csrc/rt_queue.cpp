// rt_queue.cpp — a serving frame queue (include/rt_capi.h rt_queue_*): consecutive frames of
// Scene::RenderImage (Scene.h:311-328) into device framebuffers, `depth` of them in flight on as
// many HIP streams of the context's device, so that one frame's launch tail (its last, partly
// idle wave rounds) overlaps the next frame's start.  Frames are independent: the queue adds no
// dependency between them (a camera's cached packet image, shared by frames on different
// streams, is waited for through its own event — rt_capi.cpp packet_image) — except frames
// that use scratch the context holds once: the breadth-first TraceRay arena of refraction-tree
// scenes (ctx->wf / wf_ctl) and the ray counters.  enqueue_frames orders such a render after
// the previous one on any stream of the context (scratch_wait / scratch_done, rt_capi.cpp), so
// two of them never share the arena at once, whichever API enqueued them.
#include <new>
#include <string>
#include <vector>

#include "rt_capi.h"
#include "rt_context.hpp"
#include "rt_internal.hpp"

using namespace rtamd;

struct rt_queue {
    rt_context* ctx = nullptr;
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> done;   // per slot: recorded after the slot's latest frame
    uint64_t next = 0;              // ticket of the next submitted frame (slot = ticket % depth)
};

extern "C" {

rt_status rt_queue_create(rt_context* ctx, int depth, rt_queue** out) {
    if (!ctx || !out) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_queue_create");
    if (depth < 1 || depth > 8) return fail(RT_ERR_INVALID_ARG, "queue depth must be in [1, 8]");
    *out = nullptr;
    DeviceGuard g(ctx->device);
    rt_queue* q = new (std::nothrow) rt_queue();
    if (!q) return fail(RT_ERR_OOM, "host allocation failed");
    q->ctx = ctx;
    for (int i = 0; i < depth; ++i) {
        hipStream_t s = nullptr;
        hipEvent_t e = nullptr;
        hipError_t err = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        if (err == hipSuccess) err = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (s) q->streams.push_back(s);
        if (e) q->done.push_back(e);
        if (err != hipSuccess) {
            rt_queue_destroy(q);
            return hip_fail(err, "rt_queue_create");
        }
    }
    *out = q;
    return RT_OK;
}

rt_status rt_queue_destroy(rt_queue* q) {
    if (!q) return RT_OK;
    DeviceGuard g(q->ctx->device);
    for (hipStream_t s : q->streams) (void)hipStreamSynchronize(s);
    for (hipEvent_t e : q->done) (void)hipEventDestroy(e);
    for (hipStream_t s : q->streams) (void)hipStreamDestroy(s);
    delete q;
    return RT_OK;
}

rt_status rt_queue_submit(rt_queue* q, const rt_scene* sc, const rt_camera* cam,
                          const rt_render_opts* opts, void* d_hdr64, void* d_hdr32, void* d_ldr,
                          uint64_t* ticket_out) {
    if (!q || !sc) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_queue_submit");
    rt_context* ctx = q->ctx;
    if (sc->ctx != ctx) return fail(RT_ERR_INVALID_ARG, "scene does not belong to the queue's context");
    DeviceGuard g(ctx->device);
    const size_t slot = static_cast<size_t>(q->next % q->streams.size());
    // the render goes through the context's launch path on the slot's stream
    hipStream_t saved = ctx->stream;
    ctx->stream = q->streams[slot];
    rt_status st = enqueue_render(ctx, sc, cam, opts, static_cast<double*>(d_hdr64),
                                  static_cast<float*>(d_hdr32), static_cast<uint8_t*>(d_ldr));
    hipError_t e = hipSuccess;
    if (st == RT_OK) e = hipEventRecord(q->done[slot], q->streams[slot]);
    ctx->stream = saved;
    if (st != RT_OK) return st;
    if (e != hipSuccess) return hip_fail(e, "rt_queue_submit");
    if (ticket_out) *ticket_out = q->next;
    q->next += 1;
    return RT_OK;
}

rt_status rt_queue_wait(rt_queue* q, uint64_t ticket) {
    if (!q) return fail(RT_ERR_INVALID_ARG, "queue is NULL");
    if (ticket >= q->next) return fail(RT_ERR_INVALID_ARG, "ticket " + std::to_string(ticket) +
                                                           " was not submitted");
    DeviceGuard g(q->ctx->device);
    // the slot's event marks its latest frame, which is `ticket` or a later one on the same
    // stream (in order): either way the frame has completed when it fires
    const size_t slot = static_cast<size_t>(ticket % q->streams.size());
    RT_HIP(hipEventSynchronize(q->done[slot]));
    return RT_OK;
}

rt_status rt_queue_synchronize(rt_queue* q) {
    if (!q) return fail(RT_ERR_INVALID_ARG, "queue is NULL");
    DeviceGuard g(q->ctx->device);
    for (hipStream_t s : q->streams) RT_HIP(hipStreamSynchronize(s));
    // timed launches of the queue's frames (RT_FLAG_TIME_KERNEL) into the context's stats
    return harvest_events(q->ctx, true);
}

}  // extern "C"
