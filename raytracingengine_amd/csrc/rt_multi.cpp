// rt_multi.cpp — Scene::RenderImage over the GPUs of a node (RE/Scene.h:318-325):
// the frame's rows are split block-cyclically over the ranks, every rank renders its rows, ONE
// RCCL gather per output moves them to rank 0 over xGMI, and rank 0 writes them into image
// order (rt_assemble.hip).  Two ways in:
//   * one process per GPU: rt_comm_create (ncclCommInitRank) + rt_render_gather on every rank;
//   * one process driving every GPU (the reference's single-process RenderImage):
//     rt_comm_create_all (ncclCommInitAll) + rt_render_gather_all, and rt_render_multi on top of
//     it for host framebuffers (the drop-in Scene::SetDevices path).
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "rt_capi.h"
#include "rt_context.hpp"
#include "rt_internal.hpp"

using namespace rtamd;

namespace rtamd {
hipError_t launch_assemble_rows(const void* gathered, void* image, size_t row_bytes,
                                uint32_t height, uint32_t block, uint32_t n, uint32_t max_rows,
                                uint32_t frames, hipStream_t stream);
}

static_assert(RT_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "rt_capi.h id size");

struct rt_comm {
    rt_context* ctx = nullptr;  // the context whose device and stream the renders use
    int device = -1;
    ncclComm_t nccl = nullptr;
    // rt_comm_create: a non-blocking RCCL communicator whose calls wait with a deadline
    // (comm_wait); past it, or on an asynchronous RCCL error, the communicator is aborted
    // (ncclCommAbort) and every later call on it fails with RT_ERR_RCCL
    bool nonblocking = false;
    bool aborted = false;
    long timeout_ms = 0;  // 0: no deadline
    rtamd::DeviceBuffer chk;  // rt_comm_set_root_weight's agreement check (2 ints)
    // rt_comm_create_local: no RCCL communicator; rt_render_gather_all copies every rank's rows
    // into rank 0's receive buffer (`peers` = the group in rank order, on every member)
    bool local = false;
    std::vector<rt_comm*> peers;
    hipEvent_t xfer_ready = nullptr, xfer_done = nullptr;
    int nranks = 1, rank = 0;
    // rt_comm_set_root_weight: rank 0 renders `root_weight` row sets (slots) of the block-cyclic
    // split, every other rank one; > 1 gathers with grouped P2P sends instead of ncclGather
    int root_weight = 1;
    // Two frame slots (RT_FLAG_PIPELINE alternates them; otherwise slot 0).  Per slot and output
    // kind (RT_OUT_HDR64, _HDR32, _LDR): this rank's packed rows (send) and, on rank 0, the n
    // gathered buffers (recv).
    DeviceBuffer send[2][3], recv[2][3];
    // RT_FLAG_PIPELINE: the gather + assembly run on this stream, overlapping the next frame's
    // render on the context stream; `rendered` hands a slot to it, `freed` hands it back.
    hipStream_t gstream = nullptr;
    hipEvent_t rendered[2] = {nullptr, nullptr}, freed[2] = {nullptr, nullptr};
    bool slot_used[2] = {false, false};
    // after this rank's latest frame (render, gather, assembly): what rt_comm_destroy waits for
    hipEvent_t done = nullptr;
    bool any_frame = false;
    uint64_t frame = 0;
    // RT_FLAG_TIME_KERNEL frames: before / after the render (context stream), before / after
    // the gather and after the assembly (gather stream)
    struct Ev {
        hipEvent_t e[5];
        int frames = 1;  // frames of the batch these events bracket
        bool direct = false;  // one rank: only the render's two events are recorded
    };
    std::vector<Ev> pending, spare;
    double render_ms = 0, gather_ms = 0, assemble_ms = 0;
    uint64_t frames = 0;
    uint32_t rows = 0, max_rows = 0;
};

namespace {

constexpr int kOutputs[3] = {RT_OUT_HDR64, RT_OUT_HDR32, RT_OUT_LDR};
constexpr uint32_t kDefaultBlock = 16;

size_t bytes_per_px(int k) { return k == 0 ? 24 : (k == 1 ? 12 : 3); }

rt_status nccl_fail(ncclResult_t r, const char* what) {
    return fail(RT_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

// ncclInProgress is how a non-blocking communicator's call returns: not an error (comm_wait
// then waits for it).
#define RT_NCCL(call)                                                                \
    do {                                                                             \
        ncclResult_t r_ = (call);                                                    \
        if (r_ != ncclSuccess && r_ != ncclInProgress) return nccl_fail(r_, #call);  \
    } while (0)

// Deadline of a communicator's waits (rt_comm_create; RTAMD_COMM_TIMEOUT_MS overrides; 0 = none).
long default_comm_timeout_ms() {
    const char* e = std::getenv("RTAMD_COMM_TIMEOUT_MS");
    return e ? std::atol(e) : 300000L;
}

using Clock = std::chrono::steady_clock;

bool past(const Clock::time_point& t0, long timeout_ms) {
    return timeout_ms > 0 &&
           std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() >=
               timeout_ms;
}

// Aborts the communicator (its RCCL kernels in flight observe the abort and return) and fails.
rt_status comm_abort(rt_comm* c, const std::string& what, const std::string& why) {
    if (c->nccl) (void)ncclCommAbort(c->nccl);
    c->nccl = nullptr;
    c->aborted = true;
    return fail(RT_ERR_RCCL, what + ": " + why + " (communicator aborted)");
}

rt_status comm_usable(const rt_comm* c, const char* what) {
    if (c->aborted)
        return fail(RT_ERR_RCCL, std::string(what) + ": the communicator was aborted earlier");
    return RT_OK;
}

// Waits until the communicator's last RCCL call has been issued (ncclCommGetAsyncError leaves
// ncclInProgress); an asynchronous error or the deadline aborts it.  Blocking communicators
// (ncclCommInitAll) return at once unless an error is pending.
rt_status comm_wait(rt_comm* c, const char* what) {
    if (!c->nccl) return comm_usable(c, what);
    const Clock::time_point t0 = Clock::now();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(c->nccl, &st);
        if (r != ncclSuccess) st = r;
        if (st == ncclSuccess) return RT_OK;
        if (st != ncclInProgress) return comm_abort(c, what, ncclGetErrorString(st));
        if (past(t0, c->timeout_ms))
            return comm_abort(c, what, "no completion within " + std::to_string(c->timeout_ms) +
                                           " ms");
        std::this_thread::yield();
    }
}

// This rank's share of the frame: rt_render_opts selecting the block-cyclic row set `rank` of
// `n` (a contiguous full frame when n == 1), and the rows it produces.
struct Plan {
    rt_render_opts opts;  // the first slot's
    uint32_t block = 0, rows = 0, max_rows = 0;
    // the split's row sets ("slots"): V = root_weight + n − 1 of them, dealt block-cyclically;
    // rank 0 owns slots [0, root_weight), rank r ≥ 1 slot root_weight + r − 1
    int slots = 1, first_slot = 0, nslots = 1;
    uint32_t slot_rows[64];  // rows of each of this rank's slots
};

// Slot s of a V-slot block-cyclic split of H rows in blocks of b: opts and rows.
void slot_opts(const rt_render_opts& base, uint32_t b, int V, int s, rt_render_opts& o) {
    o = base;
    o.row_begin = static_cast<uint32_t>(s) * b;
    o.row_block = static_cast<uint16_t>(b);
    o.row_cycle = static_cast<uint16_t>(V);
}

rt_status make_plan(const rt_camera* cam, const rt_render_opts* in, int n, int rank, Plan& pl,
                    int weight = 1) {
    rt_render_opts o;
    if (in) o = *in;
    else rt_render_opts_default(&o);
    if (o.row_begin != 0 || (o.row_end != 0 && o.row_end != cam->height) || o.row_cycle > 1)
        return fail(RT_ERR_INVALID_ARG, "multi-GPU frames render the whole image; the row "
                                        "split is their own (set row_block only)");
    const uint32_t H = cam->height;
    pl.block = n == 1 ? H : (o.row_block ? o.row_block : kDefaultBlock);
    o.row_end = H;
    o.row_begin = static_cast<uint32_t>(rank) * pl.block;
    o.row_block = n == 1 ? 0 : static_cast<uint16_t>(pl.block);
    o.row_cycle = n == 1 ? 0 : static_cast<uint16_t>(n);
    pl.opts = o;
    pl.rows = o.row_begin < H ? rendered_rows(o, H) : 0;
    pl.max_rows = 0;
    pl.slots = n;
    pl.first_slot = rank;
    pl.nslots = 1;
    pl.slot_rows[0] = pl.rows;
    if (n > 1 && weight > 1) {  // the weighted split: V slots, rank 0 owns `weight` of them
        const int V = weight + n - 1;
        pl.slots = V;
        pl.first_slot = rank == 0 ? 0 : weight + rank - 1;
        pl.nslots = rank == 0 ? weight : 1;
        pl.rows = 0;
        for (int j = 0; j < pl.nslots; ++j) {
            rt_render_opts q;
            slot_opts(o, pl.block, V, pl.first_slot + j, q);
            pl.slot_rows[j] = q.row_begin < H ? rendered_rows(q, H) : 0;
            pl.rows += pl.slot_rows[j];
        }
        slot_opts(o, pl.block, V, pl.first_slot, pl.opts);
    }
    for (int r = 0; r < pl.slots; ++r) {
        rt_render_opts q;
        slot_opts(o, pl.block, pl.slots, r, q);
        if (n == 1) q = o;
        if (q.row_begin < H) pl.max_rows = std::max(pl.max_rows, rendered_rows(q, H));
    }
    return RT_OK;
}

rt_status check_outputs(int outputs) {
    if (outputs == 0 || (outputs & ~(RT_OUT_HDR64 | RT_OUT_HDR32 | RT_OUT_LDR)))
        return fail(RT_ERR_INVALID_ARG, "outputs must be a non-empty set of RT_OUT_* bits");
    return RT_OK;
}

rt_status harvest(rt_comm* c, bool all) {
    size_t done = 0;
    for (auto& ev : c->pending) {
        const hipEvent_t last = ev.direct ? ev.e[1] : ev.e[4];
        if (!all && hipEventQuery(last) != hipSuccess) break;
        RT_HIP(hipEventSynchronize(last));
        float a = 0, b = 0, d = 0;
        RT_HIP(hipEventElapsedTime(&a, ev.e[0], ev.e[1]));
        if (!ev.direct) {
            RT_HIP(hipEventElapsedTime(&b, ev.e[2], ev.e[3]));
            RT_HIP(hipEventElapsedTime(&d, ev.e[3], ev.e[4]));
        }
        c->render_ms += a;
        c->gather_ms += b;
        c->assemble_ms += d;
        c->frames += static_cast<uint64_t>(ev.frames);
        c->spare.push_back(ev);
        ++done;
    }
    c->pending.erase(c->pending.begin(), c->pending.begin() + static_cast<long>(done));
    return RT_OK;
}

// One frame batch's state on one rank between the phases (nframes frames of one plan).
struct Frame {
    Plan pl;
    rt_comm::Ev* ev = nullptr;
    int slot = 0;
    int nframes = 1;
    bool pipelined = false;
    bool direct = false;       // one rank: rendered into the framebuffers, nothing to gather
    hipStream_t gs = nullptr;  // the stream of the gather and the assembly
};

// Send buffer bytes per output kind k: the render writes frame f's packed rows max_rows rows
// after frame f − 1's (every rank the same frame stride; rows past a rank's own are padding the
// assembly never reads), so the whole batch is ONE ncclGather of nframes·max_rows rows per
// output and rank 0 receives [n][nframes][max_rows] rows.  (Sixteen gathers in one ncclGroup
// cost 75 µs of stream time against 15 µs for one gather of the same bytes, measured on one
// rank: profiles/r04_rccl_group_vs_one.txt.)
size_t send_bytes(const Plan& pl, uint32_t width, int nframes, int k) {
    return static_cast<size_t>(nframes) * pl.max_rows * width * bytes_per_px(k);
}

rt_status record(rt_comm::Ev* ev, int k, hipStream_t s) {
    if (!ev) return RT_OK;
    RT_HIP(hipEventRecord(ev->e[k], s));
    return RT_OK;
}

// Phase 1 of a frame batch on one rank: this rank's rows rendered into its send buffers (the
// gathered outputs) and into the caller's rank-local buffers (`local`, outputs not gathered).
rt_status render_part(rt_comm* c, const rt_scene* sc, const rt_camera* cams, int nframes,
                      const rt_render_opts* opts, int outputs, void* const* dst,
                      void* const* local, Frame& f) {
    rt_context* ctx = c->ctx;
    if (sc->ctx != ctx)
        return fail(RT_ERR_INVALID_ARG, "scene does not belong to the communicator's context");
    const rt_camera* cam = cams;
    rt_status st = make_plan(cam, opts, c->nranks, c->rank, f.pl, c->root_weight);
    if (st != RT_OK) return st;
    Plan& pl = f.pl;
    const bool weighted = pl.slots > c->nranks;  // rank 0's slots land in its receive buffer
    f.nframes = nframes;
    // one rank: its rows are the whole frame in image order, rendered straight into the
    // caller's framebuffers (no send buffer, no gather, no assembly)
    f.direct = c->nranks == 1;
    f.pipelined = !f.direct && (pl.opts.flags & RT_FLAG_PIPELINE) != 0;
    f.slot = f.pipelined ? static_cast<int>(c->frame & 1) : 0;
    f.gs = f.pipelined ? c->gstream : ctx->stream;
    const size_t npx = static_cast<size_t>(pl.max_rows) * cam->width * nframes;
    for (int k = 0; k < 3 && !f.direct; ++k) {
        if (!(outputs & kOutputs[k])) continue;
        if (!(weighted && c->rank == 0))
            RT_HIP(c->send[f.slot][k].ensure(send_bytes(pl, cam->width, nframes, k)));
        if (c->rank == 0)
            RT_HIP(c->recv[f.slot][k].ensure(npx * bytes_per_px(k) * static_cast<size_t>(pl.slots)));
    }
    c->rows = pl.rows;
    c->max_rows = pl.max_rows;
    f.ev = nullptr;
    if (pl.opts.flags & RT_FLAG_TIME_KERNEL) {
        if (c->pending.size() >= 256) {
            st = harvest(c, false);
            if (st != RT_OK) return st;
        }
        c->pending.emplace_back();
        rt_comm::Ev& e = c->pending.back();
        if (!c->spare.empty()) {
            e = c->spare.back();
            c->spare.pop_back();
        } else {
            for (auto& x : e.e) RT_HIP(hipEventCreate(&x));
        }
        e.frames = nframes;
        e.direct = f.direct;
        f.ev = &e;
    }
    // the frame's own events replace the per-launch ones of the render
    pl.opts.flags &= ~(RT_FLAG_TIME_KERNEL | RT_FLAG_PIPELINE);
    const bool ldr = (outputs & RT_OUT_LDR) || (local && local[2]);
    if (!ldr) pl.opts.tonemap = RT_TONEMAP_NONE;
    else if (pl.opts.tonemap == RT_TONEMAP_NONE)
        return fail(RT_ERR_INVALID_ARG, "RT_OUT_LDR needs opts->tonemap");
    // the slot's buffers (and, for a serial frame, the caller's framebuffers) may still be in
    // use by an earlier pipelined frame's gather / assembly
    for (int s = 0; s < 2; ++s)
        if (c->slot_used[s] && (s == f.slot || !f.pipelined))
            RT_HIP(hipStreamWaitEvent(ctx->stream, c->freed[s], 0));
    st = record(f.ev, 0, ctx->stream);
    if (st != RT_OK) return st;
    // each of this rank's slots: all frames in one launch, frames max_rows rows apart; a slot's
    // outputs follow the previous slot's (rank-local outputs), or — rank 0 of a weighted split —
    // sit at the slot's place in the receive buffer, where the assembly reads them
    const size_t slot_px = static_cast<size_t>(nframes) * pl.max_rows * cam->width;
    for (int j = 0; j < pl.nslots; ++j) {
        if (pl.slot_rows[j] == 0) continue;
        rt_render_opts so = pl.opts;
        if (weighted) slot_opts(pl.opts, pl.block, pl.slots, pl.first_slot + j, so);
        void* out[3];
        for (int k = 0; k < 3; ++k) {
            const size_t off = j * slot_px * 3;  // elements
            char* base;
            if (!(outputs & kOutputs[k])) {
                base = local && local[k] ? static_cast<char*>(local[k]) + off * (k == 0 ? 8 : k == 1 ? 4 : 1)
                                         : nullptr;
            } else if (f.direct) {
                base = static_cast<char*>(dst[k]);
            } else if (weighted && c->rank == 0) {
                base = static_cast<char*>(c->recv[f.slot][k].ptr) +
                       static_cast<size_t>(pl.first_slot + j) * slot_px * bytes_per_px(k);
            } else {
                base = static_cast<char*>(c->send[f.slot][k].ptr);
            }
            out[k] = base;
        }
        st = enqueue_frames(ctx, sc, cams, nframes, &so, static_cast<double*>(out[0]),
                            static_cast<float*>(out[1]), static_cast<uint8_t*>(out[2]),
                            pl.max_rows);
        if (st != RT_OK) return st;
    }
    st = record(f.ev, 1, ctx->stream);
    if (st != RT_OK) return st;
    if (f.pipelined) {
        RT_HIP(hipEventRecord(c->rendered[f.slot], ctx->stream));
        RT_HIP(hipStreamWaitEvent(f.gs, c->rendered[f.slot], 0));
    }
    return f.direct ? RT_OK : record(f.ev, 2, f.gs);
}

// A batch whose render was enqueued but whose gather or assembly then failed: rt_comm_destroy
// must still wait for the render (it writes the send / receive buffers) — its `done` event is
// recorded behind it here, since assemble_part never ran.
rt_status after_failed_frame(rt_comm* c, rt_status st) {
    if (c->ctx && c->ctx->stream && hipEventRecord(c->done, c->ctx->stream) == hipSuccess)
        c->any_frame = true;
    return st;
}

// Phase 2: one ncclGather per output of the whole batch (inside the caller's group): the send
// buffer's nframes·max_rows rows land in slot `rank` of rank 0's receive buffer.
rt_status gather_part(rt_comm* c, const rt_camera* cam, int outputs, const Frame& f) {
    if (f.direct) return RT_OK;
    if (f.pl.slots > c->nranks) {
        // weighted split: rank 0's own slots are already in place; each other rank's one slot
        // goes to its place in rank 0's receive buffer (grouped P2P, equal counts)
        const int w = f.pl.slots - c->nranks + 1;
        for (int k = 0; k < 3; ++k) {
            if (!(outputs & kOutputs[k])) continue;
            const size_t count = send_bytes(f.pl, cam->width, f.nframes, k);
            if (c->rank == 0) {
                char* recv = static_cast<char*>(c->recv[f.slot][k].ptr);
                for (int r = 1; r < c->nranks; ++r)
                    RT_NCCL(ncclRecv(recv + static_cast<size_t>(w + r - 1) * count, count,
                                     ncclUint8, r, c->nccl, f.gs));
            } else {
                RT_NCCL(ncclSend(c->send[f.slot][k].ptr, count, ncclUint8, 0, c->nccl, f.gs));
            }
        }
        return RT_OK;
    }
    for (int k = 0; k < 3; ++k) {
        if (!(outputs & kOutputs[k])) continue;
        char* send = static_cast<char*>(c->send[f.slot][k].ptr);
        char* recv = c->rank == 0 ? static_cast<char*>(c->recv[f.slot][k].ptr) : send;
        RT_NCCL(ncclGather(send, recv, send_bytes(f.pl, cam->width, f.nframes, k), ncclUint8, 0,
                           c->nccl, f.gs));
    }
    return RT_OK;
}

// Phase 2 of local communicators (rt_comm_create_local, every rank in this process): rank r's
// padded send buffer into slot r of rank 0's receive buffer, as ncclGather lays it out.  Rank
// 0's gather stream waits for every rank's rows; every other rank's gather stream then waits
// for rank 0's copies, so its send slot is handed back (freed) only once it has been read.
rt_status gather_local(rt_comm* const* comms, int n, const rt_camera* cam, int outputs,
                       const std::vector<Frame>& f) {
    rt_comm* root = comms[0];
    const Frame& f0 = f[0];
    if (f0.direct) return RT_OK;
    for (int i = 0; i < n; ++i) {
        rt_comm* c = comms[i];
        if (f[i].gs != f0.gs) {
            DeviceGuard g(c->device);
            RT_HIP(hipEventRecord(c->xfer_ready, f[i].gs));
            DeviceGuard g0(root->device);
            RT_HIP(hipStreamWaitEvent(f0.gs, c->xfer_ready, 0));
        }
    }
    DeviceGuard g0(root->device);
    for (int k = 0; k < 3; ++k) {
        if (!(outputs & kOutputs[k])) continue;
        const size_t bytes = send_bytes(f0.pl, cam->width, f0.nframes, k);
        char* recv = static_cast<char*>(root->recv[f0.slot][k].ptr);
        // weighted split: rank 0's slots are in place, rank i's slot is w + i − 1
        const int w = f0.pl.slots - n + 1;
        for (int i = (w > 1 ? 1 : 0); i < n; ++i) {  // rank i's whole batch into its slot
            const void* send = comms[i]->send[f[i].slot][k].ptr;
            const size_t at = static_cast<size_t>(w > 1 ? w + i - 1 : i) * bytes;
            if (comms[i]->device == root->device)
                RT_HIP(hipMemcpyAsync(recv + at, send, bytes, hipMemcpyDeviceToDevice, f0.gs));
            else
                RT_HIP(hipMemcpyPeerAsync(recv + at, root->device, send, comms[i]->device, bytes,
                                          f0.gs));
        }
    }
    RT_HIP(hipEventRecord(root->xfer_done, f0.gs));
    for (int i = 1; i < n; ++i) {
        if (f[i].gs == f0.gs) continue;
        DeviceGuard g(comms[i]->device);
        RT_HIP(hipStreamWaitEvent(f[i].gs, root->xfer_done, 0));
    }
    return RT_OK;
}

// Phase 3 (rank 0): gathered rows into image order in the caller's device framebuffers.
rt_status assemble_part(rt_comm* c, const rt_camera* cam, int outputs, const Frame& f,
                        void* const* dst) {
    rt_status st = f.direct ? RT_OK : record(f.ev, 3, f.gs);
    if (st != RT_OK) return st;
    if (c->rank == 0 && !f.direct) {
        for (int k = 0; k < 3; ++k) {
            if (!(outputs & kOutputs[k]) || !dst[k]) continue;
            RT_HIP(launch_assemble_rows(c->recv[f.slot][k].ptr, dst[k],
                                        size_t(cam->width) * bytes_per_px(k), cam->height,
                                        f.pl.block, static_cast<uint32_t>(f.pl.slots),
                                        f.pl.max_rows, static_cast<uint32_t>(f.nframes), f.gs));
        }
    }
    st = f.direct ? RT_OK : record(f.ev, 4, f.gs);
    if (st != RT_OK) return st;
    if (f.pipelined) {
        RT_HIP(hipEventRecord(c->freed[f.slot], f.gs));
        c->slot_used[f.slot] = true;
    } else {
        RT_HIP(hipEventRecord(c->done, f.gs));
    }
    c->any_frame = true;
    c->frame += 1;
    return RT_OK;
}

// The gather stream and the slot hand-over events (the caller holds a DeviceGuard).
rt_status init_streams(rt_comm* c) {
    RT_HIP(hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking));
    RT_HIP(hipEventCreateWithFlags(&c->xfer_ready, hipEventDisableTiming));
    RT_HIP(hipEventCreateWithFlags(&c->xfer_done, hipEventDisableTiming));
    RT_HIP(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    for (int s = 0; s < 2; ++s) {
        RT_HIP(hipEventCreateWithFlags(&c->rendered[s], hipEventDisableTiming));
        RT_HIP(hipEventCreateWithFlags(&c->freed[s], hipEventDisableTiming));
    }
    return RT_OK;
}

rt_status check_root_outputs(const rt_comm* c, int outputs, void* const* dst) {
    if (c->rank != 0) return RT_OK;
    for (int k = 0; k < 3; ++k)
        if ((outputs & kOutputs[k]) && !dst[k])
            return fail(RT_ERR_INVALID_ARG, "rank 0 needs a device framebuffer for every "
                                            "requested output");
    return RT_OK;
}

// RTAMD_MULTI_HOST=1: the same block-cyclic split, each context's rows copied straight into the
// caller's host rows (every device's copies are enqueued before the first synchronisation, so
// the devices' transfers overlap).
rt_status render_multi_host(rt_context* const* ctxs, rt_scene* const* scenes, int n,
                            const rt_camera* cam, const rt_render_opts* opts, double* h64,
                            float* h32, uint8_t* hldr, rt_stats* stats) {
    // (arguments validated by rt_render_multi)
    rt_status st = RT_OK;
    rt_render_opts base;
    if (opts) base = *opts;
    else rt_render_opts_default(&base);
    if (base.row_begin != 0 || (base.row_end != 0 && base.row_end != cam->height) ||
        base.row_cycle > 1)
        return fail(RT_ERR_INVALID_ARG, "rt_render_multi renders the whole image; the row "
                                        "split is its own (row_block only)");
    if (stats) base.flags |= RT_FLAG_COUNT_RAYS;
    const uint32_t H = cam->height, W = cam->width;
    const uint32_t block = n == 1 ? 0 : (base.row_block ? base.row_block : 16);
    std::vector<rt_render_opts> o(static_cast<size_t>(n), base);
    std::vector<uint32_t> rows(static_cast<size_t>(n));
    // 1. every context renders its rows (block-cyclic) into its own device buffers, async
    for (int i = 0; i < n; ++i) {
        rt_context* ctx = ctxs[i];
        DeviceGuard g(ctx->device);
        o[i].row_end = H;
        if (block) {
            o[i].row_begin = static_cast<uint32_t>(i) * block;
            o[i].row_block = static_cast<uint16_t>(block);
            o[i].row_cycle = static_cast<uint16_t>(n);
            if (o[i].row_begin >= H) {
                rows[i] = 0;
                continue;
            }
        }
        rows[i] = rendered_rows(o[i], H);
        const size_t npx = static_cast<size_t>(rows[i]) * W;
        if (h64) RT_HIP(ctx->out64.ensure(npx * 3 * sizeof(double)));
        if (h32) RT_HIP(ctx->out32.ensure(npx * 3 * sizeof(float)));
        if (hldr) RT_HIP(ctx->ldr.ensure(npx * 3));
        if (stats)
            RT_HIP(hipMemsetAsync(ctx->counters.ptr, 0, 2 * sizeof(unsigned long long),
                                  ctx->stream));
        st = enqueue_render(ctx, scenes[i], cam, &o[i],
                     h64 ? static_cast<double*>(ctx->out64.ptr) : nullptr,
                     h32 ? static_cast<float*>(ctx->out32.ptr) : nullptr,
                     hldr ? static_cast<uint8_t*>(ctx->ldr.ptr) : nullptr);
        if (st != RT_OK) return st;
    }
    // 2. gather: each context's packed rows back to their image rows in the caller's buffers
    if (stats) std::memset(stats, 0, sizeof *stats);
    for (int i = 0; i < n; ++i) {
        if (rows[i] == 0) continue;
        rt_context* ctx = ctxs[i];
        DeviceGuard g(ctx->device);
        const size_t row64 = size_t(W) * 3 * sizeof(double), row32 = size_t(W) * 3 * sizeof(float),
                     row8 = size_t(W) * 3;
        uint32_t k = 0;  // packed row of this context
        for (uint32_t b0 = o[i].row_begin; b0 < H; b0 += block ? block * n : H) {
            const uint32_t nb = block ? std::min(block, H - b0) : rows[i];
            if (h64)
                RT_HIP(hipMemcpyAsync(reinterpret_cast<char*>(h64) + b0 * row64,
                                      static_cast<char*>(ctx->out64.ptr) + k * row64, nb * row64,
                                      hipMemcpyDeviceToHost, ctx->stream));
            if (h32)
                RT_HIP(hipMemcpyAsync(reinterpret_cast<char*>(h32) + b0 * row32,
                                      static_cast<char*>(ctx->out32.ptr) + k * row32, nb * row32,
                                      hipMemcpyDeviceToHost, ctx->stream));
            if (hldr)
                RT_HIP(hipMemcpyAsync(hldr + b0 * row8, static_cast<char*>(ctx->ldr.ptr) + k * row8,
                                      nb * row8, hipMemcpyDeviceToHost, ctx->stream));
            k += nb;
        }
    }
    for (int i = 0; i < n; ++i) {
        rt_context* ctx = ctxs[i];
        DeviceGuard g(ctx->device);
        RT_HIP(hipStreamSynchronize(ctx->stream));
        if (o[i].flags & RT_FLAG_TIME_KERNEL) {
            st = harvest_events(ctx, true);
            if (st != RT_OK) return st;
        }
        if (rows[i] == 0 || !stats) continue;
        {
            unsigned long long c[2] = {0, 0};
            RT_HIP(hipMemcpy(c, ctx->counters.ptr, sizeof c, hipMemcpyDeviceToHost));
            stats->trace_rays += c[0];
            stats->shadow_rays += c[1];
            stats->kernel_ms += ctx->timed_ms;
            stats->launches += ctx->launches;
        }
    }
    return RT_OK;
}

// One frame over n contexts into host framebuffers (rt_capi.h rt_render_multi).  Distinct GPUs:
// the RCCL path — communicators over the contexts' devices (ncclCommInitAll, cached in ctxs[0]
// until the context list changes), rt_render_gather_all into ctxs[0]'s device framebuffers,
// one device-to-host copy per output from rank 0.  Contexts sharing a GPU: the same with local
// communicators (rt_comm_create_local: the gather as device copies).
rt_status render_multi_group(rt_context* const* ctxs, rt_scene* const* scenes, int n,
                             const rt_camera* cam, const rt_render_opts* opts, int outputs,
                             bool local, double* h64, float* h32, uint8_t* hldr,
                             rt_stats* stats) {
    rt_context* root = ctxs[0];
    bool same = root->group_ctxs.size() == static_cast<size_t>(n);
    for (int i = 0; same && i < n; ++i)
        same = root->group_ctxs[i] == ctxs[i] && root->group_comms[i]->device == ctxs[i]->device &&
               root->group_comms[i]->local == local;
    if (!same) {
        release_group(root);
        std::vector<rt_comm*> comms(static_cast<size_t>(n), nullptr);
        rt_status st = local ? rt_comm_create_local(ctxs, n, comms.data())
                             : rt_comm_create_all(ctxs, n, comms.data());
        if (st != RT_OK) return st;
        root->group_ctxs.assign(ctxs, ctxs + n);
        root->group_comms = comms;
        // every member knows the group it is in, so destroying any of them first releases it
        for (int i = 1; i < n; ++i) ctxs[i]->group_roots.push_back(root);
    }
    for (int i = 0; i < n; ++i) root->group_comms[i]->ctx = ctxs[i];
    rt_render_opts o;
    if (opts) o = *opts;
    else rt_render_opts_default(&o);
    if (stats) o.flags |= RT_FLAG_COUNT_RAYS;
    // the device-to-host copies below run on root->stream: a pipelined frame would gather and
    // assemble on the communicators' own streams, unordered with them (one-shot host frames
    // gain nothing from the pipeline anyway)
    o.flags &= ~RT_FLAG_PIPELINE;
    if (stats)
        for (int i = 0; i < n; ++i) {
            DeviceGuard g(ctxs[i]->device);
            RT_HIP(hipMemsetAsync(ctxs[i]->counters.ptr, 0, 2 * sizeof(unsigned long long),
                                  ctxs[i]->stream));
        }
    const size_t npx = static_cast<size_t>(cam->width) * cam->height;
    {
        DeviceGuard g(root->device);
        if (h64) RT_HIP(root->out64.ensure(npx * 3 * sizeof(double)));
        if (h32) RT_HIP(root->out32.ensure(npx * 3 * sizeof(float)));
        if (hldr) RT_HIP(root->ldr.ensure(npx * 3));
    }
    rt_status st = rt_render_gather_all(root->group_comms.data(), scenes, n, cam, &o, outputs,
                                        h64 ? root->out64.ptr : nullptr,
                                        h32 ? root->out32.ptr : nullptr,
                                        hldr ? root->ldr.ptr : nullptr);
    if (st != RT_OK) return st;
    {
        DeviceGuard g(root->device);
        if (h64)
            RT_HIP(hipMemcpyAsync(h64, root->out64.ptr, npx * 3 * sizeof(double),
                                  hipMemcpyDeviceToHost, root->stream));
        if (h32)
            RT_HIP(hipMemcpyAsync(h32, root->out32.ptr, npx * 3 * sizeof(float),
                                  hipMemcpyDeviceToHost, root->stream));
        if (hldr)
            RT_HIP(hipMemcpyAsync(hldr, root->ldr.ptr, npx * 3, hipMemcpyDeviceToHost,
                                  root->stream));
    }
    if (stats) std::memset(stats, 0, sizeof *stats);
    for (int i = 0; i < n; ++i) {
        DeviceGuard g(ctxs[i]->device);
        RT_HIP(hipStreamSynchronize(ctxs[i]->stream));
        if (!stats) continue;
        unsigned long long c[2] = {0, 0};
        RT_HIP(hipMemcpy(c, ctxs[i]->counters.ptr, sizeof c, hipMemcpyDeviceToHost));
        stats->trace_rays += c[0];
        stats->shadow_rays += c[1];
    }
    if (stats && (o.flags & RT_FLAG_TIME_KERNEL)) {  // the frame's render time on the slowest GPU
        for (int i = 0; i < n; ++i) {
            rt_gather_timing t;
            st = rt_comm_timing(root->group_comms[i], &t, 1);
            if (st != RT_OK) return st;
            stats->kernel_ms = std::max(stats->kernel_ms, t.render_ms);
        }
        stats->launches = 1;
    }
    return RT_OK;
}

}  // namespace

extern "C" {

rt_status rt_render_multi(rt_context* const* ctxs, rt_scene* const* scenes, int n,
                          const rt_camera* cam, const rt_render_opts* opts, double* h64,
                          float* h32, uint8_t* hldr, rt_stats* stats) {
    if (n < 1 || !ctxs || !scenes) return fail(RT_ERR_INVALID_ARG, "rt_render_multi: n < 1 or NULL");
    bool distinct = true;
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i] || !scenes[i] || scenes[i]->ctx != ctxs[i])
            return fail(RT_ERR_INVALID_ARG, "rt_render_multi: scene " + std::to_string(i) +
                                                " missing or not of context " + std::to_string(i));
        for (int j = 0; j < i; ++j) {
            if (ctxs[j] == ctxs[i])  // each context renders into its own buffers
                return fail(RT_ERR_INVALID_ARG, "rt_render_multi: context repeated");
            if (ctxs[j]->device == ctxs[i]->device) distinct = false;
        }
    }
    rt_status st = validate_camera(cam);
    if (st != RT_OK) return st;
    const int outputs = (h64 ? RT_OUT_HDR64 : 0) | (h32 ? RT_OUT_HDR32 : 0) |
                        (hldr ? RT_OUT_LDR : 0);
    const char* env = std::getenv("RTAMD_MULTI_HOST");  // force the host assembly (tests)
    if (outputs && !(env && std::atoi(env) == 1)) {
        rt_render_opts o;
        if (opts) o = *opts;
        else rt_render_opts_default(&o);
        if (!hldr) o.tonemap = RT_TONEMAP_NONE;
        return render_multi_group(ctxs, scenes, n, cam, &o, outputs, !distinct, h64, h32, hldr,
                                  stats);
    }
    return render_multi_host(ctxs, scenes, n, cam, opts, h64, h32, hldr, stats);
}

}  // extern "C"

namespace rtamd {

void release_group(rt_context* ctx) {
    for (rt_comm* c : ctx->group_comms) rt_comm_destroy(c);
    for (rt_context* m : ctx->group_ctxs) {
        if (m == ctx) continue;
        auto& roots = m->group_roots;
        roots.erase(std::remove(roots.begin(), roots.end(), ctx), roots.end());
    }
    ctx->group_comms.clear();
    ctx->group_ctxs.clear();
}

void leave_groups(rt_context* ctx) {
    // the groups other contexts lead that include ctx: released before ctx goes away (their
    // communicators hold raw pointers to it); release_group edits ctx->group_roots, so copy
    const std::vector<rt_context*> roots = ctx->group_roots;
    for (rt_context* r : roots) release_group(r);
    ctx->group_roots.clear();
    release_group(ctx);
}

}  // namespace rtamd

extern "C" {

rt_status rt_comm_unique_id(uint8_t* id) {
    if (!id) return fail(RT_ERR_INVALID_ARG, "id is NULL");
    ncclUniqueId u;
    RT_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, sizeof u.internal);
    return RT_OK;
}

rt_status rt_comm_create(rt_context* ctx, int nranks, int rank, const uint8_t* id,
                         rt_comm** out) {
    return rt_comm_create_ex(ctx, nranks, rank, id, default_comm_timeout_ms(), out);
}

rt_status rt_comm_create_ex(rt_context* ctx, int nranks, int rank, const uint8_t* id,
                            long timeout_ms, rt_comm** out) {
    if (!ctx || !id || !out) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_comm_create");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return fail(RT_ERR_INVALID_ARG, "rank must be in [0, nranks)");
    if (timeout_ms < 0) return fail(RT_ERR_INVALID_ARG, "timeout_ms must be >= 0");
    *out = nullptr;
    DeviceGuard g(ctx->device);
    rt_comm* c = new (std::nothrow) rt_comm();
    if (!c) return fail(RT_ERR_OOM, "host allocation failed");
    c->ctx = ctx;
    c->device = ctx->device;
    c->nranks = nranks;
    c->rank = rank;
    c->timeout_ms = timeout_ms;
    rt_status st = init_streams(c);
    if (st != RT_OK) {
        rt_comm_destroy(c);
        return st;
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, sizeof u.internal);
    // Non-blocking initialisation: a rank that never joins (a dead or missing peer process)
    // makes the init time out here instead of blocking this rank forever.
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const ncclResult_t r = ncclCommInitRankConfig(&c->nccl, nranks, u, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        if (c->nccl) (void)ncclCommAbort(c->nccl);
        c->nccl = nullptr;
        rt_comm_destroy(c);
        return nccl_fail(r, "ncclCommInitRankConfig");
    }
    c->nonblocking = true;
    st = comm_wait(c, "ncclCommInitRankConfig");
    if (st != RT_OK) {
        const std::string msg = rt_last_error();
        rt_comm_destroy(c);
        return fail(st, msg);
    }
    *out = c;
    return RT_OK;
}

rt_status rt_comm_set_timeout(rt_comm* c, long timeout_ms) {
    if (!c) return fail(RT_ERR_INVALID_ARG, "comm is NULL");
    if (timeout_ms < 0) return fail(RT_ERR_INVALID_ARG, "timeout_ms must be >= 0");
    c->timeout_ms = timeout_ms;
    return RT_OK;
}

rt_status rt_comm_create_all(rt_context* const* ctxs, int n, rt_comm** out) {
    if (!ctxs || !out || n < 1) return fail(RT_ERR_INVALID_ARG, "rt_comm_create_all: n < 1 or NULL");
    std::vector<int> devs(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) return fail(RT_ERR_INVALID_ARG, "rt_comm_create_all: NULL context");
        devs[i] = ctxs[i]->device;
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i])  // RCCL: one rank per GPU
                return fail(RT_ERR_INVALID_ARG, "rt_comm_create_all: device " +
                                                    std::to_string(devs[i]) + " repeated");
    }
    std::vector<ncclComm_t> comms(static_cast<size_t>(n), nullptr);
    {
        DeviceGuard g(devs[0]);
        RT_NCCL(ncclCommInitAll(comms.data(), n, devs.data()));
    }
    for (int i = 0; i < n; ++i) {
        rt_comm* c = new (std::nothrow) rt_comm();
        if (!c) {
            for (int j = 0; j < i; ++j) rt_comm_destroy(out[j]);
            for (int j = i; j < n; ++j) (void)ncclCommDestroy(comms[j]);
            return fail(RT_ERR_OOM, "host allocation failed");
        }
        c->ctx = ctxs[i];
        c->device = devs[i];
        c->nccl = comms[i];
        c->nranks = n;
        c->rank = i;
        out[i] = c;
        DeviceGuard g(devs[i]);
        rt_status st = init_streams(c);
        if (st != RT_OK) {
            for (int j = 0; j <= i; ++j) rt_comm_destroy(out[j]);
            for (int j = i + 1; j < n; ++j) (void)ncclCommDestroy(comms[j]);
            return st;
        }
    }
    return RT_OK;
}

rt_status rt_comm_create_local(rt_context* const* ctxs, int n, rt_comm** out) {
    if (!ctxs || !out || n < 1) return fail(RT_ERR_INVALID_ARG, "rt_comm_create_local: n < 1 or NULL");
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) return fail(RT_ERR_INVALID_ARG, "rt_comm_create_local: NULL context");
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i])  // each rank renders into its own buffers on its own stream
                return fail(RT_ERR_INVALID_ARG, "rt_comm_create_local: context repeated");
    }
    std::vector<rt_comm*> peers(static_cast<size_t>(n), nullptr);
    for (int i = 0; i < n; ++i) {
        rt_comm* c = new (std::nothrow) rt_comm();
        rt_status st = c ? RT_OK : fail(RT_ERR_OOM, "host allocation failed");
        if (c) {
            c->ctx = ctxs[i];
            c->device = ctxs[i]->device;
            c->local = true;
            c->nranks = n;
            c->rank = i;
            peers[static_cast<size_t>(i)] = c;
            DeviceGuard g(c->device);
            st = init_streams(c);
        }
        if (st != RT_OK) {
            for (rt_comm* p : peers) rt_comm_destroy(p);
            return st;
        }
    }
    for (int i = 0; i < n; ++i) {
        peers[static_cast<size_t>(i)]->peers = peers;
        out[i] = peers[static_cast<size_t>(i)];
    }
    return RT_OK;
}

rt_status rt_comm_destroy(rt_comm* c) {
    if (!c) return RT_OK;
    DeviceGuard g(c->device);
    // Every frame's last step is recorded on an event of this comm (`freed` of its slot when
    // pipelined — its stream waited for the render first — else `done` on the render stream,
    // which the gather and assembly share): wait for those, not for the whole device (other
    // contexts' frames keep running).
    if (c->any_frame) {
        for (int s = 0; s < 2; ++s)
            if (c->slot_used[s]) (void)hipEventSynchronize(c->freed[s]);
        (void)hipEventSynchronize(c->done);
    }
    if (c->nccl && c->nonblocking) {
        // a non-blocking communicator is finalized (its outstanding operations flushed) before
        // it is freed; one that does not finish within the deadline is aborted instead
        const ncclResult_t r = ncclCommFinalize(c->nccl);
        if (r != ncclSuccess && r != ncclInProgress) (void)comm_abort(c, "ncclCommFinalize", ncclGetErrorString(r));
        else (void)comm_wait(c, "ncclCommFinalize");
    }
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    c->chk.release();
    for (auto* v : {&c->pending, &c->spare})
        for (auto& ev : *v)
            for (auto& x : ev.e) (void)hipEventDestroy(x);
    for (int s = 0; s < 2; ++s) {
        for (int k = 0; k < 3; ++k) {
            c->send[s][k].release();
            c->recv[s][k].release();
        }
        if (c->rendered[s]) (void)hipEventDestroy(c->rendered[s]);
        if (c->freed[s]) (void)hipEventDestroy(c->freed[s]);
    }
    if (c->xfer_ready) (void)hipEventDestroy(c->xfer_ready);
    if (c->xfer_done) (void)hipEventDestroy(c->xfer_done);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->gstream) (void)hipStreamDestroy(c->gstream);
    delete c;
    return RT_OK;
}

rt_status rt_comm_synchronize(rt_comm* c) {
    if (!c) return fail(RT_ERR_INVALID_ARG, "comm is NULL");
    DeviceGuard g(c->device);
    if (c->local || c->nranks == 1 || c->timeout_ms == 0 || !c->nccl) {
        RT_HIP(hipStreamSynchronize(c->ctx->stream));
        RT_HIP(hipStreamSynchronize(c->gstream));
        return comm_usable(c, "rt_comm_synchronize");
    }
    // Polls both streams and the communicator: a gather whose peer never arrives (a rank that
    // died or diverged) ends in an asynchronous RCCL error or the deadline, and the abort makes
    // its kernels return instead of spinning on the GPU for ever.
    const Clock::time_point t0 = Clock::now();
    for (;;) {
        const hipError_t a = hipStreamQuery(c->ctx->stream);
        const hipError_t b = hipStreamQuery(c->gstream);
        if (a == hipSuccess && b == hipSuccess) return RT_OK;
        if (a != hipSuccess && a != hipErrorNotReady) return hip_fail(a, "hipStreamQuery");
        if (b != hipSuccess && b != hipErrorNotReady) return hip_fail(b, "hipStreamQuery");
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(c->nccl, &st);
        if (r != ncclSuccess) st = r;
        if (st != ncclSuccess && st != ncclInProgress)
            return comm_abort(c, "rt_comm_synchronize", ncclGetErrorString(st));
        if (past(t0, c->timeout_ms))
            return comm_abort(c, "rt_comm_synchronize",
                              "frames not finished within " + std::to_string(c->timeout_ms) + " ms");
        std::this_thread::yield();
    }
}

rt_status rt_render_gather(rt_comm* c, const rt_scene* sc, const rt_camera* cam,
                           const rt_render_opts* opts, int outputs, void* d_hdr64,
                           void* d_hdr32, void* d_ldr) {
    if (!c || !sc) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_render_gather");
    return rt_render_gather_batch(c, sc, cam, 1, opts, outputs, d_hdr64, d_hdr32, d_ldr,
                                  nullptr, nullptr, nullptr);
}

rt_status rt_render_gather_batch(rt_comm* c, const rt_scene* sc, const rt_camera* cams,
                                 int nframes, const rt_render_opts* opts, int outputs,
                                 void* d_hdr64, void* d_hdr32, void* d_ldr, void* rank_hdr64,
                                 void* rank_hdr32, void* rank_ldr) {
    if (!c || !sc) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_render_gather_batch");
    rt_status st = check_batch(cams, nframes);
    if (st == RT_OK) st = check_outputs(outputs);
    void* const dst[3] = {d_hdr64, d_hdr32, d_ldr};
    void* const local[3] = {rank_hdr64, rank_hdr32, rank_ldr};
    if (st == RT_OK) st = check_root_outputs(c, outputs, dst);
    if (st != RT_OK) return st;
    for (int k = 0; k < 3; ++k)
        if ((outputs & kOutputs[k]) && local[k])
            return fail(RT_ERR_INVALID_ARG, "an output is either gathered or rank-local");
    if (c->local && c->nranks > 1)
        return fail(RT_ERR_INVALID_ARG, "local communicators (rt_comm_create_local) gather "
                                        "through rt_render_gather_all");
    st = comm_usable(c, "rt_render_gather_batch");
    if (st != RT_OK) return st;
    DeviceGuard g(c->device);
    Frame f;
    st = render_part(c, sc, cams, nframes, opts, outputs, dst, local, f);
    if (st != RT_OK) return st;
    if (!f.direct) {
        const ncclResult_t r0 = ncclGroupStart();
        if (r0 != ncclSuccess) return after_failed_frame(c, nccl_fail(r0, "ncclGroupStart"));
        st = gather_part(c, cams, outputs, f);
        const ncclResult_t r1 = ncclGroupEnd();
        if (st != RT_OK) return after_failed_frame(c, st);
        if (r1 != ncclSuccess && r1 != ncclInProgress)
            return after_failed_frame(c, nccl_fail(r1, "ncclGroupEnd"));
        st = comm_wait(c, "ncclGather");
        if (st != RT_OK) return after_failed_frame(c, st);
    }
    st = assemble_part(c, cams, outputs, f, dst);
    return st == RT_OK ? st : after_failed_frame(c, st);
}

rt_status rt_render_gather_all(rt_comm* const* comms, rt_scene* const* scenes, int n,
                               const rt_camera* cam, const rt_render_opts* opts, int outputs,
                               void* d_hdr64, void* d_hdr32, void* d_ldr) {
    return rt_render_gather_all_batch(comms, scenes, n, cam, 1, opts, outputs, d_hdr64, d_hdr32,
                                      d_ldr);
}

rt_status rt_render_gather_all_batch(rt_comm* const* comms, rt_scene* const* scenes, int n,
                                     const rt_camera* cams, int nframes,
                                     const rt_render_opts* opts, int outputs, void* d_hdr64,
                                     void* d_hdr32, void* d_ldr) {
    if (!comms || !scenes || n < 1) return fail(RT_ERR_INVALID_ARG, "rt_render_gather_all: n < 1 or NULL");
    rt_status st = check_batch(cams, nframes);
    if (st == RT_OK) st = check_outputs(outputs);
    if (st != RT_OK) return st;
    for (int i = 0; i < n; ++i)
        if (!comms[i] || !scenes[i] || comms[i]->nranks != n || comms[i]->rank != i ||
            comms[i]->local != comms[0]->local ||
            (comms[0]->local && comms[0]->peers[static_cast<size_t>(i)] != comms[i]))
            return fail(RT_ERR_INVALID_ARG, "rt_render_gather_all: comms must be the n ranks of "
                                            "one rt_comm_create_all / rt_comm_create_local, in "
                                            "rank order");
    for (int i = 0; i < n; ++i) {
        // every rank sizes its send buffer and rank 0 its receive slots from the same split
        if (comms[i]->root_weight != comms[0]->root_weight)
            return fail(RT_ERR_INVALID_ARG, "rt_render_gather_all: rank " + std::to_string(i) +
                                                " has root weight " +
                                                std::to_string(comms[i]->root_weight) +
                                                ", rank 0 " +
                                                std::to_string(comms[0]->root_weight));
        st = comm_usable(comms[i], "rt_render_gather_all");
        if (st != RT_OK) return st;
    }
    void* const dst[3] = {d_hdr64, d_hdr32, d_ldr};
    st = check_root_outputs(comms[0], outputs, dst);
    if (st != RT_OK) return st;
    std::vector<Frame> f(static_cast<size_t>(n));
    int rendered = 0;  // ranks whose render is enqueued: on failure, destroy waits for them
    auto failed = [&](rt_status e) {
        for (int i = 0; i < rendered; ++i) {
            DeviceGuard g(comms[i]->device);
            (void)after_failed_frame(comms[i], e);
        }
        return e;
    };
    for (int i = 0; i < n; ++i) {  // 1. every GPU renders its rows (asynchronous)
        DeviceGuard g(comms[i]->device);
        st = render_part(comms[i], scenes[i], cams, nframes, opts, outputs, dst, nullptr, f[i]);
        if (st != RT_OK) return failed(st);
        rendered = i + 1;
    }
    if (comms[0]->local) {  // 2. the gather as device copies into rank 0's receive buffer
        st = gather_local(comms, n, cams, outputs, f);
        if (st != RT_OK) return failed(st);
    } else if (!f[0].direct) {  // 2. one gather per frame and output over all GPUs
        const ncclResult_t r0 = ncclGroupStart();
        if (r0 != ncclSuccess) return failed(nccl_fail(r0, "ncclGroupStart"));
        for (int i = 0; i < n && st == RT_OK; ++i) {
            DeviceGuard g(comms[i]->device);
            st = gather_part(comms[i], cams, outputs, f[i]);
        }
        const ncclResult_t r1 = ncclGroupEnd();
        if (st != RT_OK) return failed(st);
        if (r1 != ncclSuccess && r1 != ncclInProgress) return failed(nccl_fail(r1, "ncclGroupEnd"));
        for (int i = 0; i < n && st == RT_OK; ++i) st = comm_wait(comms[i], "ncclGather");
        if (st != RT_OK) return failed(st);
    }
    for (int i = 0; i < n; ++i) {  // 3. rank 0 assembles; the others close their events
        DeviceGuard g(comms[i]->device);
        st = assemble_part(comms[i], cams, outputs, f[i], dst);
        if (st != RT_OK) return failed(st);
    }
    return RT_OK;
}

rt_status rt_comm_timing(rt_comm* c, rt_gather_timing* out, int reset) {
    if (!c) return fail(RT_ERR_INVALID_ARG, "comm is NULL");
    DeviceGuard g(c->device);
    rt_status st = harvest(c, true);
    if (st != RT_OK) return st;
    if (out) {
        out->render_ms = c->render_ms;
        out->gather_ms = c->gather_ms;
        out->assemble_ms = c->assemble_ms;
        out->frames = c->frames;
        out->rows = c->rows;
        out->max_rows = c->max_rows;
    }
    if (reset) {
        c->render_ms = c->gather_ms = c->assemble_ms = 0;
        c->frames = 0;
    }
    return RT_OK;
}

rt_status rt_debug_assemble_rows(rt_context* ctx, const void* gathered, size_t row_bytes,
                                 uint32_t height, uint32_t block, uint32_t n, uint32_t max_rows,
                                 void* image) {
    if (!ctx || !gathered || !image || n < 1 || block < 1)
        return fail(RT_ERR_INVALID_ARG, "bad argument to rt_debug_assemble_rows");
    DeviceGuard g(ctx->device);
    const size_t in_bytes = size_t(n) * max_rows * row_bytes, out_bytes = size_t(height) * row_bytes;
    RT_HIP(ctx->dbg.ensure(in_bytes + out_bytes + 16));
    char* d_in = static_cast<char*>(ctx->dbg.ptr);
    // the image at an offset that keeps the 16-B path when row_bytes allows it
    char* d_out = d_in + ((in_bytes + 15) & ~size_t(15));
    RT_HIP(hipMemcpyAsync(d_in, gathered, in_bytes, hipMemcpyHostToDevice, ctx->stream));
    RT_HIP(launch_assemble_rows(d_in, d_out, row_bytes, height, block, n, max_rows, 1,
                                ctx->stream));
    RT_HIP(hipMemcpyAsync(image, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

rt_status rt_comm_set_root_weight(rt_comm* c, int weight) {
    if (!c) return fail(RT_ERR_INVALID_ARG, "comm is NULL");
    if (weight < 1 || weight > 64)
        return fail(RT_ERR_INVALID_ARG, "root weight must be in [1, 64]");
    if (weight > 1 && c->nranks + weight - 1 > 65535)
        return fail(RT_ERR_INVALID_ARG, "too many row sets");
    rt_status st = comm_usable(c, "rt_comm_set_root_weight");
    if (st != RT_OK) return st;
    DeviceGuard g(c->device);
    if (c->any_frame && weight != c->root_weight) {
        // frames in flight were planned with the old weight: wait for them
        st = rt_comm_synchronize(c);
        if (st != RT_OK) return st;
    }
    if (c->nccl && c->nonblocking && c->nranks > 1) {
        // Only rt_comm_create communicators (one process per GPU, non-blocking init) agree here:
        // rt_comm_create_all / create_local ranks are driven serially from one thread, so an
        // all-reduce enqueued on one of them alone would never complete; their weights are
        // checked on the host by rt_render_gather_all_batch instead.
        // Collective on a communicator of one process per GPU: every rank must plan the same
        // split (a peer sizing its send from another weight than rank 0's receive would read
        // past buffers or pair ncclSend with ncclGather and hang), so the ranks agree on it
        // first — one all-reduce (max of {w, -w}) — and every rank fails alike if they differ.
        RT_HIP(c->chk.ensure(2 * sizeof(int32_t)));
        const int32_t v[2] = {weight, -weight};
        RT_HIP(hipMemcpyAsync(c->chk.ptr, v, sizeof v, hipMemcpyHostToDevice, c->ctx->stream));
        RT_NCCL(ncclAllReduce(c->chk.ptr, c->chk.ptr, 2, ncclInt32, ncclMax, c->nccl,
                              c->ctx->stream));
        st = comm_wait(c, "ncclAllReduce");
        if (st != RT_OK) return st;
        int32_t m[2] = {0, 0};
        RT_HIP(hipMemcpyAsync(m, c->chk.ptr, sizeof m, hipMemcpyDeviceToHost, c->ctx->stream));
        st = rt_comm_synchronize(c);
        if (st != RT_OK) return st;
        if (m[0] != weight || -m[1] != weight)
            return fail(RT_ERR_INVALID_ARG, "rt_comm_set_root_weight: the ranks asked for "
                                            "different weights (" + std::to_string(-m[1]) + ".." +
                                            std::to_string(m[0]) + "); the weight is unchanged");
    }
    c->root_weight = weight;
    return RT_OK;
}

rt_status rt_comm_info(const rt_comm* c, int* nranks, int* rank) {
    if (!c) return fail(RT_ERR_INVALID_ARG, "comm is NULL");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return RT_OK;
}

}  // extern "C"
