// rt_capi.cpp — implementation of include/rt_capi.h on HIP (gfx950).
//
// The context owns a device, a stream and growable device staging buffers; a scene is one
// HBM allocation of packed records (rt_internal.hpp).  No exception crosses the C boundary.
#include "rt_capi.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "rt_context.hpp"
#include "rt_internal.hpp"
#include "rt_wavefront.hpp"

#pragma clang fp contract(off)

using namespace rtamd;

namespace rtamd {

thread_local std::string g_last_error;

rt_status fail(rt_status st, const std::string& msg) {
    g_last_error = msg;
    return st;
}

rt_status hip_fail(hipError_t e, const char* what) {
    return fail(e == hipErrorOutOfMemory ? RT_ERR_OOM : RT_ERR_HIP,
                std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace rtamd

namespace rtamd {

// Rows a render call produces: [row_begin, row_end), or with row_cycle > 1 the row_block-row
// blocks starting at row_begin + k*row_cycle*row_block inside it (rt_render_opts).
uint32_t rendered_rows(const rt_render_opts& o, uint32_t height) {
    const uint32_t r1 = o.row_end ? std::min(o.row_end, height) : height;
    if (r1 <= o.row_begin) return 0;
    if (o.row_cycle <= 1 || o.row_block == 0) return r1 - o.row_begin;
    const uint64_t stride = static_cast<uint64_t>(o.row_block) * o.row_cycle;
    uint64_t rows = 0;
    for (uint64_t b = o.row_begin; b < r1; b += stride)
        rows += std::min<uint64_t>(o.row_block, r1 - b);
    return static_cast<uint32_t>(rows);
}

void pack_material(const rt_material& m, double* o) {
    o[0] = m.color[0];
    o[1] = m.color[1];
    o[2] = m.color[2];
    o[3] = m.shininess;
    o[4] = m.specular;
    o[5] = m.transparency;
    o[6] = m.refractive_index;
    o[7] = 0.0;
}

// Vec3::normalize (Math.h:31-37) on the host (used for the triangle normal, Shape.h:222-227).
void normalize3(const double* a, double* o) {
    const double len = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (len <= 1e-12) {
        o[0] = o[1] = o[2] = 0.0;
        return;
    }
    o[0] = a[0] / len;
    o[1] = a[1] / len;
    o[2] = a[2] / len;
}

rt_status harvest_events(rt_context* ctx, bool all) {
    size_t keep_from = 0;
    for (size_t i = 0; i < ctx->pending.size(); ++i) {
        auto& ev = ctx->pending[i];
        if (!all && hipEventQuery(ev.second) != hipSuccess) {
            keep_from = i;
            break;
        }
        RT_HIP(hipEventSynchronize(ev.second));
        float ms = 0.f;
        RT_HIP(hipEventElapsedTime(&ms, ev.first, ev.second));
        ctx->timed_ms += ms;
        ctx->launches += 1;
        ctx->free_events.push_back(ev);
        keep_from = i + 1;
    }
    ctx->pending.erase(ctx->pending.begin(), ctx->pending.begin() + keep_from);
    return RT_OK;
}

rt_status validate_camera(const rt_camera* cam) {
    if (!cam) return fail(RT_ERR_INVALID_ARG, "camera is NULL");
    if (cam->width == 0 || cam->height == 0)
        return fail(RT_ERR_INVALID_ARG, "camera width/height must be > 0");
    if (cam->aa_samples < 0) return fail(RT_ERR_INVALID_ARG, "aa_samples must be >= 0");
    if (static_cast<uint64_t>(cam->width) * cam->height > (1ull << 31))
        return fail(RT_ERR_UNSUPPORTED, "image larger than 2^31 pixels");
    return RT_OK;
}

rt_status build_params(rt_context* ctx, const rt_scene* sc, const rt_camera* cam,
                       const rt_render_opts* opts_in, TraceParams& p, int& path, bool& lds,
                       size_t& lds_bytes, uint32_t& rows) {
    if (!ctx) return fail(RT_ERR_INVALID_ARG, "context is NULL");
    if (!sc) return fail(RT_ERR_INVALID_ARG, "scene is NULL");
    if (sc->ctx != ctx) return fail(RT_ERR_INVALID_ARG, "scene belongs to another context");
    rt_status st = validate_camera(cam);
    if (st != RT_OK) return st;
    rt_render_opts opts;
    if (opts_in) opts = *opts_in;
    else rt_render_opts_default(&opts);
    const uint32_t r0 = opts.row_begin;
    const uint32_t r1 = opts.row_end ? opts.row_end : cam->height;
    if (r1 > cam->height || r0 >= r1)
        return fail(RT_ERR_INVALID_ARG, "row range [" + std::to_string(r0) + "," +
                                            std::to_string(r1) + ") invalid for height " +
                                            std::to_string(cam->height));
    if (opts.row_cycle > 1 && opts.row_block == 0)
        return fail(RT_ERR_INVALID_ARG, "row_cycle > 1 needs row_block >= 1");
    if (opts.tonemap < RT_TONEMAP_NONE || opts.tonemap >= RT_TONEMAP_COUNT)
        return fail(RT_ERR_INVALID_ARG, "tonemap operator out of range");
    rows = rendered_rows(opts, cam->height);

    const double* base = static_cast<const double*>(sc->buf.ptr);
    std::memset(&p, 0, sizeof p);
    p.sph = base + sc->off_sph;
    p.sph_mat = base + sc->off_sph_mat;
    p.pl = base + sc->off_pl;
    p.pl_mat = base + sc->off_pl_mat;
    p.tri = base + sc->off_tri;
    p.tri_mat = base + sc->off_tri_mat;
    if (sc->bvh_nodes > 0 && !(opts.flags & RT_FLAG_NO_BVH)) {
        p.bvh = base + sc->off_bvh;
        p.bvh_tri = reinterpret_cast<const int32_t*>(base + sc->off_bvh_tri);
    }
    p.lt = base + sc->off_lt;
    if (sc->np > 0) {
        p.box = base + sc->off_box;
        for (int k = 0; k < 4; ++k) p.box_n[k] = sc->box_n[k];
    }
    if (sc->ns >= kSphChunkMin) {
        p.sph_bnd = base + sc->off_sbnd;
        p.sph_perm = reinterpret_cast<const int32_t*>(base + sc->off_sperm);
    }
    p.ns = sc->ns;
    p.np = sc->np;
    p.nt = sc->nt;
    p.nl = sc->nl;
    if (sc->has_area && sc->area.samples > 0) {
        const rt_area_light& a = sc->area;
        const int k = static_cast<int>(std::lround(std::sqrt(static_cast<double>(a.samples))));
        if (k * k != a.samples)
            return fail(RT_ERR_INVALID_ARG, "area light samples must be a perfect square");
        const double li = a.intensity / static_cast<double>(a.samples);
        for (int i = 0; i < 3; ++i) {
            p.al_corner[i] = a.corner[i];
            p.al_u[i] = a.edge_u[i];
            p.al_v[i] = a.edge_v[i];
            p.al_E[i] = a.color[i] * li;
        }
        p.al_samples = a.samples;
        p.al_k = k;
    }
    for (int i = 0; i < 3; ++i) p.cam_pos[i] = cam->position[i];
    p.focal = cam->focal;
    p.width = cam->width;
    p.height = cam->height;
    p.aa = cam->aa_samples;
    p.max_rec = opts.max_recursion;
    p.bias = opts.bias;
    p.seed = opts.seed;
    p.row0 = r0;
    if (opts.row_cycle > 1) {
        p.row_block = opts.row_block;
        p.row_stride = static_cast<uint32_t>(opts.row_block) * opts.row_cycle;
    }
    p.rows = rows;
    p.tonemap = opts.tonemap;

    // Which TraceRay shape can this scene produce?  (Scene.h:175-195)
    if (sc->any_transparent) path = kPathTree;
    else if (!(sc->max_specular <= opts.bias) && opts.max_recursion >= 1) path = kPathChain;
    else path = kPathDirect;
    if (path != kPathDirect && opts.max_recursion > kMaxDepth)
        return fail(RT_ERR_UNSUPPORTED, "max_recursion > " + std::to_string(kMaxDepth) +
                                            " with reflective/transparent materials");
    lds_bytes = sizeof(double) * (static_cast<size_t>(kSphStride) * sc->ns +
                                  static_cast<size_t>(kPlStride) * sc->np +
                                  static_cast<size_t>(kLtStride) * sc->nl);
    lds = lds_bytes <= ctx->lds_limit;
    return RT_OK;
}

// The packet kernel's LDS image for this scene and camera (p.pk_image): looked up by camera
// position and formed by one setup launch the SECOND time a camera is rendered, then copied by
// every workgroup instead of being recomputed per workgroup.  A camera seen once (a moving
// camera) takes the in-kernel prologue and costs no setup launch; the last kMaxPkSeen such
// positions are remembered.  Past kMaxPkImages cached cameras the kernel forms it in LDS.
constexpr size_t kMaxPkImages = 16;
constexpr size_t kMaxPkSeen = 16;
// Launch shapes (grid, row set) with their own costliest-first tile order per cached camera.
constexpr size_t kMaxTileOrders = 8;
// A camera without a cached image gets a publish slot instead: the launch's first workgroup
// forms the image and hands it to the later ones through {epoch, word} granules (rt_packet.hip).
// Slots rotate so that launches in flight on other streams keep theirs; a slot overwritten by a
// later launch only fails its tags (the workgroup then forms the image itself).  Images above
// kPkPubMaxWords 32-bit words (4 KiB, about 32 spheres) are formed per workgroup: reading twice
// their size in granules costs as much as forming them (moving camera, MI355X: C2's 1.9 KiB
// image 54.1 -> 50.8 us; C3's 14.3 KiB 555 -> 555 us; C5's 6.5 KiB 522 -> 530 us).
constexpr size_t kPkPubSlots = 32;
constexpr size_t kPkPubMaxWords = 1024;
// Epochs are unique across the process (not per scene): a slot whose memory held another
// scene's granules (a freed and re-allocated buffer) can never match a later launch's tags.
std::atomic<uint32_t> g_pk_epoch{0};
rt_status packet_publish_slot(rt_context* ctx, const rt_scene* sc, TraceParams& p) {
    const size_t words = packet_lds_bytes(p.ns, p.np, p.nl) / 4;
    static const bool off = [] {  // RTAMD_PK_PUB=0: every workgroup forms it (A/B runs)
        const char* e = std::getenv("RTAMD_PK_PUB");
        return e && std::atoi(e) == 0;
    }();
    if (off || words > kPkPubMaxWords) return RT_OK;
    const size_t slot = kPkPubMaxWords * sizeof(unsigned long long);
    if (!sc->pk_pub.ptr) {
        // zeroed (epoch 0 is never used) and complete before any stream's launch reads it
        RT_HIP(sc->pk_pub.ensure(kPkPubSlots * slot));
        RT_HIP(hipMemsetAsync(sc->pk_pub.ptr, 0, kPkPubSlots * slot, ctx->stream));
        RT_HIP(hipStreamSynchronize(ctx->stream));
    }
    uint32_t ep = ++g_pk_epoch;
    if (ep == 0) ep = ++g_pk_epoch;
    p.pk_epoch = ep;
    // the first resident round: 256 CUs x 10 workgroups of 128 threads (20 waves per CU)
    static const long first_env = [] {
        const char* e = std::getenv("RTAMD_PK_PUB_FIRST");
        return e ? std::atol(e) : -1L;
    }();
    int cus = 0;
    RT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    p.pk_pub_first = first_env >= 0 ? static_cast<uint32_t>(first_env)
                                    : static_cast<uint32_t>(cus > 0 ? cus : 256) * 10u;
    p.pk_pub = reinterpret_cast<unsigned long long*>(static_cast<char*>(sc->pk_pub.ptr) +
                                                     (ep % kPkPubSlots) * slot);
    return RT_OK;
}
// Costliest tiles first (rt_packet.hip packet_order_kernel): the launch that creates a camera's
// packet image also records every wave's duration; the next launch of the same shape sorts the
// tiles by them (one small kernel, once) and every later one dispatches the costliest tiles
// first, so the cheapest fill the partly idle end of the launch.  The order only permutes which
// workgroup renders which tile: every pixel is computed by the same instructions, so images do
// not change (RT_FLAG_NO_TILE_ORDER: the default order, for A/B runs and the tests).  `*rec`
// receives the entry whose recording launch enqueue_render marks complete.
// existing_only: use an order already built for this shape, never record or build one (frame
// batches with several cameras: their launch neither pays the recording nor waits on a build).
rt_status tile_order(rt_context* ctx, rt_scene::PkImage& im, TraceParams& p, int flags,
                     rt_scene::PkImage::TileOrder** rec, bool existing_only = false) {
    *rec = nullptr;
    if (flags & RT_FLAG_NO_TILE_ORDER) return RT_OK;
    uint32_t gx, gy, waves;
    packet_grid(p, gx, gy, waves);
    const uint32_t key[8] = {gx, gy, waves, p.width, p.height, p.rows, p.row0,
                             (p.row_block << 16) ^ p.row_stride};
    const uint32_t tiles = gx * gy;
    size_t idx = 0;
    while (idx < im.ords.size() && std::memcmp(im.ords[idx].key, key, sizeof key) != 0) ++idx;
    if (existing_only && (idx == im.ords.size() || im.ords[idx].state != 2)) return RT_OK;
    if (idx == im.ords.size()) {  // a new launch shape: record this launch
        if (im.ords.size() >= kMaxTileOrders) return RT_OK;  // the default order
        if (im.ords.capacity() < kMaxTileOrders) im.ords.reserve(kMaxTileOrders);
        im.ords.emplace_back();
        auto& o = im.ords.back();
        im.last_ord = static_cast<int>(idx);
        hipError_t e = o.cost.ensure(sizeof(uint32_t) * tiles * waves);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&o.recorded, hipEventDisableTiming);
        if (e != hipSuccess) {
            o.cost.release();
            im.ords.pop_back();
            im.last_ord = -1;
            return hip_fail(e, "tile order");
        }
        std::memcpy(o.key, key, sizeof key);
        o.state = 1;
        p.tile_cost = static_cast<uint32_t*>(o.cost.ptr);
        *rec = &o;
        return RT_OK;
    }
    auto& o = im.ords[idx];
    im.last_ord = static_cast<int>(idx);
    if (o.state == 1) {  // build the order (after the recording launch, on whatever stream)
        RT_HIP(o.keys.ensure(sizeof(uint32_t) * tiles));
        RT_HIP(o.order.ensure(sizeof(uint32_t) * tiles));
        if (!o.built) RT_HIP(hipEventCreateWithFlags(&o.built, hipEventDisableTiming));
        if (!o.verdict) RT_HIP(hipHostMalloc(reinterpret_cast<void**>(&o.verdict), sizeof(uint32_t)));
        __atomic_store_n(o.verdict, 0u, __ATOMIC_RELAXED);
        RT_HIP(hipStreamWaitEvent(ctx->stream, o.recorded, 0));
        RT_HIP(launch_packet_order(static_cast<const uint32_t*>(o.cost.ptr), gx, gy, waves,
                                   static_cast<uint32_t*>(o.keys.ptr),
                                   static_cast<uint32_t*>(o.order.ptr), o.verdict, ctx->stream));
        RT_HIP(hipEventRecord(o.built, ctx->stream));
        o.state = 2;
    } else {
        // a narrow cost distribution keeps the default order: no table at all (the verdict is
        // only ever read as "narrow" once the order kernel has written it)
        if (__atomic_load_n(o.verdict, __ATOMIC_RELAXED) == 1u) return RT_OK;
        RT_HIP(hipStreamWaitEvent(ctx->stream, o.built, 0));  // built on another stream
    }
    p.tile_order = static_cast<const uint32_t*>(o.order.ptr);
    return RT_OK;
}

// A launch whose camera has no image entry yet (a moving camera): an order built earlier for the
// same launch shape under another camera of the scene, if any — an order only permutes which
// workgroup renders which tile, and nearby cameras share their costly tiles.
rt_status scene_tile_order(rt_context* ctx, const rt_scene* sc, TraceParams& p, int flags,
                           rt_scene::PkImage::TileOrder** rec) {
    for (auto& im : sc->pk_images) {
        const rt_status st = tile_order(ctx, im, p, flags, rec, true);
        if (st != RT_OK || p.tile_order) return st;
    }
    return RT_OK;
}

// The cached image of this camera position, or null; a render on another stream than the one
// that formed it waits for the entry's event until it has completed.
rt_status packet_image_cached(rt_context* ctx, const rt_scene* sc, const double* cam,
                              rt_scene::PkImage** out) {
    *out = nullptr;
    for (auto& im : sc->pk_images) {
        if (std::memcmp(im.cam, cam, sizeof im.cam) != 0) continue;
        if (!im.done && im.stream != ctx->stream) {
            const hipError_t q = hipEventQuery(im.ready);
            if (q == hipSuccess) im.done = true;
            else if (q == hipErrorNotReady) RT_HIP(hipStreamWaitEvent(ctx->stream, im.ready, 0));
            else return hip_fail(q, "hipEventQuery");
        }
        *out = &im;
        return RT_OK;
    }
    return RT_OK;
}

// A camera without a cached image: true when it was seen before (the last kMaxPkSeen first
// sightings) and the cache has room, i.e. it should get a cache entry now (removed from the seen
// list); otherwise it is remembered as seen once.
bool packet_second_sighting(const rt_scene* sc, const double* cam) {
    auto& seen = sc->pk_seen;
    auto it = std::find_if(seen.begin(), seen.end(), [&](const std::array<double, 3>& c) {
        return std::memcmp(c.data(), cam, 3 * sizeof(double)) == 0;
    });
    if (it == seen.end()) {
        if (seen.size() >= kMaxPkSeen) seen.erase(seen.begin());
        seen.push_back({cam[0], cam[1], cam[2]});
        return false;
    }
    if (sc->pk_images.size() >= kMaxPkImages) return false;
    seen.erase(it);
    return true;
}

// A new cache entry for this camera (its buffer allocated, its event created; the caller
// enqueues the launch that forms the image and records `ready` after it on ctx->stream).
rt_status packet_image_entry(rt_context* ctx, const rt_scene* sc, const double* cam,
                             const TraceParams& p, rt_scene::PkImage** out) {
    *out = nullptr;
    // never reallocated: a frame batch holds entries of earlier frames while adding one
    if (sc->pk_images.capacity() < kMaxPkImages) sc->pk_images.reserve(kMaxPkImages);
    sc->pk_images.emplace_back();
    rt_scene::PkImage& im = sc->pk_images.back();
    std::memcpy(im.cam, cam, sizeof im.cam);
    im.stream = ctx->stream;
    hipError_t e = im.buf.ensure(packet_lds_bytes(p.ns, p.np, p.nl));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&im.ready, hipEventDisableTiming);
    if (e != hipSuccess) {
        im.buf.release();
        if (im.ready) (void)hipEventDestroy(im.ready);
        sc->pk_images.pop_back();
        return hip_fail(e, "packet image entry");
    }
    *out = &im;
    return RT_OK;
}

// One-frame launches: the cached image; on a camera's second sighting a one-workgroup setup
// launch forms its cache entry; on a first sighting a publish slot.
rt_status packet_image(rt_context* ctx, const rt_scene* sc, TraceParams& p, int flags,
                       rt_scene::PkImage::TileOrder** rec) {
    *rec = nullptr;
    rt_scene::PkImage* found = nullptr;
    rt_status st = packet_image_cached(ctx, sc, p.cam_pos, &found);
    if (st != RT_OK) return st;
    if (found) {
        p.pk_image = static_cast<const double*>(found->buf.ptr);
        return tile_order(ctx, *found, p, flags, rec);
    }
    if (!packet_second_sighting(sc, p.cam_pos)) {
        const rt_status st2 = packet_publish_slot(ctx, sc, p);
        return st2 != RT_OK ? st2 : scene_tile_order(ctx, sc, p, flags, rec);
    }
    rt_scene::PkImage* im = nullptr;
    st = packet_image_entry(ctx, sc, p.cam_pos, p, &im);
    if (st != RT_OK) return st;
    hipError_t e = launch_packet_image(p, static_cast<double*>(im->buf.ptr), ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(im->ready, ctx->stream);
    if (e != hipSuccess) {
        im->buf.release();
        (void)hipEventDestroy(im->ready);
        sc->pk_images.pop_back();
        return hip_fail(e, "packet image setup");
    }
    p.pk_image = static_cast<const double*>(im->buf.ptr);
    return tile_order(ctx, *im, p, flags, rec);
}

// A frame batch's image sources (p.fr[f].img for every frame, before the batch launch): a
// cached image, or one formed by ONE small launch for every frame that has none — into a new
// cache entry when the camera was seen before (so a revisited position costs no launch of its
// own), else into the batch's ring slot (an entry of kPkBatchRing, reused once the launches that
// read it have completed).  Frames with the camera of an earlier frame of the batch share its
// image.  The tile order: frame 0's, recorded / built only when every frame has frame 0's
// camera (a static camera), otherwise only an order built earlier for the shape.
rt_status packet_batch_images(rt_context* ctx, const rt_scene* sc, const rt_camera* cams,
                              int nframes, TraceParams& p, int flags,
                              rt_scene::PkImage::TileOrder** rec, int* batch_ring) {
    *rec = nullptr;
    *batch_ring = -1;
    enum Kind { kCached, kPromote, kRing, kDup };
    Kind kind[kPkMaxBatch];
    int dup_of[kPkMaxBatch];
    rt_scene::PkImage* ent[kPkMaxBatch] = {};
    bool same_cam = true;
    bool any_ring = false;
    const size_t cache_before = sc->pk_images.size();
    // Every error exit after the first promotion drops the entries this call created (newest
    // last): an entry that never received its image, with a `ready` event never recorded, would
    // be taken as a formed image by every later render from that camera position.
    struct Rollback {
        const rt_scene* sc;
        size_t keep;
        bool armed = true;
        ~Rollback() {
            if (!armed) return;
            while (sc->pk_images.size() > keep) {
                auto& im = sc->pk_images.back();
                im.buf.release();
                if (im.ready) (void)hipEventDestroy(im.ready);
                sc->pk_images.pop_back();
            }
        }
    } rollback{sc, cache_before};
    for (int f = 0; f < nframes; ++f) {
        PkFrame& F = p.fr[f];
        for (int i = 0; i < 3; ++i) F.cam[i] = cams[f].position[i];
        F.img = nullptr;
        F.pub = nullptr;
        F.epoch = 0;
        F._pad = 0;
        if (std::memcmp(F.cam, p.fr[0].cam, sizeof F.cam) != 0) same_cam = false;
        int g = 0;
        while (g < f && std::memcmp(p.fr[g].cam, F.cam, sizeof F.cam) != 0) ++g;
        if (g < f) {
            kind[f] = kDup;
            dup_of[f] = g;
            continue;
        }
        rt_status st = packet_image_cached(ctx, sc, F.cam, &ent[f]);
        if (st != RT_OK) return st;
        if (ent[f]) {
            kind[f] = kCached;
            F.img = static_cast<const double*>(ent[f]->buf.ptr);
            continue;
        }
        if (packet_second_sighting(sc, F.cam)) {
            st = packet_image_entry(ctx, sc, F.cam, p, &ent[f]);
            if (st != RT_OK) return st;
            kind[f] = kPromote;
            F.img = static_cast<const double*>(ent[f]->buf.ptr);
            continue;
        }
        kind[f] = kRing;
        any_ring = true;
    }
    const size_t img_doubles = ((packet_lds_bytes(p.ns, p.np, p.nl) + 255) & ~size_t(255)) /
                               sizeof(double);
    double* ring = nullptr;
    if (any_ring) {
        const size_t entry = img_doubles * sizeof(double) * kPkMaxBatch;
        RT_HIP(sc->pk_batch.ensure(entry * rt_scene::kPkBatchRing));
        const int r = sc->pk_batch_next;
        sc->pk_batch_next = (r + 1) % rt_scene::kPkBatchRing;
        if (!sc->pk_batch_done[r])
            RT_HIP(hipEventCreateWithFlags(&sc->pk_batch_done[r], hipEventDisableTiming));
        if (sc->pk_batch_used[r])  // the batch that last read this entry, on any stream
            RT_HIP(hipStreamWaitEvent(ctx->stream, sc->pk_batch_done[r], 0));
        ring = reinterpret_cast<double*>(static_cast<char*>(sc->pk_batch.ptr) +
                                         static_cast<size_t>(r) * entry);
        *batch_ring = r;
    }
    PkImageJobs jobs;
    std::memset(&jobs, 0, sizeof jobs);
    for (int f = 0; f < nframes; ++f) {
        PkFrame& F = p.fr[f];
        if (kind[f] == kRing) F.img = ring + static_cast<size_t>(f) * img_doubles;
        if (kind[f] == kDup) F.img = p.fr[dup_of[f]].img;
        if (kind[f] == kRing || kind[f] == kPromote) {
            jobs.dst[jobs.n] = const_cast<double*>(F.img);
            jobs.frame[jobs.n] = f;
            ++jobs.n;
        }
    }
    hipError_t e = launch_packet_image_batch(p, jobs, ctx->stream);
    for (int f = 0; f < nframes && e == hipSuccess; ++f)
        if (kind[f] == kPromote) e = hipEventRecord(ent[f]->ready, ctx->stream);
    if (e != hipSuccess) return hip_fail(e, "packet batch images");  // the rollback drops them
    rollback.armed = false;  // every promoted entry now has its image and its recorded event
    if (kind[0] == kCached) return tile_order(ctx, *ent[0], p, flags, rec, !same_cam);
    return scene_tile_order(ctx, sc, p, flags, rec);
}

// Whether a render of this TraceRay shape takes the breadth-first path, whose arena (ctx->wf,
// ctx->wf_ctl) is one per context: refraction trees, and reflection chains when
// RTAMD_WF_CHAIN=1 forces them there.
bool uses_wavefront_arena(int path, int flags) {
    if (flags & RT_FLAG_GENERIC_KERNEL) return false;
    const char* wf_chain = std::getenv("RTAMD_WF_CHAIN");
    return path == kPathTree || (path == kPathChain && wf_chain && std::atoi(wf_chain) == 1);
}

rt_status scratch_wait(rt_context* ctx) {
    // the latest user on this same stream is ordered before us already
    if (ctx->scratch_used && ctx->scratch_stream != ctx->stream)
        RT_HIP(hipStreamWaitEvent(ctx->stream, ctx->scratch_event, 0));
    return RT_OK;
}

rt_status scratch_done(rt_context* ctx) {
    RT_HIP(hipEventRecord(ctx->scratch_event, ctx->stream));
    ctx->scratch_used = true;
    ctx->scratch_stream = ctx->stream;
    return RT_OK;
}

// The packet kernel's fix-up buffers for a launch of `px` output pixels (rt_internal.hpp
// TraceParams.fix_list): the list grows on demand; the two counts are zeroed once, then each
// fix-up launch zeroes the one the next launch uses (ctx->fix_parity alternates).
rt_status fixup_buffers(rt_context* ctx, size_t px, TraceParams& p) {
    if (px >= (size_t(1) << 32)) return fail(RT_ERR_UNSUPPORTED, "fix-up list above 2^32 pixels");
    if (!ctx->fix_ctl.ptr) {
        RT_HIP(ctx->fix_ctl.ensure(2 * sizeof(uint32_t)));
        RT_HIP(hipMemsetAsync(ctx->fix_ctl.ptr, 0, 2 * sizeof(uint32_t), ctx->stream));
    }
    if (ctx->fix_list.bytes < px * sizeof(uint32_t)) {
        // the list may still be read by a fix-up launch on any stream the context used; every
        // user of the list is a scratch user, so the context's last scratch event covers them
        // all (not hipDeviceSynchronize: it would also wait on an RCCL gather of a dead peer
        // and on other contexts' work)
        if (ctx->scratch_used) RT_HIP(hipEventSynchronize(ctx->scratch_event));
        RT_HIP(ctx->fix_list.ensure(px * sizeof(uint32_t)));
    }
    p.fix_list = static_cast<uint32_t*>(ctx->fix_list.ptr);
    p.fix_ctl = static_cast<uint32_t*>(ctx->fix_ctl.ptr) + ctx->fix_parity;
    p.fix_next = static_cast<uint32_t*>(ctx->fix_ctl.ptr) + (1 - ctx->fix_parity);
    return RT_OK;
}

rt_status check_batch(const rt_camera* cams, int nframes) {
    if (!cams || nframes < 1) return fail(RT_ERR_INVALID_ARG, "frame batch: no cameras");
    for (int f = 0; f < nframes; ++f) {
        rt_status st = validate_camera(cams + f);
        if (st != RT_OK) return st;
        if (cams[f].width != cams[0].width || cams[f].height != cams[0].height ||
            cams[f].aa_samples != cams[0].aa_samples ||
            std::memcmp(&cams[f].focal, &cams[0].focal, sizeof(double)) != 0)
            return fail(RT_ERR_INVALID_ARG, "frame batch: every camera must have the first's "
                                            "width, height, focal and aa_samples");
    }
    return RT_OK;
}

rt_status enqueue_render(rt_context* ctx, const rt_scene* sc, const rt_camera* cam,
                         const rt_render_opts* opts, double* d64, float* d32, uint8_t* dldr) {
    return enqueue_frames(ctx, sc, cam, 1, opts, d64, d32, dldr);
}

rt_status enqueue_frames(rt_context* ctx, const rt_scene* sc, const rt_camera* cams, int nframes,
                         const rt_render_opts* opts, double* d64, float* d32, uint8_t* dldr,
                         uint32_t frame_rows) {
    TraceParams p;
    int path;
    bool lds;
    size_t lds_bytes;
    uint32_t rows;
    rt_status st = nframes == 1 ? RT_OK : check_batch(cams, nframes);
    if (st != RT_OK) return st;
    st = build_params(ctx, sc, cams, opts, p, path, lds, lds_bytes, rows);
    if (st != RT_OK) return st;
    p.out64 = d64;
    p.out32 = d32;
    p.ldr = dldr;
    const int flags = opts ? opts->flags : 0;
    if (!dldr) p.tonemap = RT_TONEMAP_NONE;
    if (dldr && p.tonemap == RT_TONEMAP_NONE) p.ldr = nullptr;
    const bool packet_path = path == kPathDirect && !(flags & RT_FLAG_GENERIC_KERNEL) &&
                             p.ns <= packet_max_spheres() &&
                             packet_lds_bytes(p.ns, p.np, p.nl) <= ctx->lds_limit;
    if (frame_rows && frame_rows < rows)
        return fail(RT_ERR_INVALID_ARG, "frame batch: frame stride below the rendered rows");
    const size_t frame_px = static_cast<size_t>(frame_rows ? frame_rows : rows) * p.width;
    if (nframes > 1 && (!packet_path || nframes > kPkMaxBatch)) {
        // one launch per frame (other kernels), or per kPkMaxBatch frames
        const int step = packet_path ? kPkMaxBatch : 1;
        for (int f0 = 0; f0 < nframes; f0 += step) {
            const size_t off = 3 * frame_px * static_cast<size_t>(f0);
            st = enqueue_frames(ctx, sc, cams + f0, std::min(step, nframes - f0), opts,
                                d64 ? d64 + off : nullptr, d32 ? d32 + off : nullptr,
                                dldr ? dldr + off : nullptr, frame_rows);
            if (st != RT_OK) return st;
        }
        return RT_OK;
    }
    bool scratch = (flags & RT_FLAG_COUNT_RAYS) || uses_wavefront_arena(path, flags);

    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (flags & RT_FLAG_TIME_KERNEL) {
        if (ctx->pending.size() >= 1024) {
            st = harvest_events(ctx, false);
            if (st != RT_OK) return st;
        }
        if (!ctx->free_events.empty()) {
            ev = ctx->free_events.back();
            ctx->free_events.pop_back();
        } else {
            RT_HIP(hipEventCreate(&ev.first));
            RT_HIP(hipEventCreate(&ev.second));
        }
        RT_HIP(hipEventRecord(ev.first, ctx->stream));
    }
    // Scenes without secondary rays take the packet-culled kernel when its LDS image fits.
    const bool packet = packet_path;
    rt_scene::PkImage::TileOrder* rec = nullptr;  // set: this launch records wave durations
    int batch_ring = -1;  // the ring entry of this batch's formed images, if any
    if (packet && nframes > 1) {
        // a frame batch: frame f's camera and image source, all formed before the launch by at
        // most one small launch (packet_batch_images)
        p.nframes = static_cast<uint32_t>(nframes);
        p.frame_px = frame_px;
        st = packet_batch_images(ctx, sc, cams, nframes, p, flags, &rec, &batch_ring);
        if (st != RT_OK) return st;
    } else if (packet) {
        st = packet_image(ctx, sc, p, flags, &rec);
        if (st != RT_OK) return st;
    }
    // the fix-up variant of the packet kernel (undecided shadow rays re-rendered per pixel after
    // the launch) uses the context's fix-up list: ordered across streams like the counters
    const bool fixup = packet && packet_uses_fixup(p, false, sc->max_specular > 0.0);
    if (fixup) {
        st = fixup_buffers(ctx, nframes > 1 ? static_cast<size_t>(nframes) * frame_px
                                             : static_cast<size_t>(rows) * p.width, p);
        if (st != RT_OK) return st;
        scratch = true;
    }
    if (scratch) {
        st = scratch_wait(ctx);
        if (st != RT_OK) return st;
    }
    // generic kernels without triangle / area-light code for scenes that use neither
    const bool lean_generic = p.nt == 0 && p.al_samples == 0;
    // reflection chains of scenes made of planes (and up to kBoxMaxSpheres spheres) take the
    // scalar-cache chain kernel (rt_box.hip); RTAMD_BOX_SPH=0 keeps scenes with spheres on the
    // generic chain kernel (A/B runs)
    static const bool box_sph = [] {
        const char* e = std::getenv("RTAMD_BOX_SPH");
        return !(e && std::atoi(e) == 0);
    }();
    const bool box = path == kPathChain && p.nt == 0 && p.al_samples == 0 &&
                     (p.ns == 0 ? p.np > 0 : (box_sph && p.ns <= kBoxMaxSpheres)) &&
                     !(flags & RT_FLAG_GENERIC_KERNEL);
    const bool spar = !(flags & RT_FLAG_NO_SAMPLE_PARALLEL);
    auto launch = [&](const TraceParams& q, bool count) {
        if (box)
            return launch_box_chain(q, count, !(flags & RT_FLAG_NO_SAMPLE_PARALLEL), ctx->stream);
        return packet ? launch_packet_direct(q, count, sc->max_specular > 0.0, ctx->stream)
                      : (lean_generic ? lean::launch_trace(q, path, count, lds, lds_bytes, ctx->stream, spar)
                                      : launch_trace(q, path, count, lds, lds_bytes, ctx->stream, spar));
    };
    // Scenes with refraction trees take the breadth-first TraceRay when the roots fit the arena
    // budget (RTAMD_WF_MB, default 4096 MiB); trees that overflow it are re-rendered per pixel.
    // Reflection chains stay per pixel: measured 2-3x faster there (coherent, no stack), while
    // the glass tree renders 4.6x faster breadth-first.  RTAMD_WF_CHAIN=1 forces chains too.
    bool wavefront = false;
    if (uses_wavefront_arena(path, flags)) {
        const size_t n0 = static_cast<size_t>(rows) * p.width *
                          static_cast<size_t>(p.aa > 0 ? p.aa : 0);
        const char* env = std::getenv("RTAMD_WF_MB");
        const size_t budget = (env && std::atoll(env) > 0 ? static_cast<size_t>(std::atoll(env))
                                                          : size_t(4096)) << 20;
        // the deferred-direct queue is laid out only when that pass runs (refraction trees)
        const bool defer = path == kPathTree && wf_defer_selected();
        const size_t root_bytes = wf_arena_bytes(n0, n0, defer);
        if (n0 < (size_t(1) << 30) && root_bytes <= budget) {
            // ~100 B per non-root node (+16 B of queue when deferred)
            size_t extra = (budget - root_bytes) / (defer ? 116 : 100);
            extra = std::min(extra, std::max<size_t>(n0, 1) * 64);
            extra = std::min(extra, (size_t(1) << 31) - 1 - n0);
            const size_t cap = n0 + extra;
            RT_HIP(ctx->wf.ensure(wf_arena_bytes(n0, cap, defer)));
            RT_HIP(ctx->wf_ctl.ensure(sizeof(WfCtl)));
            const WfArena A = wf_arena_layout(ctx->wf.ptr, n0, cap,
                                              static_cast<WfCtl*>(ctx->wf_ctl.ptr), defer);
            RT_HIP(lean_generic ? lean::launch_wavefront(p, path, A, lds, lds_bytes, ctx->stream)
                                : launch_wavefront(p, path, A, lds, lds_bytes, ctx->stream));
            wavefront = true;
        }
    }
    if (!wavefront) RT_HIP(launch(p, false));
    if (fixup) {
        const hipError_t fe = launch_packet_fixup(p, ctx->stream);
        if (fe != hipSuccess) {
            // the packet launch appended to the list and no fix-up launch zeroes the next count:
            // reset both, or a later fix-variant launch would append at a stale base past its list
            (void)hipMemsetAsync(ctx->fix_ctl.ptr, 0, 2 * sizeof(uint32_t), ctx->stream);
            return hip_fail(fe, "launch_packet_fixup");
        }
        ctx->fix_parity ^= 1;  // the next fix-variant launch appends to the count just zeroed
    }
    if (rec) RT_HIP(hipEventRecord(rec->recorded, ctx->stream));
    if (flags & RT_FLAG_TIME_KERNEL) {
        RT_HIP(hipEventRecord(ev.second, ctx->stream));
        ctx->pending.push_back(ev);
    }
    if (flags & RT_FLAG_COUNT_RAYS) {
        // Counting variant: same trace with wave-reduced atomics, outputs discarded.
        TraceParams pc = p;
        pc.out64 = nullptr;
        pc.out32 = nullptr;
        pc.ldr = nullptr;
        pc.counters = static_cast<unsigned long long*>(ctx->counters.ptr);
        pc.tile_cost = nullptr;  // the durations are the image launch's
        RT_HIP(launch(pc, true));
    }
    if (batch_ring >= 0) {  // the entry is free again once these launches have completed
        RT_HIP(hipEventRecord(sc->pk_batch_done[batch_ring], ctx->stream));
        sc->pk_batch_used[batch_ring] = true;
    }
    return scratch ? scratch_done(ctx) : RT_OK;
}

}  // namespace rtamd

extern "C" {

const char* rt_last_error(void) { return g_last_error.c_str(); }

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void rt_render_opts_default(rt_render_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof *o);
    o->max_recursion = 10;         // Scene.h:24
    o->tonemap = RT_TONEMAP_ACES;  // RaytracingEngine.cpp:301 tonemap()
    o->bias = 1e-3;                // Scene.h:291
    o->seed = 0x5EEDull;
}

rt_status rt_context_create(int device, rt_context** out) {
    if (!out) return fail(RT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n)
        return fail(RT_ERR_NO_DEVICE, "device " + std::to_string(device) + " not in [0," +
                                          std::to_string(n) + ")");
    hipDeviceProp_t prop;
    RT_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RT_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName +
                                          ", this build targets gfx950 only");
    DeviceGuard g(device);
    rt_context* ctx = new (std::nothrow) rt_context();
    if (!ctx) return fail(RT_ERR_OOM, "host allocation failed");
    ctx->device = device;
    // stay at <= 40 KiB of staged scene per 256-thread workgroup so >= 4 workgroups fit a CU
    ctx->lds_limit = 40 * 1024;
    hipError_t e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = ctx->counters.ensure(2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(ctx->counters.ptr, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->scratch_event, hipEventDisableTiming);
    if (e != hipSuccess) {
        rt_context_destroy(ctx);
        return hip_fail(e, "rt_context_create");
    }
    ctx->stream = ctx->own_stream;
    *out = ctx;
    return RT_OK;
}

rt_status rt_context_destroy(rt_context* ctx) {
    if (!ctx) return RT_OK;
    DeviceGuard g(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto* v : {&ctx->pending, &ctx->free_events})
        for (auto& ev : *v) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
    if (ctx->scratch_event) {
        (void)hipEventSynchronize(ctx->scratch_event);
        (void)hipEventDestroy(ctx->scratch_event);
    }
    leave_groups(ctx);  // communicators of any group this context is in go first
    for (DeviceBuffer* b : {&ctx->out64, &ctx->out32, &ctx->ldr, &ctx->tm_in, &ctx->tm_out,
                            &ctx->dbg, &ctx->rays, &ctx->counters, &ctx->wf, &ctx->wf_ctl,
                            &ctx->fix_list, &ctx->fix_ctl})
        b->release();
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return RT_OK;
}

rt_status rt_context_set_stream(rt_context* ctx, void* hip_stream) {
    if (!ctx) return fail(RT_ERR_INVALID_ARG, "context is NULL");
    ctx->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->own_stream;
    return RT_OK;
}

rt_status rt_context_synchronize(rt_context* ctx) {
    if (!ctx) return fail(RT_ERR_INVALID_ARG, "context is NULL");
    DeviceGuard g(ctx->device);
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

rt_status rt_scene_create(rt_context* ctx, const rt_scene_desc* d, rt_scene** out) {
    if (!ctx || !d || !out) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_scene_create");
    *out = nullptr;
    if (d->n_spheres < 0 || d->n_planes < 0 || d->n_triangles < 0 || d->n_lights < 0)
        return fail(RT_ERR_INVALID_ARG, "negative primitive count");
    if ((d->n_spheres && !d->spheres) || (d->n_planes && !d->planes) ||
        (d->n_triangles && !d->triangles) || (d->n_lights && !d->lights))
        return fail(RT_ERR_INVALID_ARG, "primitive count > 0 with NULL array");
    DeviceGuard g(ctx->device);

    rt_scene* sc = new (std::nothrow) rt_scene();
    if (!sc) return fail(RT_ERR_OOM, "host allocation failed");
    sc->ctx = ctx;
    sc->ns = d->n_spheres;
    sc->np = d->n_planes;
    sc->nt = d->n_triangles;
    sc->nl = d->n_lights;
    size_t off = 0;
    auto take = [&off](size_t n) {
        size_t o = off;
        off += (n + 1) & ~size_t(1);  // keep every array 16-byte aligned
        return o;
    };
    sc->off_sph = take(size_t(kSphStride) * sc->ns);
    sc->off_pl = take(size_t(kPlStride) * sc->np);
    sc->off_tri = take(size_t(kTriStride) * sc->nt);
    sc->off_lt = take(size_t(kLtStride) * sc->nl);
    // one material table [spheres | planes | triangles]: a hit's material is one integer
    // offset away (no pointer select, so global loads instead of flat ones)
    sc->off_sph_mat = take(size_t(kMatStride) * (size_t(sc->ns) + sc->np + sc->nt));
    sc->off_pl_mat = sc->off_sph_mat + size_t(kMatStride) * sc->ns;
    sc->off_tri_mat = sc->off_pl_mat + size_t(kMatStride) * sc->np;
    std::vector<double> h(off + 2, 0.0);

    bool transparent = false;
    double max_spec = 0.0;
    auto note = [&](const rt_material& m) {
        if (!(m.transparency <= 0.0)) transparent = true;
        if (std::isnan(m.specular)) max_spec = INFINITY;
        else if (m.specular > max_spec) max_spec = m.specular;
    };
    for (int i = 0; i < sc->ns; ++i) {
        const rt_sphere& s = d->spheres[i];
        double* o = &h[sc->off_sph + size_t(kSphStride) * i];
        o[0] = s.center[0];
        o[1] = s.center[1];
        o[2] = s.center[2];
        o[3] = s.radius * s.radius;  // Shape.h:77
        pack_material(s.material, &h[sc->off_sph_mat + size_t(kMatStride) * i]);
        note(s.material);
    }
    for (int i = 0; i < sc->np; ++i) {
        const rt_plane& pl = d->planes[i];
        double* o = &h[sc->off_pl + size_t(kPlStride) * i];
        for (int k = 0; k < 3; ++k) {
            o[k] = pl.point[k];
            o[3 + k] = pl.normal[k];
        }
        pack_material(pl.material, &h[sc->off_pl_mat + size_t(kMatStride) * i]);
        note(pl.material);
    }
    for (int i = 0; i < sc->nt; ++i) {
        const rt_triangle& t = d->triangles[i];
        double* o = &h[sc->off_tri + size_t(kTriStride) * i];
        double a0[3], a1[3], a2[3], e1u[3], e2u[3], n[3];
        for (int k = 0; k < 3; ++k) {
            a0[k] = t.v0[k] + t.translation[k];  // tv0() Shape.h:198
            a1[k] = t.v1[k] + t.translation[k];
            a2[k] = t.v2[k] + t.translation[k];
            e1u[k] = t.v1[k] - t.v0[k];          // untranslated edges for the normal
            e2u[k] = t.v2[k] - t.v0[k];
        }
        const double c[3] = {e1u[1] * e2u[2] - e1u[2] * e2u[1], e1u[2] * e2u[0] - e1u[0] * e2u[2],
                             e1u[0] * e2u[1] - e1u[1] * e2u[0]};
        normalize3(c, n);
        for (int k = 0; k < 3; ++k) {
            o[k] = a0[k];
            o[3 + k] = a1[k] - a0[k];  // edge1 = tv1() - a0
            o[6 + k] = a2[k] - a0[k];  // edge2 = tv2() - a0
            o[9 + k] = n[k];
        }
        pack_material(t.material, &h[sc->off_tri_mat + size_t(kMatStride) * i]);
        note(t.material);
    }
    for (int i = 0; i < sc->nl; ++i) {
        const rt_light& l = d->lights[i];
        double* o = &h[sc->off_lt + size_t(kLtStride) * i];
        for (int k = 0; k < 3; ++k) {
            o[k] = l.position[k];
            o[3 + k] = l.color[k] * l.intensity;  // Scene.h:110 emitted
        }
    }
    sc->any_transparent = transparent;
    sc->max_specular = max_spec;

    // triangle BVH (rt_bvh.cpp) appended to the same allocation: nodes, then the leaf-order
    // triangle ids packed two per double slot
    if (sc->nt >= kBvhMinTris) {
        std::vector<double> nodes;
        std::vector<int32_t> order;
        build_triangle_bvh(&h[sc->off_tri], sc->nt, nodes, order);
        sc->off_bvh = h.size();
        sc->off_bvh_tri = sc->off_bvh + nodes.size();
        h.resize(sc->off_bvh_tri + (order.size() + 1) / 2 + 2, 0.0);
        std::memcpy(&h[sc->off_bvh], nodes.data(), nodes.size() * sizeof(double));
        std::memcpy(&h[sc->off_bvh_tri], order.data(), order.size() * sizeof(int32_t));
        sc->bvh_nodes = static_cast<int32_t>(nodes.size() / kBvhNodeStride);
    }

    // spatial sphere chunks of the packet kernel's culls: permutation (packed two per double
    // slot) and one bounding sphere per chunk
    if (sc->ns >= kSphChunkMin) {
        std::vector<int32_t> perm;
        std::vector<double> bnd;
        build_sphere_chunks(&h[sc->off_sph], sc->ns, perm, bnd);
        sc->off_sbnd = (h.size() + 1) & ~size_t(1);
        sc->off_sperm = sc->off_sbnd + bnd.size();
        h.resize(sc->off_sperm + (perm.size() + 1) / 2 + 2, 0.0);
        std::memcpy(&h[sc->off_sbnd], bnd.data(), bnd.size() * sizeof(double));
        std::memcpy(&h[sc->off_sperm], perm.data(), perm.size() * sizeof(int32_t));
    }

    // planes-only chain table (rt_box.hip): the planes grouped by the axis of their normal —
    // exactly ±e_x, ±e_y, ±e_z (two zero components, the third ±1), then the rest — each group
    // in scene order, with the plane's material, a flag for normals whose normalize() returns
    // them unchanged (|n| rounds to 1: sqrt of the reference's dot, correctly rounded as on the
    // device) and the scene index for closest-hit ties
    if (sc->np > 0) {
        std::vector<int> grp(sc->np);
        for (int i = 0; i < sc->np; ++i) {
            const double* q = &h[sc->off_pl + size_t(kPlStride) * i];
            const double* n = q + 3;
            grp[i] = 3;
            const bool bounded = std::fabs(q[0]) <= 0x1p1000 && std::fabs(q[1]) <= 0x1p1000 &&
                                 std::fabs(q[2]) <= 0x1p1000;  // p − o stays finite (rt_box.hip)
            for (int k = 0; k < 3 && bounded; ++k)
                if (std::fabs(n[k]) == 1.0 && n[(k + 1) % 3] == 0.0 && n[(k + 2) % 3] == 0.0)
                    grp[i] = k;
        }
        sc->off_box = (h.size() + 1) & ~size_t(1);
        h.resize(sc->off_box + size_t(kBoxRec) * sc->np + 2, 0.0);
        size_t r = 0;
        for (int g = 0; g < 4; ++g) {
            for (int i = 0; i < sc->np; ++i) {
                if (grp[i] != g) continue;
                const double* pl = &h[sc->off_pl + size_t(kPlStride) * i];
                double* o = &h[sc->off_box + size_t(kBoxRec) * r++];
                for (int k = 0; k < 6; ++k) o[k] = pl[k];
                o[6] = g < 3 ? pl[g] : 0.0;
                const double nn = pl[3] * pl[3] + pl[4] * pl[4] + pl[5] * pl[5];
                o[7] = std::sqrt(nn) == 1.0 ? 1.0 : 0.0;
                for (int k = 0; k < kMatStride - 1; ++k)
                    o[8 + k] = h[sc->off_pl_mat + size_t(kMatStride) * i + k];
                const int32_t idx[2] = {i, 0};
                std::memcpy(&o[15], idx, sizeof idx);
                ++sc->box_n[g];
            }
        }
    }

    hipError_t e = sc->buf.ensure(h.size() * sizeof(double));
    if (e == hipSuccess)
        e = hipMemcpyAsync(sc->buf.ptr, h.data(), h.size() * sizeof(double),
                           hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        sc->buf.release();
        delete sc;
        return hip_fail(e, "rt_scene_create upload");
    }
    *out = sc;
    return RT_OK;
}

rt_status rt_scene_destroy(rt_scene* sc) {
    if (!sc) return RT_OK;
    DeviceGuard g(sc->ctx->device);
    // Launches that read the scene or its packet images may be in flight on any stream the
    // context used (rt_context_set_stream switches it; pipelined frames use several), not only
    // the current one: wait for the whole device before freeing.
    (void)hipDeviceSynchronize();
    sc->buf.release();
    sc->pk_pub.release();
    sc->pk_batch.release();
    for (auto& e : sc->pk_batch_done)
        if (e) (void)hipEventDestroy(e);
    for (auto& im : sc->pk_images) {
        im.buf.release();
        if (im.ready) (void)hipEventDestroy(im.ready);
        for (auto& o : im.ords) {
            o.cost.release();
            o.keys.release();
            o.order.release();
            if (o.recorded) (void)hipEventDestroy(o.recorded);
            if (o.built) (void)hipEventDestroy(o.built);
            if (o.verdict) (void)hipHostFree(o.verdict);
        }
    }
    delete sc;
    return RT_OK;
}

rt_status rt_scene_set_area_light(rt_scene* sc, const rt_area_light* light) {
    if (!sc) return fail(RT_ERR_INVALID_ARG, "scene is NULL");
    if (!light) {
        sc->has_area = false;
        return RT_OK;
    }
    if (light->samples <= 0) return fail(RT_ERR_INVALID_ARG, "area light needs samples > 0");
    const int k = static_cast<int>(std::lround(std::sqrt(static_cast<double>(light->samples))));
    if (k * k != light->samples)
        return fail(RT_ERR_INVALID_ARG, "area light samples must be a perfect square");
    sc->area = *light;
    sc->has_area = true;
    return RT_OK;
}

rt_status rt_render_device(rt_context* ctx, const rt_scene* sc, const rt_camera* cam,
                           const rt_render_opts* opts, void* d64, void* d32, void* dldr) {
    if (!ctx) return fail(RT_ERR_INVALID_ARG, "context is NULL");
    DeviceGuard g(ctx->device);
    return enqueue_render(ctx, sc, cam, opts, static_cast<double*>(d64), static_cast<float*>(d32),
                   static_cast<uint8_t*>(dldr));
}

rt_status rt_render_batch(rt_context* ctx, const rt_scene* sc, const rt_camera* cams,
                          int nframes, const rt_render_opts* opts, void* d64, void* d32,
                          void* dldr) {
    if (!ctx) return fail(RT_ERR_INVALID_ARG, "context is NULL");
    rt_status st = check_batch(cams, nframes);
    if (st != RT_OK) return st;
    DeviceGuard g(ctx->device);
    return enqueue_frames(ctx, sc, cams, nframes, opts, static_cast<double*>(d64),
                          static_cast<float*>(d32), static_cast<uint8_t*>(dldr));
}

rt_status rt_render(rt_context* ctx, const rt_scene* sc, const rt_camera* cam,
                    const rt_render_opts* opts, double* h64, float* h32, uint8_t* hldr,
                    rt_stats* stats) {
    if (!ctx) return fail(RT_ERR_INVALID_ARG, "context is NULL");
    rt_status st = validate_camera(cam);
    if (st != RT_OK) return st;
    DeviceGuard g(ctx->device);
    rt_render_opts o;
    if (opts) o = *opts;
    else rt_render_opts_default(&o);
    if (stats) o.flags |= RT_FLAG_COUNT_RAYS;
    const uint32_t rows = rendered_rows(o, cam->height);
    const size_t npx = static_cast<size_t>(rows) * cam->width;
    if (h64) RT_HIP(ctx->out64.ensure(npx * 3 * sizeof(double)));
    if (h32) RT_HIP(ctx->out32.ensure(npx * 3 * sizeof(float)));
    if (hldr) RT_HIP(ctx->ldr.ensure(npx * 3));
    if (stats) {
        st = scratch_wait(ctx);  // the counters: after any counting render on another stream
        if (st != RT_OK) return st;
        RT_HIP(hipMemsetAsync(ctx->counters.ptr, 0, 2 * sizeof(unsigned long long), ctx->stream));
    }
    st = enqueue_render(ctx, sc, cam, &o, h64 ? static_cast<double*>(ctx->out64.ptr) : nullptr,
                 h32 ? static_cast<float*>(ctx->out32.ptr) : nullptr,
                 hldr ? static_cast<uint8_t*>(ctx->ldr.ptr) : nullptr);
    if (st != RT_OK) return st;
    if (h64)
        RT_HIP(hipMemcpyAsync(h64, ctx->out64.ptr, npx * 3 * sizeof(double),
                              hipMemcpyDeviceToHost, ctx->stream));
    if (h32)
        RT_HIP(hipMemcpyAsync(h32, ctx->out32.ptr, npx * 3 * sizeof(float),
                              hipMemcpyDeviceToHost, ctx->stream));
    if (hldr)
        RT_HIP(hipMemcpyAsync(hldr, ctx->ldr.ptr, npx * 3, hipMemcpyDeviceToHost, ctx->stream));
    unsigned long long c[2] = {0, 0};
    if (stats) {
        // the read-back is the counters' last use: a counting render queued on another stream
        // waits for it (scratch_event), not only for the counting launch
        RT_HIP(hipMemcpyAsync(c, ctx->counters.ptr, sizeof c, hipMemcpyDeviceToHost, ctx->stream));
        st = scratch_done(ctx);
        if (st != RT_OK) return st;
    }
    RT_HIP(hipStreamSynchronize(ctx->stream));
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        stats->trace_rays = c[0];
        stats->shadow_rays = c[1];
        if (o.flags & RT_FLAG_TIME_KERNEL) {
            st = harvest_events(ctx, true);
            if (st != RT_OK) return st;
            stats->kernel_ms = ctx->timed_ms;
            stats->launches = ctx->launches;
        }
    }
    return RT_OK;
}

rt_status rt_stats_read(rt_context* ctx, rt_stats* out) {
    if (!ctx || !out) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_stats_read");
    DeviceGuard g(ctx->device);
    RT_HIP(hipStreamSynchronize(ctx->stream));
    rt_status st = harvest_events(ctx, true);
    if (st != RT_OK) return st;
    unsigned long long c[2] = {0, 0};
    RT_HIP(hipMemcpy(c, ctx->counters.ptr, sizeof c, hipMemcpyDeviceToHost));
    out->trace_rays = c[0];
    out->shadow_rays = c[1];
    out->kernel_ms = ctx->timed_ms;
    out->launches = ctx->launches;
    return RT_OK;
}

rt_status rt_stats_reset(rt_context* ctx) {
    if (!ctx) return fail(RT_ERR_INVALID_ARG, "context is NULL");
    DeviceGuard g(ctx->device);
    RT_HIP(hipStreamSynchronize(ctx->stream));
    rt_status st = harvest_events(ctx, true);
    if (st != RT_OK) return st;
    ctx->timed_ms = 0.0;
    ctx->launches = 0;
    RT_HIP(hipMemset(ctx->counters.ptr, 0, 2 * sizeof(unsigned long long)));
    return RT_OK;
}

// A 1×1 camera: the batch entry points reuse build_params for the scene/opts part only.
static rt_camera batch_camera() {
    rt_camera c;
    std::memset(&c, 0, sizeof c);
    c.width = 1;
    c.height = 1;
    c.aa_samples = 1;
    return c;
}

rt_status rt_trace_rays(rt_context* ctx, const rt_scene* sc, const rt_render_opts* opts,
                        const double* rays, size_t n, double* rgb, rt_stats* stats) {
    if (!ctx || (n && (!rays || !rgb))) return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_trace_rays");
    DeviceGuard g(ctx->device);
    const rt_camera cam = batch_camera();
    rt_render_opts o;
    if (opts) o = *opts;
    else rt_render_opts_default(&o);
    o.row_begin = 0;
    o.row_end = 0;
    TraceParams p;
    int path;
    bool lds;
    size_t lds_bytes;
    uint32_t rows;
    rt_status st = build_params(ctx, sc, &cam, &o, p, path, lds, lds_bytes, rows);
    if (st != RT_OK) return st;
    if (stats) std::memset(stats, 0, sizeof *stats);
    if (n == 0) return RT_OK;
    RT_HIP(ctx->rays.ensure(n * 9 * sizeof(double)));
    double* d_rays = static_cast<double*>(ctx->rays.ptr);
    double* d_out = d_rays + 6 * n;
    RT_HIP(hipMemcpyAsync(d_rays, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    RT_HIP(launch_trace_rays(p, path, false, d_rays, n, d_out, ctx->stream));
    RT_HIP(hipMemcpyAsync(rgb, d_out, n * 3 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    if (stats) {
        p.counters = static_cast<unsigned long long*>(ctx->counters.ptr);
        st = scratch_wait(ctx);
        if (st != RT_OK) return st;
        RT_HIP(hipMemsetAsync(p.counters, 0, 2 * sizeof(unsigned long long), ctx->stream));
        RT_HIP(launch_trace_rays(p, path, true, d_rays, n, d_out, ctx->stream));
        unsigned long long c[2] = {0, 0};
        RT_HIP(hipMemcpyAsync(c, p.counters, sizeof c, hipMemcpyDeviceToHost, ctx->stream));
        st = scratch_done(ctx);  // the counters' last user is this read-back
        if (st != RT_OK) return st;
        RT_HIP(hipStreamSynchronize(ctx->stream));
        stats->trace_rays = c[0];
        stats->shadow_rays = c[1];
        return RT_OK;
    }
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

rt_status rt_intersect_rays(rt_context* ctx, const rt_scene* sc, const double* rays, size_t n,
                            double* hits) {
    if (!ctx || (n && (!rays || !hits)))
        return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_intersect_rays");
    DeviceGuard g(ctx->device);
    const rt_camera cam = batch_camera();
    TraceParams p;
    int path;
    bool lds;
    size_t lds_bytes;
    uint32_t rows;
    rt_status st = build_params(ctx, sc, &cam, nullptr, p, path, lds, lds_bytes, rows);
    if (st != RT_OK) return st;
    if (n == 0) return RT_OK;
    RT_HIP(ctx->rays.ensure(n * 15 * sizeof(double)));
    double* d_rays = static_cast<double*>(ctx->rays.ptr);
    double* d_out = d_rays + 6 * n;
    RT_HIP(hipMemcpyAsync(d_rays, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    RT_HIP(launch_intersect_rays(p, d_rays, n, d_out, ctx->stream));
    RT_HIP(hipMemcpyAsync(hits, d_out, n * 9 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

rt_status rt_tonemap(rt_context* ctx, const double* hdr, size_t n, int op, uint8_t* out) {
    if (!ctx || (!hdr && n) || (!out && n))
        return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_tonemap");
    if (op < 0 || op > RT_TONEMAP_COUNT) return fail(RT_ERR_INVALID_ARG, "tonemap op out of range");
    if (n == 0) return RT_OK;
    DeviceGuard g(ctx->device);
    const size_t planes = op == RT_TONEMAP_COUNT ? RT_TONEMAP_COUNT : 1;
    RT_HIP(ctx->tm_in.ensure(n * 3 * sizeof(double)));
    RT_HIP(ctx->tm_out.ensure(planes * n * 3));
    RT_HIP(hipMemcpyAsync(ctx->tm_in.ptr, hdr, n * 3 * sizeof(double), hipMemcpyHostToDevice,
                          ctx->stream));
    RT_HIP(launch_tonemap(static_cast<const double*>(ctx->tm_in.ptr), n, op,
                          static_cast<uint8_t*>(ctx->tm_out.ptr), ctx->stream));
    RT_HIP(hipMemcpyAsync(out, ctx->tm_out.ptr, planes * n * 3, hipMemcpyDeviceToHost,
                          ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

rt_status rt_debug_f64_ops(rt_context* ctx, const double* x, const double* y, size_t n,
                           double* out) {
    if (!ctx || !x || !y || !out) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    DeviceGuard g(ctx->device);
    RT_HIP(ctx->dbg.ensure(n * 7 * sizeof(double)));
    double* dx = static_cast<double*>(ctx->dbg.ptr);
    double* dy = dx + n;
    double* dout = dy + n;
    RT_HIP(hipMemcpyAsync(dx, x, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    RT_HIP(hipMemcpyAsync(dy, y, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    RT_HIP(launch_debug_f64(dx, dy, n, dout, ctx->stream));
    RT_HIP(hipMemcpyAsync(out, dout, 5 * n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

rt_status rt_debug_tile_order(rt_context* ctx, const rt_scene* sc, const rt_camera* cam,
                              uint32_t* order, uint32_t* cost, size_t capacity, uint32_t* tiles,
                              uint32_t* waves, int* state) {
    if (!ctx || !sc || !cam || !tiles || !waves || !state)
        return fail(RT_ERR_INVALID_ARG, "NULL argument to rt_debug_tile_order");
    *tiles = *waves = 0;
    *state = 0;
    DeviceGuard g(ctx->device);
    RT_HIP(hipDeviceSynchronize());
    for (const auto& im : sc->pk_images) {
        if (std::memcmp(im.cam, cam->position, sizeof im.cam) != 0) continue;
        if (im.last_ord < 0) return RT_OK;
        const auto& o = im.ords[static_cast<size_t>(im.last_ord)];
        *state = o.state;
        if (o.state == 0) return RT_OK;
        *tiles = o.key[0] * o.key[1];
        *waves = o.key[2];
        if (order && o.state == 2) {
            if (capacity < *tiles) return fail(RT_ERR_INVALID_ARG, "order capacity too small");
            RT_HIP(hipMemcpy(order, o.order.ptr, sizeof(uint32_t) * *tiles, hipMemcpyDeviceToHost));
        }
        if (cost) {
            if (capacity < size_t(*tiles) * *waves)
                return fail(RT_ERR_INVALID_ARG, "cost capacity too small");
            RT_HIP(hipMemcpy(cost, o.cost.ptr, sizeof(uint32_t) * *tiles * *waves,
                             hipMemcpyDeviceToHost));
        }
        return RT_OK;
    }
    return RT_OK;
}

rt_status rt_debug_vec_ops(rt_context* ctx, const double* v, size_t n, double* out) {
    if (!ctx || !v || !out) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    DeviceGuard g(ctx->device);
    RT_HIP(ctx->dbg.ensure(n * 19 * sizeof(double)));
    double* dv = static_cast<double*>(ctx->dbg.ptr);
    double* dout = dv + 3 * n;
    RT_HIP(hipMemcpyAsync(dv, v, 3 * n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    RT_HIP(launch_debug_vec(dv, n, dout, ctx->stream));
    RT_HIP(hipMemcpyAsync(out, dout, 16 * n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

}  // extern "C"
