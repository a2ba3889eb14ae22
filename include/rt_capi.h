/*
 * rt_capi.h — C-ABI of the MI355X (gfx950) renderer that replaces the CPU hot path of
 * Sorax5/RaytracingEngine.  Plain C types only: pointers, sizes, PODs.  No exceptions cross
 * this boundary; every entry point returns an rt_status and the message of the last failure
 * on the calling thread is available from rt_last_error().
 *
 * Reference interface each entry point replaces (paths relative to /root/reference/RaytracingEngine):
 *
 *   rt_render / rt_render_device   std::vector<Vec3> Scene::RenderImage() const      Scene.h:311-328
 *                                  (per pixel: GeneratePixelAt Scene.h:283-304 → TraceRay Scene.h:131-198
 *                                   → IntersectClosest Scene.h:218-257, directLightning Scene.h:79-129,
 *                                   computeTransmittance Scene.h:35-77, backgroundColor Scene.h:30-33)
 *   rt_tonemap                     tonemap() RaytracingEngine.cpp:165-174 and the operators of
 *                                  tonemapAll() RaytracingEngine.cpp:176-214, each followed by
 *                                  toColor() RaytracingEngine.cpp:113-121
 *   rt_scene_create                the scene state Scene::AddSphere/AddPlane/AddLight/AddTriangle/
 *                                  AddModel accumulate (Scene.h:208-212)
 *   rt_camera                      Camera (Math.h:85-122); antiAliasingAmount Math.h:94
 *
 * The C++20 drop-in headers under raytracingengine_amd/api/ (Math.h, Shape.h, Light.h, Scene.h,
 * Image.h) are the reference-shaped API above this ABI; see INTEGRATION.md.
 *
 * Numerics: all geometry and shading is IEEE binary64 evaluated in the reference's operation
 * order without FMA contraction, so images are bit-identical to the reference except where the
 * reference calls libm pow/log (Blinn-Phong, Fresnel, Reinhard-Jodie), which may differ by an ulp.
 */
#ifndef RT_CAPI_H
#define RT_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_CAPI_VERSION 1

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = 1, /* null pointer, zero size, inconsistent counts, bad row range   */
    RT_ERR_HIP = 2,         /* a HIP runtime call failed (message names the call)           */
    RT_ERR_OOM = 3,         /* device allocation failed                                     */
    RT_ERR_UNSUPPORTED = 4, /* a request outside what this build implements                 */
    RT_ERR_NO_DEVICE = 5,   /* no gfx950 device at the requested ordinal                    */
    RT_ERR_RCCL = 6         /* an RCCL call failed (message names the call)                 */
} rt_status;

/* Material (Shape.h:13-19).  Defaults in the reference: shininess 128, specular 0,
 * transparency 0, refractive_index 1. */
typedef struct rt_material {
    double color[3];
    double shininess;
    double specular;
    double transparency;
    double refractive_index;
} rt_material;

/* Sphere (Shape.h:59-133): centre = Transform.position, radius. */
typedef struct rt_sphere {
    double center[3];
    double radius;
    rt_material material;
} rt_sphere;

/* Plane (Shape.h:135-186).  `normal` is the normal as the Plane object stores it, i.e.
 * already passed through Vec3::normalize() by the constructor (Shape.h:141-142). */
typedef struct rt_plane {
    double point[3];
    double normal[3];
    rt_material material;
} rt_plane;

/* Triangle (Shape.h:188-246): untranslated vertices plus Transform.position, which the
 * reference adds to every vertex on each query (tv0/tv1/tv2, Shape.h:198-200).  A Model
 * (Shape.h:248-307) is flattened into triangles that carry the model's material and
 * translation.  Order in rt_scene_desc.triangles: the scene's standalone triangles in
 * AddTriangle order, then every model's triangles in AddModel order and index order — the
 * closest-hit order of Scene::IntersectClosest (Scene.h:243-254). */
typedef struct rt_triangle {
    double v0[3];
    double v1[3];
    double v2[3];
    double translation[3];
    rt_material material;
} rt_triangle;

/* Point light (Light.h:6-15). */
typedef struct rt_light {
    double position[3];
    double color[3];
    double intensity;
} rt_light;

typedef struct rt_scene_desc {
    const rt_sphere* spheres;
    int32_t n_spheres;
    const rt_plane* planes;
    int32_t n_planes;
    const rt_triangle* triangles;
    int32_t n_triangles;
    const rt_light* lights;
    int32_t n_lights;
} rt_scene_desc;

/* Camera (Math.h:85-122).  aa_samples = Camera::antiAliasingAmount (reference default 32).
 * near/far are carried for API completeness; the trace does not read them (as in the
 * reference). */
typedef struct rt_camera {
    double position[3];
    double focal;
    uint32_t width;
    uint32_t height;
    int32_t aa_samples;
    int32_t _pad0;
    double near_plane;
    double far_plane;
} rt_camera;

/* Tonemap operators (RaytracingEngine.cpp:123-174), in tonemapAll()'s output order. */
typedef enum rt_tonemap_op {
    RT_TONEMAP_NONE = -1,                    /* no LDR output                               */
    RT_TONEMAP_SIMPLE = 0,                   /* simple()                       :123-131     */
    RT_TONEMAP_REINHARD = 1,                 /* reinhardSimple()               :133-135     */
    RT_TONEMAP_REINHARD_EXTENDED = 2,        /* reinhardExtended(c, 5.0)       :137-141,193 */
    RT_TONEMAP_REINHARD_EXTENDED_LUMINANCE = 3, /* reinhardExtendedLuminance(c, 5.0) :143-148,195 */
    RT_TONEMAP_REINHARD_JODIE = 4,           /* reinhardJodie(c, 0.18)         :150-154     */
    RT_TONEMAP_UNCHARTED2 = 5,               /* uncharted2()                   :156-163     */
    RT_TONEMAP_ACES = 6,                     /* aces_approx() == tonemap()     :89-98,165   */
    RT_TONEMAP_COUNT = 7
} rt_tonemap_op;

/* Soft-shadow extension (BASELINE config 5).  The reference has point lights only
 * (Light.h); an area light is a build-defined extension with no reference semantics. */
typedef struct rt_area_light {
    double corner[3];    /* one corner of the parallelogram emitter                        */
    double edge_u[3];    /* first edge vector                                              */
    double edge_v[3];    /* second edge vector                                             */
    double color[3];
    double intensity;    /* total intensity, split evenly over the samples                 */
    int32_t samples;     /* stratified samples per shading point (sqrt must be integral)   */
    int32_t _pad0;
} rt_area_light;

typedef struct rt_render_opts {
    int32_t max_recursion;   /* Scene::maxRecursion, reference value 10 (Scene.h:24)        */
    int32_t tonemap;         /* rt_tonemap_op applied to the LDR output, if requested       */
    double bias;             /* GeneratePixelAt's bias, reference value 1e-3 (Scene.h:291)  */
    uint64_t seed;           /* key of the counter-based AA jitter RNG (samples 1..N-1)     */
    uint32_t row_begin;      /* render rows [row_begin, row_end) only (row tiles for        */
    uint32_t row_end;        /*  multi-GPU); row_end == 0 means the full image height       */
    int32_t flags;           /* RT_FLAG_* bits                                              */
    /* Block-cyclic row sets (load-balanced multi-GPU frames).  With row_cycle > 1 the call
     * renders the blocks of row_block rows starting at row_begin + k*row_cycle*row_block
     * (k = 0, 1, ...), clipped to row_end, packed one after another in the outputs: rank r of
     * n passes row_begin = r*row_block, row_cycle = n.  0 / 1: the contiguous range above. */
    uint16_t row_block;
    uint16_t row_cycle;
} rt_render_opts;

#define RT_FLAG_COUNT_RAYS 0x1   /* also run the ray-counting pass (fills rt_stats counts)   */
#define RT_FLAG_TIME_KERNEL 0x2  /* bracket each render launch with HIP events              */
#define RT_FLAG_GENERIC_KERNEL 0x4 /* ablation: bypass the packet-culled kernel              */
#define RT_FLAG_NO_BVH 0x8         /* ablation: test every triangle (no triangle BVH)          */
#define RT_FLAG_PIPELINE 0x10      /* rt_render_gather: gather + assembly on the communicator's
                                      own stream, overlapping the next frame's render (two
                                      frame slots); rt_comm_synchronize waits for the frame   */
#define RT_FLAG_NO_TILE_ORDER 0x20 /* ablation: the packet kernel's default tile order instead
                                      of costliest tiles first (the image is the same)        */
#define RT_FLAG_NO_SAMPLE_PARALLEL 0x40 /* ablation: multi-sample planes-only chains loop over
                                      the samples per thread instead of one thread per sample
                                      (the image is the same)                                 */

/* Fills opts with the reference defaults: max_recursion 10, bias 1e-3, tonemap ACES,
 * full image, seed 0x5EED, no flags. */
void rt_render_opts_default(rt_render_opts* opts);

typedef struct rt_stats {
    uint64_t trace_rays;   /* TraceRay invocations that reach IntersectClosest              */
    uint64_t shadow_rays;  /* computeTransmittance invocations                              */
    double kernel_ms;      /* summed HIP-event time of render launches (RT_FLAG_TIME_KERNEL)*/
    uint64_t launches;     /* render launches timed into kernel_ms                          */
} rt_stats;

typedef struct rt_context rt_context;
typedef struct rt_scene rt_scene;

/* Thread-local message of the most recent failure ("" if none). */
const char* rt_last_error(void);

/* The build record of this library (no reference counterpart): a static JSON object with the
 * sha256 of the sources, headers and flags it was compiled from ("source_sha256"), the target
 * ("arch") and the compiler ("hipcc"), so that a run can check which sources its binary holds
 * (raytracingengine_amd/build.py source_digest). */
const char* rt_build_info(void);

/* Number of visible HIP devices (0 when none). */
int rt_device_count(void);

/* A context owns one HIP device, one stream and growable device buffers.  One context per
 * host thread; calls on a context are not thread-safe. */
rt_status rt_context_create(int device, rt_context** out);
rt_status rt_context_destroy(rt_context* ctx);
/* Make the context launch on an externally owned hipStream_t (NULL = its own stream). */
rt_status rt_context_set_stream(rt_context* ctx, void* hip_stream);
rt_status rt_context_synchronize(rt_context* ctx);

/* Upload a scene to the context's device (done once; the render then reads it from HBM). */
rt_status rt_scene_create(rt_context* ctx, const rt_scene_desc* desc, rt_scene** out);
rt_status rt_scene_destroy(rt_scene* scene);
/* Attach (or with NULL, detach) a build-defined area light to an uploaded scene. */
rt_status rt_scene_set_area_light(rt_scene* scene, const rt_area_light* light);

/* Synchronous host-buffer render: Scene::RenderImage().  Any of the three outputs may be
 * NULL.  hdr64_out: rows*width*3 doubles, row-major, idx = (y-row_begin)*W + x, RGB (the
 * reference's std::vector<Vec3> layout).  hdr32_out: the same as float.  ldr_out:
 * rows*width*3 bytes of opts->tonemap followed by toColor().  stats may be NULL. */
rt_status rt_render(rt_context* ctx, const rt_scene* scene, const rt_camera* cam,
                    const rt_render_opts* opts, double* hdr64_out, float* hdr32_out,
                    uint8_t* ldr_out, rt_stats* stats);

/* One frame on n contexts (one per GPU, each with its own copy of the scene: scenes[i] belongs to
 * ctxs[i]), returned in the caller's host buffers — Scene::RenderImage (Scene.h:311-328) over the
 * GPUs of a node from one process.  Context i renders the block-cyclic row set i of n
 * (opts->row_block rows per block, default 16; the row range and row_cycle of opts must be left
 * at the whole image).  Contexts on distinct GPUs: the RCCL path — communicators over their
 * devices (ncclCommInitAll, created on first use and cached in ctxs[0] until the list changes),
 * rt_render_gather_all into ctxs[0]'s device, one device-to-host copy per output.  Contexts that
 * share a GPU (RCCL allows one rank per GPU): the same through rt_comm_create_local (the gather
 * as device copies); RTAMD_MULTI_HOST=1 copies each context's rows straight to their host rows.
 * Stats, when requested, are summed over the contexts (kernel_ms: the slowest GPU's render). */
rt_status rt_render_multi(rt_context* const* ctxs, rt_scene* const* scenes, int n,
                          const rt_camera* cam, const rt_render_opts* opts, double* hdr64_out,
                          float* hdr32_out, uint8_t* rgb8_out, rt_stats* stats);

/* ---- Row-tiled frames over the GPUs of a node with ONE RCCL gather ----------
 * Replaces the pixel loop of Scene::RenderImage (Scene.h:318-325) split by rows: rank r of n
 * renders the block-cyclic row set r (blocks of opts->row_block rows, default 16, starting at
 * row r*block and every n*block rows after it), one ncclGather per requested output moves every
 * rank's rows (padded to the largest rank's) to rank 0 over xGMI, and rank 0 writes them into
 * image row order in its device framebuffers.  Everything is enqueued on the communicator's
 * context stream; no host synchronisation. */
#define RT_COMM_ID_BYTES 128    /* == NCCL_UNIQUE_ID_BYTES                                   */
#define RT_OUT_HDR64 0x1        /* float64 Vec3 framebuffer (24 B/px)                        */
#define RT_OUT_HDR32 0x2        /* float32 framebuffer (12 B/px)                             */
#define RT_OUT_LDR 0x4          /* tonemapped bytes of opts->tonemap (3 B/px)                */

typedef struct rt_comm rt_comm;

typedef struct rt_gather_timing {
    double render_ms;    /* summed over the timed frames (RT_FLAG_TIME_KERNEL), this rank   */
    double gather_ms;    /* the ncclGather(s), from the end of this rank's render           */
    double assemble_ms;  /* rank 0: the gathered rows written into image order              */
    uint64_t frames;     /* frames timed                                                    */
    uint32_t rows;       /* rows this rank renders per frame                                */
    uint32_t max_rows;   /* rows every rank sends (the largest rank's)                      */
} rt_gather_timing;

/* ncclGetUniqueId: called on one process, the bytes handed to every rank (any transport). */
rt_status rt_comm_unique_id(uint8_t* id /* RT_COMM_ID_BYTES */);
/* One rank of an n-rank communicator on ctx's device (non-blocking ncclCommInitRankConfig): one
 * process per GPU.  Destroy communicators before their contexts.  Failure detection (SURVEY §5;
 * the reference has no communicator): every wait on the communicator — its initialisation, the
 * issue of each gather, rt_comm_synchronize, rt_comm_set_root_weight — polls
 * ncclCommGetAsyncError with a deadline (rt_comm_create: RTAMD_COMM_TIMEOUT_MS, default 300000;
 * 0 = none).  On an asynchronous RCCL error or at the deadline the communicator is aborted
 * (ncclCommAbort: its kernels in flight return) and the call fails with RT_ERR_RCCL; every later
 * call on it fails the same way (destroy it and create a new one).  A rank whose peers never
 * join therefore gets RT_ERR_RCCL from rt_comm_create instead of blocking for ever. */
rt_status rt_comm_create(rt_context* ctx, int nranks, int rank, const uint8_t* id, rt_comm** out);
/* rt_comm_create with its deadline in milliseconds (0 = wait without a deadline). */
rt_status rt_comm_create_ex(rt_context* ctx, int nranks, int rank, const uint8_t* id,
                            long timeout_ms, rt_comm** out);
/* The deadline of the communicator's later waits (milliseconds, 0 = none). */
rt_status rt_comm_set_timeout(rt_comm* comm, long timeout_ms);
/* n communicators, one per context, over n DISTINCT devices from one process (ncclCommInitAll);
 * comms_out[i] is rank i on ctxs[i]. */
rt_status rt_comm_create_all(rt_context* const* ctxs, int n, rt_comm** comms_out);
/* n communicators over n contexts of ONE process that may share a GPU (RCCL allows one rank per
 * GPU): the same multi-rank frame — row plan, padded send buffers, rank 0's receive layout and
 * assembly, the pipelined slots — with the gather done as device-to-device copies of every
 * rank's packed rows into rank 0's receive buffer (what ncclGather delivers).  Driven only by
 * rt_render_gather_all; rt_render_multi uses it for contexts that share a device. */
rt_status rt_comm_create_local(rt_context* const* ctxs, int n, rt_comm** comms_out);
rt_status rt_comm_destroy(rt_comm* comm);
rt_status rt_comm_info(const rt_comm* comm, int* nranks, int* rank);
/* Weighted row split (every rank of the communicator sets the same weight before its next frame;
 * default 1).  Collective on an rt_comm_create communicator with n > 1: the ranks check that
 * they agree (one all-reduce) and all return RT_ERR_INVALID_ARG, weight unchanged, if not.
 * rt_render_gather_all[_batch] checks that its communicators carry one weight.  The frame's blocks are dealt over weight + n − 1 row sets, rank 0 renders `weight`
 * of them and every other rank one — rank 0's rows never cross a link, so when the peers' gathers
 * are link-bound it takes a larger share.  With weight > 1 the gather is a group of P2P sends of
 * equal counts (ncclSend / ncclRecv) into rank 0's receive buffer, where rank 0 renders its own
 * row sets in place; rank-local outputs of rank 0 hold its row sets one after another (each
 * nframes*max_rows*W*3 elements).  rt_gather_timing.rows is a rank's total. */
rt_status rt_comm_set_root_weight(rt_comm* comm, int weight);
/* Collective: every rank calls it with the same camera, opts and outputs (RT_OUT_* bits).  The
 * scene belongs to the communicator's context.  On rank 0 the d_* are whole-frame device
 * framebuffers (W*H*3 elements, image order) for every requested output; elsewhere ignored.
 * opts->flags RT_FLAG_TIME_KERNEL records the frame's render / gather / assembly times. */
rt_status rt_render_gather(rt_comm* comm, const rt_scene* scene, const rt_camera* cam,
                           const rt_render_opts* opts, int outputs, void* d_hdr64,
                           void* d_hdr32, void* d_ldr);
/* The same from one process for every rank of an rt_comm_create_all (one ncclGroup) or of an
 * rt_comm_create_local.  With n == 1 the rank renders straight into the framebuffers. */
rt_status rt_render_gather_all(rt_comm* const* comms, rt_scene* const* scenes, int n,
                               const rt_camera* cam, const rt_render_opts* opts, int outputs,
                               void* d_hdr64, void* d_hdr32, void* d_ldr);
/* A batch of nframes frames (see rt_render_batch: one camera per frame, same width / height /
 * focal / aa_samples) in one call: this rank renders its rows of every frame in one launch,
 * frame after frame at a stride of max_rows rows (the largest rank's row count), then ONE
 * ncclGather per gathered output moves the whole batch, and rank 0 assembles every frame (one
 * launch).  On rank 0 the d_* hold nframes whole frames back to back (frame f at f*W*H*3
 * elements).  rank_* (any may be NULL) receive outputs that are rendered but NOT gathered: this
 * rank's rows of every frame, packed, frame f at f*max_rows*W*3 elements (max_rows =
 * rt_gather_timing.max_rows; a rank with fewer rows leaves the rest of each frame's stride
 * unwritten; buffers of nframes*max_rows*W*3 elements) — e.g. the float64 HDR framebuffer kept
 * where it was rendered while the tonemapped bytes are gathered.  An output is either gathered
 * (in `outputs`) or rank-local, not both.  rt_render_gather = nframes 1, no rank_*. */
rt_status rt_render_gather_batch(rt_comm* comm, const rt_scene* scene, const rt_camera* cams,
                                 int nframes, const rt_render_opts* opts, int outputs,
                                 void* d_hdr64, void* d_hdr32, void* d_ldr, void* rank_hdr64,
                                 void* rank_hdr32, void* rank_ldr);
/* rt_render_gather_all for a batch of frames (the layouts of rt_render_gather_batch). */
rt_status rt_render_gather_all_batch(rt_comm* const* comms, rt_scene* const* scenes, int n,
                                     const rt_camera* cams, int nframes,
                                     const rt_render_opts* opts, int outputs, void* d_hdr64,
                                     void* d_hdr32, void* d_ldr);
/* Waits for every frame enqueued on the communicator (render, gather, assembly); on an
 * rt_comm_create communicator with n > 1 it polls the streams and ncclCommGetAsyncError and
 * aborts the communicator on an RCCL error or at its deadline (RT_ERR_RCCL). */
rt_status rt_comm_synchronize(rt_comm* comm);
/* Summed frame timings since the last reset (waits for the timed frames to finish). */
rt_status rt_comm_timing(rt_comm* comm, rt_gather_timing* out, int reset);

/* Asynchronous render into DEVICE buffers on the context's stream (inputs and outputs stay
 * resident in HBM).  Same layouts as rt_render; pointers are device pointers or NULL. */
rt_status rt_render_device(rt_context* ctx, const rt_scene* scene, const rt_camera* cam,
                           const rt_render_opts* opts, void* d_hdr64, void* d_hdr32,
                           void* d_ldr);
/* A batch of frames: Scene::RenderImage (Scene.h:311-328) once per camera of cams[0..nframes)
 * — views of one scene from several positions (an animation's frames, a camera path) — into
 * device buffers holding the frames back to back (frame f at f*rows*W*3 elements of each
 * output).  Every camera must have cams[0]'s width, height, focal and aa_samples; the position
 * may differ.  Scenes the packet kernel renders (no secondary rays) take up to 32 frames per
 * launch (one grid plane per frame), so the launch's ramp and drain are paid once per batch;
 * other scenes take one launch per frame.  Each frame is the frame rt_render_device gives. */
rt_status rt_render_batch(rt_context* ctx, const rt_scene* scene, const rt_camera* cams,
                          int nframes, const rt_render_opts* opts, void* d_hdr64,
                          void* d_hdr32, void* d_ldr);

/* ---- Serving frame queue -------------------------------------------------------------------
 * Consecutive Scene::RenderImage() frames (Scene.h:311-328) into device framebuffers with
 * `depth` frames in flight on as many HIP streams of the context's device (depth 1..8), so that
 * one frame's launch tail can overlap the next frame's start.  Measured on MI355X with the C2
 * 1080p frame at the sustained clock it does not pay (45.4 µs per frame on one stream; 48.3 /
 * 47.3 / 46.1 µs at depth 2 / 3 / 4: concurrent frames contend for the same CUs); it serves
 * applications that submit frames from one thread without managing streams.  Frames are
 * independent; each submit returns a ticket, and
 * rt_queue_wait(ticket) returns once that frame's outputs are written.  The caller keeps the
 * framebuffers of frames in flight untouched (e.g. `depth` sets of them, used round-robin). */
typedef struct rt_queue rt_queue;
rt_status rt_queue_create(rt_context* ctx, int depth, rt_queue** out);
rt_status rt_queue_destroy(rt_queue* queue);
/* rt_render_device on the queue's next stream; *ticket (may be NULL) numbers the frame. */
rt_status rt_queue_submit(rt_queue* queue, const rt_scene* scene, const rt_camera* cam,
                          const rt_render_opts* opts, void* d_hdr64, void* d_hdr32, void* d_ldr,
                          uint64_t* ticket);
rt_status rt_queue_wait(rt_queue* queue, uint64_t ticket);
/* Waits for every submitted frame (and folds RT_FLAG_TIME_KERNEL timings into rt_stats). */
rt_status rt_queue_synchronize(rt_queue* queue);

/* Ray counts (and, with RT_FLAG_TIME_KERNEL, accumulated kernel time) since the last reset. */
rt_status rt_stats_read(rt_context* ctx, rt_stats* out);
rt_status rt_stats_reset(rt_context* ctx);

/* Batch Scene::TraceRay (Scene.h:131-198) at recursion depth 0 for n arbitrary host rays
 * {ox,oy,oz,dx,dy,dz}: the per-sample body of GenerateAntiAliasing (Scene.h:306-309).
 * rgb_out: n*3 doubles.  opts->max_recursion/bias/seed apply; the area-light RNG is keyed by
 * the ray's index.  stats may be NULL. */
rt_status rt_trace_rays(rt_context* ctx, const rt_scene* scene, const rt_render_opts* opts,
                        const double* rays, size_t n, double* rgb_out, rt_stats* stats);

/* Batch Scene::IntersectClosest (Scene.h:218-257) for n host rays.  hits_out: n*9 doubles
 * {type, index, distance, normal.xyz, hitPoint.xyz}; type 0 = miss (index -1), 1 sphere,
 * 2 plane, 3 triangle (index into rt_scene_desc.triangles). */
rt_status rt_intersect_rays(rt_context* ctx, const rt_scene* scene, const double* rays,
                            size_t n, double* hits_out);

/* Device tonemap of host FP64 radiance: op in [0, RT_TONEMAP_COUNT) writes n*3 bytes;
 * op == RT_TONEMAP_COUNT writes all seven operators, tonemapAll() order, 7*n*3 bytes. */
rt_status rt_tonemap(rt_context* ctx, const double* hdr, size_t n_pixels, int op,
                     uint8_t* ldr_out);

/* Test hook: evaluates x/y, sqrt(x), pow(x,y), log(x) and the Blinn-Phong pow of the trace
 * kernels (rt_device.hpp pow_bp) on the device for n inputs so the parity suite can pin device
 * libm against the host's.  out: 5*n doubles. */
rt_status rt_debug_f64_ops(rt_context* ctx, const double* x, const double* y, size_t n,
                           double* out);

/* Test hook: per 3-vector v (3*n doubles), the normalize / light-vector results of the fast
 * sqrt/division cores next to the compiler's exact lowering, so the parity suite can pin them bit
 * for bit.  out: 16*n doubles (layout in rt_trace.hip, debug_vec_kernel). */
rt_status rt_debug_vec_ops(rt_context* ctx, const double* v, size_t n, double* out);

/* Test hook: rank 0's assembly step alone (gathered [n][max_rows][row_bytes] host buffer ->
 * image-order [height][row_bytes] host buffer) for row plans the 1-GPU test box cannot run. */
rt_status rt_debug_assemble_rows(rt_context* ctx, const void* gathered, size_t row_bytes,
                                 uint32_t height, uint32_t block, uint32_t n, uint32_t max_rows,
                                 void* image);

/* Test hook: the packet kernel's costliest-first tile order of `scene` seen from cam->position
 * (rt_capi.cpp tile_order): *tiles / *waves receive the launch shape (0 when the camera has no
 * order state), `order` (capacity `tiles`) the dispatch order once built, `cost` (capacity
 * tiles*waves) the recorded wave durations (100 MHz ticks); either may be NULL. */
rt_status rt_debug_tile_order(rt_context* ctx, const rt_scene* scene, const rt_camera* cam,
                              uint32_t* order, uint32_t* cost, size_t capacity, uint32_t* tiles,
                              uint32_t* waves, int* state);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* RT_CAPI_H */
