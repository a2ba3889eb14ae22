"""ctypes binding of ``include/rt_capi.h`` (the HIP library ``librtamd.so``).

This is plumbing for the bench and the parity tests: every call goes straight to the C-ABI.
There is no CPU fallback — if the library or a gfx950 device is missing, the calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .scene import AREA_LIGHT_DTYPE, SceneData

HERE = os.path.dirname(os.path.abspath(__file__))
# RTAMD_LIB overrides the library path (A/B builds in tools/); default: the in-tree build.
LIB_PATH = os.environ.get("RTAMD_LIB", os.path.join(HERE, "librtamd.so"))

(RT_OK, RT_ERR_INVALID_ARG, RT_ERR_HIP, RT_ERR_OOM, RT_ERR_UNSUPPORTED, RT_ERR_NO_DEVICE,
 RT_ERR_RCCL) = range(7)
STATUS_NAMES = {0: "RT_OK", 1: "RT_ERR_INVALID_ARG", 2: "RT_ERR_HIP", 3: "RT_ERR_OOM",
                4: "RT_ERR_UNSUPPORTED", 5: "RT_ERR_NO_DEVICE", 6: "RT_ERR_RCCL"}

TONEMAP_NONE = -1
TONEMAPS = ["simple", "reinhard_simple", "reinhard_extended", "reinhard_extended_luminance",
            "reinhard_jodie", "uncharted2", "aces"]
TONEMAP_ALL = 7
RT_FLAG_COUNT_RAYS = 0x1
RT_FLAG_TIME_KERNEL = 0x2
RT_FLAG_GENERIC_KERNEL = 0x4
RT_FLAG_NO_BVH = 0x8
RT_FLAG_PIPELINE = 0x10
RT_FLAG_NO_TILE_ORDER = 0x20
RT_FLAG_NO_SAMPLE_PARALLEL = 0x40
RT_OUT_HDR64, RT_OUT_HDR32, RT_OUT_LDR = 0x1, 0x2, 0x4
RT_COMM_ID_BYTES = 128

# Every symbol include/rt_capi.h declares (checked by tests/test_capi_symbols.py).
EXPORTED = [
    "rt_last_error", "rt_build_info", "rt_device_count", "rt_render_opts_default", "rt_context_create",
    "rt_context_destroy", "rt_context_set_stream", "rt_context_synchronize", "rt_scene_create",
    "rt_scene_destroy", "rt_scene_set_area_light", "rt_render", "rt_render_device",
    "rt_render_multi", "rt_comm_unique_id", "rt_comm_create", "rt_comm_create_all",
    "rt_comm_create_local", "rt_comm_destroy", "rt_comm_info", "rt_comm_set_root_weight",
    "rt_comm_create_ex", "rt_comm_set_timeout", "rt_render_gather", "rt_render_gather_all",
    "rt_comm_timing", "rt_comm_synchronize", "rt_debug_assemble_rows", "rt_debug_tile_order",
    "rt_stats_read", "rt_stats_reset", "rt_trace_rays", "rt_intersect_rays", "rt_tonemap",
    "rt_debug_f64_ops", "rt_debug_vec_ops", "rt_queue_create", "rt_queue_destroy",
    "rt_queue_submit", "rt_queue_wait", "rt_queue_synchronize", "rt_render_batch",
    "rt_render_gather_batch", "rt_render_gather_all_batch",
]


class RtError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class SceneDesc(ctypes.Structure):
    _fields_ = [
        ("spheres", ctypes.c_void_p), ("n_spheres", ctypes.c_int32),
        ("planes", ctypes.c_void_p), ("n_planes", ctypes.c_int32),
        ("triangles", ctypes.c_void_p), ("n_triangles", ctypes.c_int32),
        ("lights", ctypes.c_void_p), ("n_lights", ctypes.c_int32),
    ]


class RenderOpts(ctypes.Structure):
    _fields_ = [
        ("max_recursion", ctypes.c_int32), ("tonemap", ctypes.c_int32),
        ("bias", ctypes.c_double), ("seed", ctypes.c_uint64),
        ("row_begin", ctypes.c_uint32), ("row_end", ctypes.c_uint32),
        ("flags", ctypes.c_int32), ("row_block", ctypes.c_uint16), ("row_cycle", ctypes.c_uint16),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("trace_rays", ctypes.c_uint64), ("shadow_rays", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double), ("launches", ctypes.c_uint64),
    ]


class GatherTiming(ctypes.Structure):
    _fields_ = [
        ("render_ms", ctypes.c_double), ("gather_ms", ctypes.c_double),
        ("assemble_ms", ctypes.c_double), ("frames", ctypes.c_uint64),
        ("rows", ctypes.c_uint32), ("max_rows", ctypes.c_uint32),
    ]


_lib = None


def load_library(path: str = LIB_PATH):
    """Load librtamd.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        # One HIP runtime per process: torch ships its own libamdhip64.so.7; loading it first
        # makes librtamd.so's NEEDED entry bind to that copy instead of /opt/rocm's.
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (hipcc --offload-arch=gfx950). The renderer has no CPU fallback.")
    L = ctypes.CDLL(path)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    L.rt_last_error.restype = ctypes.c_char_p
    if hasattr(L, "rt_build_info") or "RTAMD_LIB" not in os.environ:
        L.rt_build_info.restype = ctypes.c_char_p
        L.rt_build_info.argtypes = []
    L.rt_device_count.restype = i32
    L.rt_render_opts_default.argtypes = [vp]
    L.rt_render_opts_default.restype = None
    for name, args in {
        "rt_context_create": [i32, vp],
        "rt_context_destroy": [vp],
        "rt_context_set_stream": [vp, vp],
        "rt_context_synchronize": [vp],
        "rt_scene_create": [vp, vp, vp],
        "rt_scene_destroy": [vp],
        "rt_scene_set_area_light": [vp, vp],
        "rt_render": [vp, vp, vp, vp, vp, vp, vp, vp],
        "rt_render_device": [vp, vp, vp, vp, vp, vp, vp],
        "rt_render_batch": [vp, vp, vp, i32, vp, vp, vp, vp],
        "rt_render_multi": [vp, vp, i32, vp, vp, vp, vp, vp, vp],
        "rt_stats_read": [vp, vp],
        "rt_stats_reset": [vp],
        "rt_trace_rays": [vp, vp, vp, vp, ctypes.c_size_t, vp, vp],
        "rt_intersect_rays": [vp, vp, vp, ctypes.c_size_t, vp],
        "rt_tonemap": [vp, vp, ctypes.c_size_t, i32, vp],
        "rt_debug_f64_ops": [vp, vp, vp, ctypes.c_size_t, vp],
        "rt_debug_vec_ops": [vp, vp, ctypes.c_size_t, vp],
        "rt_comm_unique_id": [vp],
        "rt_comm_create": [vp, i32, i32, vp, vp],
        "rt_comm_create_ex": [vp, i32, i32, vp, ctypes.c_long, vp],
        "rt_comm_set_timeout": [vp, ctypes.c_long],
        "rt_comm_create_all": [vp, i32, vp],
        "rt_comm_create_local": [vp, i32, vp],
        "rt_comm_destroy": [vp],
        "rt_comm_info": [vp, vp, vp],
        "rt_comm_set_root_weight": [vp, i32],
        "rt_render_gather": [vp, vp, vp, vp, i32, vp, vp, vp],
        "rt_render_gather_all": [vp, vp, i32, vp, vp, i32, vp, vp, vp],
        "rt_render_gather_batch": [vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp],
        "rt_render_gather_all_batch": [vp, vp, i32, vp, i32, vp, i32, vp, vp, vp],
        "rt_comm_timing": [vp, vp, i32],
        "rt_comm_synchronize": [vp],
        "rt_queue_create": [vp, i32, vp],
        "rt_queue_destroy": [vp],
        "rt_queue_submit": [vp, vp, vp, vp, vp, vp, vp, vp],
        "rt_queue_wait": [vp, ctypes.c_uint64],
        "rt_queue_synchronize": [vp],
        "rt_debug_tile_order": [vp, vp, vp, vp, vp, ctypes.c_size_t, vp, vp, vp],
        "rt_debug_assemble_rows": [vp, vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_uint32, vp],
    }.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if "RTAMD_LIB" in os.environ:  # an older A/B build (tools/variants): dev use only
                continue
            raise
        fn.argtypes = args
        fn.restype = i32
    _lib = L
    return L


def build_info() -> dict:
    """The loaded library's build record (rt_build_info), plus `matches_tree`: whether its
    source_sha256 equals the digest of the sources in this tree (raytracingengine_amd/build.py
    source_digest) — False means the binary is stale against its sources."""
    import json
    info = json.loads(load_library().rt_build_info().decode())
    from . import build
    info["matches_tree"] = info.get("source_sha256") == build.source_digest()
    return info


def _check(status: int):
    if status != RT_OK:
        raise RtError(status, _lib.rt_last_error().decode(errors="replace"))


def rendered_rows(o: RenderOpts, height: int) -> int:
    """Rows a render call produces (rt_capi.h rt_render_opts: a row range, or block-cyclic row
    blocks when row_cycle > 1) — the height of the output buffers."""
    r1 = min(o.row_end, height) if o.row_end else height
    if r1 <= o.row_begin:
        return 0
    if o.row_cycle <= 1 or o.row_block == 0:
        return r1 - o.row_begin
    stride = o.row_block * o.row_cycle
    return sum(min(o.row_block, r1 - b) for b in range(o.row_begin, r1, stride))


def default_opts(**kw) -> RenderOpts:
    o = RenderOpts()
    load_library().rt_render_opts_default(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def device_count() -> int:
    return load_library().rt_device_count()


class Context:
    """One HIP device + stream (rt_context)."""

    def __init__(self, device: int = 0):
        L = load_library()
        self._h = ctypes.c_void_p()
        _check(L.rt_context_create(device, ctypes.byref(self._h)))
        self.device = device

    def close(self):
        if self._h:
            _lib.rt_context_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: int | None):
        _check(_lib.rt_context_set_stream(self._h, stream_ptr))

    def synchronize(self):
        _check(_lib.rt_context_synchronize(self._h))

    def scene(self, sc: SceneData) -> "DeviceScene":
        return DeviceScene(self, sc)

    def stats(self) -> Stats:
        s = Stats()
        _check(_lib.rt_stats_read(self._h, ctypes.byref(s)))
        return s

    def reset_stats(self):
        _check(_lib.rt_stats_reset(self._h))

    def tonemap(self, hdr: np.ndarray, op: int) -> np.ndarray:
        hdr = np.ascontiguousarray(hdr, np.float64).reshape(-1, 3)
        planes = 7 if op == TONEMAP_ALL else 1
        out = np.empty((planes, hdr.shape[0], 3), np.uint8)
        _check(_lib.rt_tonemap(self._h, hdr.ctypes.data, hdr.shape[0], op, out.ctypes.data))
        return out if planes > 1 else out[0]

    def debug_f64_ops(self, x: np.ndarray, y: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        out = np.empty((x.size, 5), np.float64)
        _check(_lib.rt_debug_f64_ops(self._h, x.ctypes.data, y.ctypes.data, x.size,
                                     out.ctypes.data))
        return out

    def debug_assemble_rows(self, gathered: np.ndarray, height: int, block: int, n: int,
                            max_rows: int) -> np.ndarray:
        """rank 0's assembly step alone: gathered uint8 [n, max_rows, row_bytes] -> image rows."""
        g = np.ascontiguousarray(gathered, np.uint8).reshape(n, max_rows, -1)
        out = np.empty((height, g.shape[2]), np.uint8)
        _check(_lib.rt_debug_assemble_rows(self._h, g.ctypes.data, g.shape[2], height, block, n,
                                           max_rows, out.ctypes.data))
        return out

    def debug_vec_ops(self, v: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(v, np.float64).reshape(-1, 3)
        out = np.empty((v.shape[0], 16), np.float64)
        _check(_lib.rt_debug_vec_ops(self._h, v.ctypes.data, v.shape[0], out.ctypes.data))
        return out


class DeviceScene:
    """A scene uploaded to HBM (rt_scene) plus the camera it is rendered with."""

    def __init__(self, ctx: Context, sc: SceneData):
        self.ctx = ctx
        self.data = sc
        self._arrays = (sc.sphere_array(), sc.plane_array(), sc.triangle_array(), sc.light_array())
        sp, pl, tr, lt = self._arrays
        desc = SceneDesc(sp.ctypes.data if len(sp) else None, len(sp),
                         pl.ctypes.data if len(pl) else None, len(pl),
                         tr.ctypes.data if len(tr) else None, len(tr),
                         lt.ctypes.data if len(lt) else None, len(lt))
        self._h = ctypes.c_void_p()
        _check(_lib.rt_scene_create(ctx.handle, ctypes.byref(desc), ctypes.byref(self._h)))
        self.camera = sc.camera.to_struct()
        self._area = None
        if sc.area_light is not None:
            self._area = sc.area_light.to_struct()
            _check(_lib.rt_scene_set_area_light(self._h, self._area.ctypes.data))

    def close(self):
        if self._h:
            _lib.rt_scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, *, hdr64=True, hdr32=False, tonemap: int = TONEMAP_NONE, opts=None,
               stats=False, **opt_kw):
        """Synchronous render into host arrays (rt_render).  Returns dict of outputs."""
        cam = self.data.camera
        o = opts if opts is not None else default_opts(tonemap=tonemap, **opt_kw)
        if opts is None:
            o.tonemap = tonemap
        rows = rendered_rows(o, cam.height)
        out = {}
        a64 = np.empty((rows, cam.width, 3), np.float64) if hdr64 else None
        a32 = np.empty((rows, cam.width, 3), np.float32) if hdr32 else None
        ldr = np.empty((rows, cam.width, 3), np.uint8) if tonemap != TONEMAP_NONE else None
        st = Stats()
        _check(_lib.rt_render(self.ctx.handle, self._h, self.camera.ctypes.data, ctypes.byref(o),
                              a64.ctypes.data if a64 is not None else None,
                              a32.ctypes.data if a32 is not None else None,
                              ldr.ctypes.data if ldr is not None else None,
                              ctypes.byref(st) if stats else None))
        if a64 is not None:
            out["hdr64"] = a64
        if a32 is not None:
            out["hdr32"] = a32
        if ldr is not None:
            out["ldr"] = ldr
        if stats:
            out["trace_rays"] = st.trace_rays
            out["shadow_rays"] = st.shadow_rays
        return out

    def render_host(self, h_hdr64: int | None, h_hdr32: int | None, h_ldr: int | None,
                    opts: RenderOpts, stats: bool = False):
        """Synchronous render into caller-owned HOST buffers (rt_render): the drop-in
        RenderImage() path, device-to-host copies included."""
        st = Stats()
        _check(_lib.rt_render(self.ctx.handle, self._h, self.camera.ctypes.data, ctypes.byref(opts),
                              h_hdr64, h_hdr32, h_ldr, ctypes.byref(st) if stats else None))
        return st if stats else None

    def trace_rays(self, rays: np.ndarray, stats=False, **opt_kw):
        """Batch TraceRay at depth 0 (rt_trace_rays): rays [n,6] -> rgb [n,3]."""
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        out = np.empty((rays.shape[0], 3), np.float64)
        o = default_opts(**opt_kw)
        st = Stats()
        _check(_lib.rt_trace_rays(self.ctx.handle, self._h, ctypes.byref(o), rays.ctypes.data,
                                  rays.shape[0], out.ctypes.data,
                                  ctypes.byref(st) if stats else None))
        return (out, st) if stats else out

    def intersect_rays(self, rays: np.ndarray) -> np.ndarray:
        """Batch IntersectClosest (rt_intersect_rays): rays [n,6] -> hits [n,9]."""
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        out = np.empty((rays.shape[0], 9), np.float64)
        _check(_lib.rt_intersect_rays(self.ctx.handle, self._h, rays.ctypes.data, rays.shape[0],
                                      out.ctypes.data))
        return out

    def debug_tile_order(self):
        """The packet kernel's tile-order state for this scene's camera (rt_debug_tile_order):
        (state, order[tiles] or None, cost[tiles, waves] or None)."""
        tiles, waves, state = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
        _check(_lib.rt_debug_tile_order(self.ctx.handle, self._h, self.camera.ctypes.data, None,
                                        None, 0, ctypes.byref(tiles), ctypes.byref(waves),
                                        ctypes.byref(state)))
        if state.value == 0:
            return 0, None, None
        n, w = tiles.value, waves.value
        order = np.empty(n, np.uint32)
        cost = np.empty(n * w, np.uint32)
        _check(_lib.rt_debug_tile_order(self.ctx.handle, self._h, self.camera.ctypes.data,
                                        order.ctypes.data if state.value == 2 else None,
                                        cost.ctypes.data, cost.size, ctypes.byref(tiles),
                                        ctypes.byref(waves), ctypes.byref(state)))
        return state.value, (order if state.value == 2 else None), cost.reshape(n, w)

    def render_device(self, d_hdr64: int | None, d_hdr32: int | None, d_ldr: int | None,
                      opts: RenderOpts):
        """Asynchronous render into device pointers (rt_render_device)."""
        _check(_lib.rt_render_device(self.ctx.handle, self._h, self.camera.ctypes.data,
                                     ctypes.byref(opts), d_hdr64, d_hdr32, d_ldr))

    def cameras(self, positions) -> np.ndarray:
        """rt_camera records of this scene's camera moved to each of `positions` ([n, 3])."""
        pos = np.asarray(positions, np.float64).reshape(-1, 3)
        cams = np.repeat(self.camera, len(pos))
        cams["position"] = pos
        return cams

    def render_batch(self, cams: np.ndarray, d_hdr64: int | None, d_hdr32: int | None,
                     d_ldr: int | None, opts: RenderOpts):
        """Asynchronous render of len(cams) frames into device buffers holding them back to
        back (rt_render_batch)."""
        cams = np.ascontiguousarray(cams)
        _check(_lib.rt_render_batch(self.ctx.handle, self._h, cams.ctypes.data, len(cams),
                                    ctypes.byref(opts), d_hdr64, d_hdr32, d_ldr))


def render_multi(scenes: list, *, hdr64=True, tonemap: int = TONEMAP_NONE, stats=False,
                 row_block: int = 0, **opt_kw) -> dict:
    """One frame over several contexts (rt_render_multi): `scenes` are DeviceScenes of the same
    SceneData, one per context; block-cyclic rows, assembled on the host."""
    L = load_library()
    n = len(scenes)
    cam = scenes[0].data.camera
    o = default_opts(tonemap=tonemap, row_block=row_block, **opt_kw)
    ctxs = (ctypes.c_void_p * n)(*[ds.ctx.handle for ds in scenes])
    scs = (ctypes.c_void_p * n)(*[ds._h for ds in scenes])
    a64 = np.empty((cam.height, cam.width, 3), np.float64) if hdr64 else None
    ldr = np.empty((cam.height, cam.width, 3), np.uint8) if tonemap != TONEMAP_NONE else None
    st = Stats()
    _check(L.rt_render_multi(ctxs, scs, n, scenes[0].camera.ctypes.data, ctypes.byref(o),
                             a64.ctypes.data if a64 is not None else None, None,
                             ldr.ctypes.data if ldr is not None else None,
                             ctypes.byref(st) if stats else None))
    out = {}
    if a64 is not None:
        out["hdr64"] = a64
    if ldr is not None:
        out["ldr"] = ldr
    if stats:
        out["trace_rays"], out["shadow_rays"] = st.trace_rays, st.shadow_rays
    return out


class _StdoutToStderr:
    """RCCL prints its version banner to stdout when a communicator is created; a bench's
    stdout carries exactly one JSON line, so the banner goes to stderr instead (fd level, C
    stdio flushed on both sides)."""

    def __enter__(self):
        import sys
        sys.stdout.flush()
        self._libc = ctypes.CDLL(None)
        self._libc.fflush(None)
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        self._libc.fflush(None)
        os.dup2(self._saved, 1)
        os.close(self._saved)


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (rt_comm_unique_id): made on one rank, handed to all of them."""
    buf = (ctypes.c_uint8 * RT_COMM_ID_BYTES)()
    _check(load_library().rt_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """One rank of a row-tiled multi-GPU frame (rt_comm): render this rank's rows, one RCCL
    gather to rank 0, assembled into rank 0's device framebuffers (rt_render_gather)."""

    def __init__(self, ctx: Context, nranks: int, rank: int, uid: bytes, _handle=None,
                 timeout_ms: int | None = None):
        """timeout_ms: the deadline of the communicator's waits (rt_comm_create_ex; None = the
        library default, RTAMD_COMM_TIMEOUT_MS or 300 s; 0 = none)."""
        L = load_library()
        self.ctx = ctx
        self.nranks, self.rank = nranks, rank
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
            return
        if len(uid) != RT_COMM_ID_BYTES:
            raise ValueError("unique id must be RT_COMM_ID_BYTES bytes")
        idbuf = (ctypes.c_uint8 * RT_COMM_ID_BYTES).from_buffer_copy(uid)
        with _StdoutToStderr():
            if timeout_ms is None:
                st = L.rt_comm_create(ctx.handle, nranks, rank, idbuf, ctypes.byref(self._h))
            else:
                st = L.rt_comm_create_ex(ctx.handle, nranks, rank, idbuf, int(timeout_ms),
                                         ctypes.byref(self._h))
        _check(st)

    @classmethod
    def create_all(cls, ctxs: list) -> list:
        """n communicators over n distinct devices from this process (rt_comm_create_all)."""
        n = len(ctxs)
        hs = (ctypes.c_void_p * n)(*[c.handle for c in ctxs])
        out = (ctypes.c_void_p * n)()
        with _StdoutToStderr():
            st = load_library().rt_comm_create_all(hs, n, out)
        _check(st)
        return [cls(c, n, i, b"", _handle=ctypes.c_void_p(out[i])) for i, c in enumerate(ctxs)]

    @classmethod
    def create_local(cls, ctxs: list) -> list:
        """n communicators over n contexts of this process that may share a GPU
        (rt_comm_create_local: the gather as device copies); driven by render_gather_all."""
        n = len(ctxs)
        hs = (ctypes.c_void_p * n)(*[c.handle for c in ctxs])
        out = (ctypes.c_void_p * n)()
        _check(load_library().rt_comm_create_local(hs, n, out))
        return [cls(c, n, i, b"", _handle=ctypes.c_void_p(out[i])) for i, c in enumerate(ctxs)]

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            _lib.rt_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render_gather(self, dscene: "DeviceScene", opts: RenderOpts, outputs: int,
                      d_hdr64: int | None = None, d_hdr32: int | None = None,
                      d_ldr: int | None = None):
        """Collective (every rank): enqueue this rank's rows + the gather (+ rank 0's
        assembly into the d_* device framebuffers) on the context's stream."""
        _check(_lib.rt_render_gather(self._h, dscene._h, dscene.camera.ctypes.data,
                                     ctypes.byref(opts), outputs, d_hdr64, d_hdr32, d_ldr))

    def render_gather_batch(self, dscene: "DeviceScene", cams: np.ndarray, opts: RenderOpts,
                            outputs: int, d_hdr64: int | None = None, d_hdr32: int | None = None,
                            d_ldr: int | None = None, rank_hdr64: int | None = None,
                            rank_hdr32: int | None = None, rank_ldr: int | None = None):
        """Collective: len(cams) frames, this rank's rows of each in one launch, one gather of
        the whole batch per output, rank 0 assembles (rt_render_gather_batch); rank_* receive
        outputs rendered but not gathered (this rank's rows, frames max_rows rows apart)."""
        cams = np.ascontiguousarray(cams)
        _check(_lib.rt_render_gather_batch(self._h, dscene._h, cams.ctypes.data, len(cams),
                                           ctypes.byref(opts), outputs, d_hdr64, d_hdr32, d_ldr,
                                           rank_hdr64, rank_hdr32, rank_ldr))

    def synchronize(self):
        _check(_lib.rt_comm_synchronize(self._h))

    def set_timeout(self, timeout_ms: int):
        _check(_lib.rt_comm_set_timeout(self._h, int(timeout_ms)))

    def set_root_weight(self, weight: int):
        """Weighted row split (rt_comm_set_root_weight): rank 0 renders `weight` of the
        weight + n − 1 row sets, every other rank one; the same value on every rank."""
        _check(_lib.rt_comm_set_root_weight(self._h, int(weight)))

    def timing(self, reset: bool = False) -> GatherTiming:
        t = GatherTiming()
        _check(_lib.rt_comm_timing(self._h, ctypes.byref(t), int(reset)))
        return t


class Queue:
    """Serving frame queue (rt_queue): frames of one context rendered into device framebuffers
    with `depth` of them in flight on as many HIP streams."""

    def __init__(self, ctx: Context, depth: int = 2):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        _check(load_library().rt_queue_create(ctx.handle, depth, ctypes.byref(self._h)))

    def submit(self, dscene: "DeviceScene", opts: RenderOpts, d_hdr64: int | None = None,
               d_hdr32: int | None = None, d_ldr: int | None = None) -> int:
        t = ctypes.c_uint64()
        _check(_lib.rt_queue_submit(self._h, dscene._h, dscene.camera.ctypes.data,
                                    ctypes.byref(opts), d_hdr64, d_hdr32, d_ldr, ctypes.byref(t)))
        return t.value

    def wait(self, ticket: int):
        _check(_lib.rt_queue_wait(self._h, ticket))

    def synchronize(self):
        _check(_lib.rt_queue_synchronize(self._h))

    def close(self):
        if self._h:
            _lib.rt_queue_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_gather_all(comms: list, scenes: list, opts: RenderOpts, outputs: int,
                      d_hdr64: int | None = None, d_hdr32: int | None = None,
                      d_ldr: int | None = None):
    """rt_render_gather_all: every rank of a Comm.create_all group from this process."""
    n = len(comms)
    cs = (ctypes.c_void_p * n)(*[c.handle for c in comms])
    ss = (ctypes.c_void_p * n)(*[s._h for s in scenes])
    _check(load_library().rt_render_gather_all(cs, ss, n, scenes[0].camera.ctypes.data,
                                               ctypes.byref(opts), outputs, d_hdr64, d_hdr32,
                                               d_ldr))


def render_gather_all_batch(comms: list, scenes: list, cams: np.ndarray, opts: RenderOpts,
                            outputs: int, d_hdr64: int | None = None, d_hdr32: int | None = None,
                            d_ldr: int | None = None):
    """rt_render_gather_all_batch: a batch of frames over every rank of a Comm.create_all /
    create_local group from this process."""
    n = len(comms)
    cs = (ctypes.c_void_p * n)(*[c.handle for c in comms])
    ss = (ctypes.c_void_p * n)(*[s._h for s in scenes])
    cams = np.ascontiguousarray(cams)
    _check(load_library().rt_render_gather_all_batch(cs, ss, n, cams.ctypes.data, len(cams),
                                                     ctypes.byref(opts), outputs, d_hdr64,
                                                     d_hdr32, d_ldr))
