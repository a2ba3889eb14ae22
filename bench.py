#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary+shadow) of the per-pixel trace at 1920×1080 (BASELINE
config 2: 16 spheres + 2 planes + 1 point light, Reinhard tonemap) on 1..N MI355X.

Contract (driver):  python bench.py --gpus N --steps K --warmup W
  * N=1 runs in-process; N>1 is launched by torch.distributed.run, one rank per GPU.
  * N=1 (mode "frames"): a step = one pass of the hot path over one frame — Scene::RenderImage()
    of the C2 frame into the float64 Vec3 framebuffer + the fused Reinhard tonemap to uint8
    (RaytracingEngine.cpp:133), everything resident in HBM (scene uploaded once, outputs stay
    on the device).
  * N>1 (mode "tiled", BASELINE config 4 / SURVEY §8e): a step = ONE 7680×4320 C4 frame split
    into block-cyclic row sets over the ranks, each rank renders its rows (fused Reinhard
    uint8), ONE RCCL gather (ncclGather over xGMI, behind the C-ABI: rt_render_gather) moves
    them to rank 0, and rank 0 assembles the frame in image order in its device framebuffer.
    Strong scaling; the per-rank render / gather / assembly times are in the line, and the
    weak-scaling C2 frames throughput is an extra field (`weak_frames`).
  * Untimed steps for --clock-warmup-ms (default 50 ms) of wall time so the GPU is at its
    sustained clock (it needs ~30 ms of load to leave idle: 143 → 45 µs per C2 frame,
    tools/clock_ramp.py), then W untimed steps, then exactly K timed steps bracketed by
    barrier + synchronize on both sides; the max over ranks is the time; rank 0 prints ONE
    JSON line.

Extra fields (N=1): `roofline` (HBM-write bound of the trace kernel from live per-launch HIP
events; traffic and VALU counters from the committed PMC summaries), `roofline_f32` (the same
launch with the north star's float3 framebuffer), `moving_camera` (a new camera position every
frame: no cached per-camera packet image), `d2h` (frames/s of the synchronous host-buffer
render, the drop-in RenderImage()'s path, pageable and pinned), `tiled_1gpu` (the N>1 default
workload on one GPU through the same gather path: the strong-scaling anchor), `pipelined` (the
same frames through the C-ABI serving queue rt_queue, 2 in flight), `cpu_baseline`
(the unmodified reference renderer, oracle/_ref, timed on this host's cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
HDR_BYTES = {"f64": 24, "f32": 12}
GATHER_OUT = {"u8": ("RT_OUT_LDR", 3), "f32": ("RT_OUT_HDR32", 12), "f64": ("RT_OUT_HDR64", 24)}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=None,
                    help="c1..c5 (BASELINE configs), mirror, glass, mesh; default c2 (frames), "
                         "c4 (tiled)")
    ap.add_argument("--mode", choices=["frames", "tiled"], default=None,
                    help="default: frames at N=1, tiled at N>1")
    ap.add_argument("--tonemap", default="reinhard_simple",
                    help="fused LDR operator, or 'none' (HDR only)")
    ap.add_argument("--row-block", type=int, default=16,
                    help="tiled mode: rows per block of the block-cyclic split")
    ap.add_argument("--gather", choices=sorted(GATHER_OUT), default="u8",
                    help="tiled mode: the framebuffer each rank renders and rank 0 gathers")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="tiled mode: gather on the render stream (no overlap of frame k's "
                         "gather with frame k+1's render)")
    ap.add_argument("--hdr", choices=["f64", "f32"], default="f64",
                    help="frames mode HDR framebuffer: f64 = the reference's std::vector<Vec3>")
    ap.add_argument("--clock-warmup-ms", type=float, default=50.0,
                    help="untimed steps for this much wall time before the W warmup steps, so "
                         "that the K timed steps run at the GPU's sustained clock")
    ap.add_argument("--event-every", type=int, default=10,
                    help="bracket every n-th timed step with HIP events (0: none)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="> 1: also measure the frames with this many in flight through the "
                         "C-ABI serving queue, rt_queue ('pipelined' field; N=1 extras)")
    ap.add_argument("--no-extras", action="store_true",
                    help="headline only (no f32 / moving-camera / D2H / tiled / weak fields)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=6,
                    help="reference frames timed for cpu_baseline (first one is warm-up)")
    return ap.parse_args(argv)


def load_profile(name: str):
    path = os.path.join(HERE, "profiles", name)
    if not os.path.exists(path):
        return None, None
    with open(path) as fh:
        return json.load(fh), os.path.relpath(path, HERE)


def granted_cores() -> int:
    """Cores this process may run on: the affinity mask, capped by OMP_NUM_THREADS when the
    environment sets one (the GPU box grants a 16-core share of a larger machine)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def cpu_baseline(sc, rays_per_frame: int, frames: int):
    """The reference CPU loop on this host: oracle/_ref/ref_harness (unmodified reference
    Scene::RenderImage, OpenMP on the granted cores, threads bound one per core), median of
    frames-1 after one warm-up, and one frame on one thread.  Falls back to the C restatement
    (kind "port") when the reference build is absent."""
    from oracle import pyoracle as po
    threads = granted_cores()
    ref = po.ref_available()

    def run(nthreads, repeat):
        if ref:
            _, ms, used = po.ref_render(sc, repeat=repeat, threads=nthreads, want_image=False,
                                        bind=True)
            return ms, used
        ms = []
        for _ in range(repeat):
            t0 = time.perf_counter()
            po.render(sc, nthreads=nthreads)
            ms.append((time.perf_counter() - t0) * 1e3)
        return ms, nthreads

    ms, used = run(threads, frames)
    timed = sorted(ms[1:] if len(ms) > 1 else ms)
    med = timed[len(timed) // 2]
    ms1, _ = run(1, 1)
    single = {"value": rays_per_frame / (ms1[0] / 1e3) / 1e6, "cores": 1, "ms_per_frame": ms1[0]}
    multi = {"value": rays_per_frame / (med / 1e3) / 1e6, "cores": used, "ms_per_frame": med}
    # The reference's chunk-1 dynamic OpenMP loop (Scene.h:318) can run slower on many threads
    # than on one; the baseline is the faster of the two runs, both are in the line.
    best = multi if multi["value"] >= single["value"] else single
    return {
        "value": best["value"],
        "unit": "Mrays/s",
        "cores": best["cores"],
        "kind": "reference" if ref else "port",
        "sample": f"{len(ms)} full {sc.camera.width}x{sc.camera.height} frames of config "
                  f"{sc.name} on {used} threads bound to cores (Scene::RenderImage only, first "
                  f"frame warm-up; median {med:.1f} ms/frame) and one frame on 1 thread "
                  f"({ms1[0]:.1f} ms); value = the faster",
        "ms_per_frame": best["ms_per_frame"],
        "all_threads": multi,
        "single_core": single,
    }


class Runner:
    """Per-process state: the rank, a torch stream the library launches on, timing helpers."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus and self.world > 1:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={self.world}")
        torch.cuda.set_device(self.local_rank)
        if self.world > 1:
            dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank))
        from raytracingengine_amd import capi
        self.capi = capi
        self.ctx = capi.Context(self.local_rank)
        self.stream = torch.cuda.Stream()
        self.ctx.set_stream(self.stream.cuda_stream)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, *vals):
        if self.world == 1:
            return vals
        t = self.torch.tensor(vals, dtype=self.torch.float64, device="cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return tuple(float(x) for x in t)

    def sum_over_ranks(self, *vals):
        if self.world == 1:
            return vals
        t = self.torch.tensor(vals, dtype=self.torch.float64, device="cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return tuple(float(x) for x in t)

    def gather_rows(self, vals):
        """Every rank's list of floats, on every rank ([world][len])."""
        if self.world == 1:
            return [list(vals)]
        t = self.torch.tensor(vals, dtype=self.torch.float64, device="cuda")
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [[float(x) for x in o] for o in out]

    def timed(self, step, steps, warmup, region_events=True, warm_step=None):
        """Untimed steps for `--clock-warmup-ms` of wall time (the GPU leaves its idle clock
        only after ~30 ms of sustained load: tools/clock_ramp.py, C2 143 → 54 → 45 µs/frame
        over the first 30 ms), then W untimed steps, then K timed steps between barrier +
        synchronize; returns (elapsed seconds max over ranks, HIP-event region ms per step on
        the launch stream).  `warm_step` (default `step`) is what the clock warm-up runs: it
        must not be a collective, since each rank warms up for its own wall time."""
        torch = self.torch
        warm = warm_step or step
        t_end = time.perf_counter() + self.args.clock_warmup_ms / 1e3
        k = 0
        while time.perf_counter() < t_end:
            for _ in range(16):
                warm(-1000000 - k, False)
                k += 1
            torch.cuda.synchronize()
        for i in range(warmup):
            step(i, False)
        # drain this rank's work (its RCCL gathers included) before the process group's own
        # collective: two communicators' kernels are never in flight together
        torch.cuda.synchronize()
        self.barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(self.stream)   # on the stream the trace kernel is launched on
        for i in range(steps):
            step(i, True)
        ev1.record(self.stream)
        torch.cuda.synchronize()
        self.barrier()
        elapsed = time.perf_counter() - t0
        region_ms = ev0.elapsed_time(ev1) / steps if region_events else None
        (elapsed,) = self.max_over_ranks(elapsed)
        return elapsed, region_ms

    def count_rays(self, dscene, opts):
        """Rays of one render with these options (separate counting launch, never timed)."""
        capi = self.capi
        o = capi.default_opts()
        for f, _ in capi.RenderOpts._fields_:
            setattr(o, f, getattr(opts, f))
        o.flags = capi.RT_FLAG_COUNT_RAYS
        o.tonemap = -1
        rows = capi.rendered_rows(o, dscene.data.camera.height)
        W = dscene.data.camera.width
        buf = self.torch.empty(max(rows, 1) * W * 3, dtype=self.torch.float32, device="cuda")
        with self.torch.cuda.stream(self.stream):
            self.ctx.reset_stats()
            if rows:
                dscene.render_device(None, buf.data_ptr(), None, o)
            st = self.ctx.stats()
            self.ctx.reset_stats()
        return st.trace_rays + st.shadow_rays


# ------------------------------------------------------------------------------ frames mode
def frames_mode(R: Runner, sc, steps, warmup, hdr="f64", tonemap=1, event_every=10,
                camera_step=None):
    """Every rank renders whole frames (weak scaling).  camera_step(i) -> new camera position
    per frame (moving camera), else a static camera."""
    torch, capi = R.torch, R.capi
    W, H = sc.camera.width, sc.camera.height
    dscene = R.ctx.scene(sc)
    hdr_t = torch.empty(H * W * 3, dtype=torch.float64 if hdr == "f64" else torch.float32,
                        device="cuda")
    ldr = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda") if tonemap >= 0 else None
    hargs = (hdr_t.data_ptr(), None) if hdr == "f64" else (None, hdr_t.data_ptr())
    opts = capi.default_opts(tonemap=tonemap)
    timed_opts = capi.default_opts(tonemap=tonemap, flags=capi.RT_FLAG_TIME_KERNEL)
    rays = R.count_rays(dscene, opts)
    base = dscene.camera["position"][0].copy()

    def step(i, timed):
        if camera_step is not None:
            dscene.camera["position"][0] = camera_step(base, i if timed else -1 - i)
        ev = timed and event_every > 0 and i % event_every == 0
        dscene.render_device(*hargs, ldr.data_ptr() if ldr is not None else None,
                             timed_opts if ev else opts)

    R.ctx.reset_stats()
    elapsed, region_ms = R.timed(step, steps, warmup)
    kst = R.ctx.stats()
    dscene.camera["position"][0] = base
    dscene.close()
    sampled_ms = kst.kernel_ms / kst.launches if kst.launches else None
    return {"rays": rays, "elapsed": elapsed, "region_ms": region_ms, "sampled_ms": sampled_ms,
            "px": W * H, "bufs": (hdr_t, ldr)}


def pipelined_frames(R: Runner, sc, steps, warmup, inflight, tonemap=1):
    """The same K frames through the C-ABI serving queue (rt_queue): `inflight` frames in flight
    on as many HIP streams, each with its own framebuffers — one frame's launch tail overlaps the
    next frame's start."""
    torch, capi = R.torch, R.capi
    W, H = sc.camera.width, sc.camera.height
    dscene = R.ctx.scene(sc)
    q = capi.Queue(R.ctx, inflight)
    bufs = [(torch.empty(H * W * 3, dtype=torch.float64, device="cuda"),
             torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")) for _ in range(inflight)]
    opts = capi.default_opts(tonemap=tonemap)

    def step(i, timed):
        # frame i goes to slot i mod depth: the queue's stream order keeps a slot's frames in
        # order, so its framebuffers are rewritten only after the previous frame wrote them (a
        # consumer would rt_queue_wait(ticket) before reading; nothing here reads them)
        h, l = bufs[i % inflight]
        q.submit(dscene, opts, h.data_ptr(), None, l.data_ptr())

    elapsed, _ = R.timed(step, steps, warmup, region_events=False)
    q.synchronize()
    q.close()
    dscene.close()
    return elapsed


def d2h_frames(R: Runner, sc, frames=20, tonemap=1):
    """The drop-in RenderImage() path: synchronous rt_render into HOST framebuffers (float64
    Vec3 + the fused bytes), frames/s including the device-to-host copies — into pageable
    numpy arrays (a std::vector) and into pinned memory."""
    import numpy as np
    torch, capi = R.torch, R.capi
    W, H = sc.camera.width, sc.camera.height
    dscene = R.ctx.scene(sc)
    out = {}
    pageable = (np.empty((H, W, 3), np.float64), np.empty((H, W, 3), np.uint8))
    pinned = (torch.empty((H, W, 3), dtype=torch.float64).pin_memory(),
              torch.empty((H, W, 3), dtype=torch.uint8).pin_memory())
    o = capi.default_opts(tonemap=tonemap)
    for kind, (a64, a8) in (("pageable", pageable), ("pinned", pinned)):
        p64 = a64.ctypes.data if kind == "pageable" else a64.data_ptr()
        p8 = a8.ctypes.data if kind == "pageable" else a8.data_ptr()
        for _ in range(3):
            dscene.render_host(p64, None, p8, o)
        t0 = time.perf_counter()
        for _ in range(frames):
            dscene.render_host(p64, None, p8, o)
        dt = (time.perf_counter() - t0) / frames
        out[kind] = {"frames_per_sec": round(1.0 / dt, 2), "ms_per_frame": round(dt * 1e3, 4)}
    dscene.close()
    out["bytes_per_frame"] = W * H * 27
    out["note"] = ("rt_render (synchronous): render + D2H of the float64 Vec3 framebuffer and "
                   "the Reinhard bytes into host memory, as the drop-in Scene::RenderImage()")
    return out


# ------------------------------------------------------------------------------ tiled mode
def tiled_mode(R: Runner, sc, steps, warmup, gather="u8", tonemap=1, block=16,
               event_every=10, pipeline=True):
    """One frame split over the ranks: block-cyclic rows, one RCCL gather to rank 0, rank 0
    assembles the frame in image order (rt_render_gather).  Returns per-rank timings."""
    torch, capi = R.torch, R.capi
    W, H = sc.camera.width, sc.camera.height
    if R.world > 1:
        uid = [capi.comm_unique_id() if R.rank == 0 else None]
        R.dist.broadcast_object_list(uid, src=0)
        uid = uid[0]
    else:
        uid = capi.comm_unique_id()
    comm = capi.Comm(R.ctx, R.world, R.rank, uid)
    dscene = R.ctx.scene(sc)
    out_name, bpp = GATHER_OUT[gather]
    outputs = getattr(capi, out_name)
    dtype = {"u8": torch.uint8, "f32": torch.float32, "f64": torch.float64}[gather]
    frame = torch.empty(H * W * 3 if R.rank == 0 else 1, dtype=dtype, device="cuda")
    ptrs = [None, None, None]
    if R.rank == 0:
        ptrs[{"f64": 0, "f32": 1, "u8": 2}[gather]] = frame.data_ptr()
    tm = tonemap if gather == "u8" else -1
    pf = capi.RT_FLAG_PIPELINE if pipeline else 0
    opts = capi.default_opts(tonemap=tm, row_block=block, flags=pf)
    timed_opts = capi.default_opts(tonemap=tm, row_block=block,
                                   flags=pf | capi.RT_FLAG_TIME_KERNEL)
    # this rank's rays: its rows of the frame (the gather's plan)
    plan = capi.default_opts(tonemap=-1)
    if R.world > 1:
        plan.row_begin, plan.row_end = R.rank * block, H
        plan.row_block, plan.row_cycle = block, R.world
    rays_rank = R.count_rays(dscene, plan) if plan.row_begin < H else 0

    def step(i, timed):
        ev = timed and event_every > 0 and i % event_every == 0
        comm.render_gather(dscene, timed_opts if ev else opts, outputs, *ptrs)

    # the clock warm-up renders this rank's rows without the gather (no collective)
    wopts = capi.default_opts(tonemap=tm)
    for f, _ in capi.RenderOpts._fields_:
        if f.startswith("row_"):
            setattr(wopts, f, getattr(plan, f))
    wrows = capi.rendered_rows(wopts, H) if wopts.row_begin < H else 0
    wbuf = torch.empty(max(wrows, 1) * W * bpp, dtype=torch.uint8, device="cuda")
    wptrs = [None, None, None]
    wptrs[{"f64": 0, "f32": 1, "u8": 2}[gather]] = wbuf.data_ptr()

    def warm_step(i, timed):
        if wrows:
            dscene.render_device(*wptrs, wopts)

    comm.timing(reset=True)
    elapsed, _ = R.timed(step, steps, warmup, region_events=False, warm_step=warm_step)
    t = comm.timing(reset=True)
    per = [t.render_ms / max(t.frames, 1), t.gather_ms / max(t.frames, 1),
           t.assemble_ms / max(t.frames, 1), float(t.rows), float(rays_rank)]
    ranks = R.gather_rows(per)
    (rays_all,) = R.sum_over_ranks(float(rays_rank))
    dscene.close()
    comm.close()
    return {"elapsed": elapsed, "rays": rays_all, "ranks": ranks, "px": W * H, "bpp": bpp,
            "max_rows": t.max_rows, "pipeline": pipeline}


def tiled_summary(res, steps, W, gather, block):
    ranks = res["ranks"]
    render = [r[0] for r in ranks]
    mean_render = sum(render) / len(render)
    return {
        "per_rank": [{"rank": i, "rows": int(r[3]), "rays": int(r[4]), "render_ms": round(r[0], 5),
                      "gather_ms": round(r[1], 5), "assemble_ms": round(r[2], 5)}
                     for i, r in enumerate(ranks)],
        "render_ms_max": round(max(render), 5),
        "render_imbalance": round(max(render) / mean_render, 4) if mean_render > 0 else None,
        "gather_bytes_per_rank": res["max_rows"] * W * res["bpp"],
        "gathered": gather,
        "row_block": block,
        "pipelined": res["pipeline"],
        "ms_per_frame": round(res["elapsed"] / steps * 1e3, 5),
        "value": round(res["rays"] * steps / res["elapsed"] / 1e6, 3),
    }


# ------------------------------------------------------------------------------ main
def main(argv=None):
    args = parse_args(argv)
    R = Runner(args)
    capi = R.capi
    from raytracingengine_amd.configs import make_config

    mode = args.mode or ("frames" if R.world == 1 else "tiled")
    config = args.config or ("c2" if mode == "frames" else "c4")
    tonemap = -1 if args.tonemap == "none" else capi.TONEMAPS.index(args.tonemap)
    sc = make_config(config, aa=1)
    W, H = sc.camera.width, sc.camera.height
    line = None
    extras = not args.no_extras

    if mode == "frames":
        res = frames_mode(R, sc, args.steps, args.warmup, args.hdr, tonemap, args.event_every)
        elapsed, rays_rank = res["elapsed"], res["rays"]
        (kernel_ms,) = R.max_over_ranks(res["region_ms"])
        (rays_all,) = R.sum_over_ranks(float(rays_rank))
        value = rays_all * args.steps / elapsed / 1e6
        frames = R.world * args.steps
        bytes_per_launch = res["px"] * (HDR_BYTES[args.hdr] + (3 if tonemap >= 0 else 0))
        achieved = bytes_per_launch / (kernel_ms / 1e3) / 1e9
        traffic, traffic_src = load_profile(f"pmc_{config}_frames.json")
        valu, valu_src = load_profile(f"r03_{config}_valu.json")
        line = {
            "metric": "Mrays/sec (primary+shadow) at 1920x1080" if config == "c2"
                      else f"Mrays/sec (primary+shadow), config {config}",
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": R.world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{config}: {W}x{H}, {len(sc.spheres)} spheres, {len(sc.planes)} "
                            f"planes, {len(sc.lights)} point lights, AA=1, {args.hdr} Vec3 HDR "
                            f"framebuffer + fused {args.tonemap} u8, static camera",
                "global_batch": frames, "resolution": [W, H],
                "parallelism": f"frames x{R.world}", "rays_per_frame": rays_rank,
            },
            "frames_per_sec": round(frames / elapsed, 3),
            "clock_warmup_ms": args.clock_warmup_ms,
            "kernel_ms_per_launch": round(kernel_ms, 6),
            "kernel_ms_sampled_events": round(res["sampled_ms"], 6) if res["sampled_ms"] else None,
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                "alg_bytes_per_launch": bytes_per_launch, "traffic_source": traffic_src,
            },
            "valu": valu, "valu_source": valu_src,
            "cpu_baseline": None,
        }
        if extras and R.world == 1:
            steps_x = min(args.steps, 100)
            # the north star's float3 framebuffer (+ u8): 15 B/px instead of 27
            f32 = frames_mode(R, sc, steps_x, args.warmup, "f32", tonemap, 0)
            b32 = f32["px"] * (12 + (3 if tonemap >= 0 else 0))
            a32 = b32 / (f32["region_ms"] / 1e3) / 1e9
            line["roofline_f32"] = {
                "achieved": round(a32, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(a32 / HBM_PEAK_GBS, 5), "alg_bytes_per_launch": b32,
                "kernel_ms_per_launch": round(f32["region_ms"], 6),
                "value": round(f32["rays"] * steps_x / f32["elapsed"] / 1e6, 3)}
            # a camera that moves every frame: never the cached per-camera packet image
            mv = frames_mode(R, sc, steps_x, args.warmup, args.hdr, tonemap, 0,
                             camera_step=lambda base, i: base + (i * 1e-7, 0.0, 0.0))
            line["moving_camera"] = {
                "ms_per_step": round(mv["elapsed"] / steps_x * 1e3, 5),
                "kernel_ms_per_launch": round(mv["region_ms"], 6),
                "value": round(mv["rays"] * steps_x / mv["elapsed"] / 1e6, 3),
                "note": "camera x moved by 1e-7 every frame: the per-camera packet image is "
                        "never reused (each launch's first workgroup forms it and hands it to "
                        "the later ones, DESIGN §4); rays counted at the first position"}
            if args.inflight > 1:
                el = pipelined_frames(R, sc, steps_x, args.warmup, args.inflight, tonemap)
                line["pipelined"] = {
                    "inflight": args.inflight,
                    "value": round(rays_rank * steps_x / el / 1e6, 3),
                    "ms_per_step": round(el / steps_x * 1e3, 5),
                    "note": "the same frames through the C-ABI serving queue (rt_queue), "
                            "several in flight on separate HIP streams; serving throughput, "
                            "not the headline value"}
            # BASELINE config 1: the reference main()'s own scene and sampling
            sc1 = make_config("c1", aa=32)
            c1 = frames_mode(R, sc1, 10, 2, "f64", R.capi.TONEMAPS.index("aces"), 0)
            line["reference_main_c1"] = {
                "workload": "c1: the reference main() box (5 mirrored axis planes, 2 point "
                            "lights), 1000x1000, AA=32, f64 Vec3 HDR + fused ACES u8",
                "ms_per_frame": round(c1["elapsed"] / 10 * 1e3, 4),
                "kernel_ms_per_launch": round(c1["region_ms"], 4),
                "rays_per_frame": c1["rays"],
                "value": round(c1["rays"] * 10 / c1["elapsed"] / 1e6, 3), "unit": "Mrays/s"}
            line["d2h"] = d2h_frames(R, sc, min(args.steps, 20), tonemap)
            # the N>1 default workload (C4 tiled + RCCL gather) on this one GPU
            sc4 = make_config("c4", aa=1)
            t1 = tiled_mode(R, sc4, min(args.steps, 20), min(args.warmup, 3), "u8", 1,
                            args.row_block, 1, not args.no_pipeline)
            line["tiled_1gpu"] = tiled_summary(t1, min(args.steps, 20), sc4.camera.width, "u8",
                                               args.row_block)
            line["tiled_1gpu"]["workload"] = ("c4 7680x4320, 256 spheres, 8 lights, Reinhard "
                                              "u8 through rt_render_gather on 1 rank")
        if R.world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(sc, rays_rank, args.cpu_frames)
            except Exception as e:  # a reported baseline, never the product path
                line["cpu_baseline"] = {"error": repr(e)}
    else:
        res = tiled_mode(R, sc, args.steps, args.warmup, args.gather, tonemap, args.row_block,
                         args.event_every, not args.no_pipeline)
        summ = tiled_summary(res, args.steps, W, args.gather, args.row_block)
        elapsed = res["elapsed"]
        value = res["rays"] * args.steps / elapsed / 1e6
        r0 = res["ranks"][0]
        bytes_rank0 = int(r0[3]) * W * res["bpp"]
        achieved = bytes_rank0 / (r0[0] / 1e3) / 1e9 if r0[0] > 0 else 0.0
        line = {
            "metric": "Mrays/sec (primary+shadow), row-tiled frame + RCCL gather",
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": R.world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{config}: {W}x{H}, {len(sc.spheres)} spheres, {len(sc.planes)} "
                            f"planes, {len(sc.lights)} point lights, AA=1, one frame per step "
                            f"split over {R.world} GPUs, fused {args.tonemap} {args.gather} "
                            f"gathered to rank 0",
                "global_batch": args.steps, "resolution": [W, H],
                "parallelism": f"block-cyclic rows ({args.row_block}-row blocks) x{R.world} + "
                               f"one ncclGather per frame",
                "rays_per_frame": res["rays"],
            },
            "frames_per_sec": round(args.steps / elapsed, 3),
            "clock_warmup_ms": args.clock_warmup_ms,
            "tiled": summ,
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "alg_bytes_per_launch": bytes_rank0,
                "note": "rank 0's render launch: its rows' framebuffer bytes / render time",
            },
            "cpu_baseline": None,
        }
        if extras:
            sc2 = make_config("c2", aa=1)
            wk = frames_mode(R, sc2, args.steps, args.warmup, "f64", tonemap, 0)
            (rays2,) = R.sum_over_ranks(float(wk["rays"]))
            line["weak_frames"] = {
                "value": round(rays2 * args.steps / wk["elapsed"] / 1e6, 3),
                "ms_per_step": round(wk["elapsed"] / args.steps * 1e3, 5),
                "workload": "c2 1920x1080 frames, every rank its own (f64 Vec3 + Reinhard u8)",
                "scaling": "weak"}
    if R.rank == 0:
        print(json.dumps(line), flush=True)
    R.ctx.close()
    if R.world > 1:
        R.dist.destroy_process_group()


if __name__ == "__main__":
    main()
