#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary+shadow) of the per-pixel trace at 1920×1080 (BASELINE
config 2: 16 spheres + 2 planes + 1 point light, Reinhard tonemap) on 1, 2, 4 or 8 MI355X.

Contract (driver):  python bench.py --gpus N --steps K --warmup W
  * N=1 runs in-process; N>1 is launched by torch.distributed.run, one rank per GPU.
  * The SAME workload and code path at every N (RE/Scene.h:318-325): a step = one
    C2 frame — Scene::RenderImage() into the float64 Vec3 framebuffer + the fused Reinhard bytes
    (RaytracingEngine.cpp:133), everything resident in HBM — split into block-cyclic 8-row
    blocks over the N ranks.  Every rank renders its rows (f64 HDR rows kept on the rank, the
    bytes into its send buffer), ONE ncclGather per batch moves the bytes to rank 0 over xGMI,
    and rank 0 writes them into image order (rt_render_gather_batch).  At N=1 the one rank's
    rows are the frame: it renders straight into the frame buffers, nothing to gather.
  * Frames go in batches of --batch per call: one render launch per batch (one grid plane per
    frame, so a small per-rank share of a frame does not pay a whole launch's ramp and drain),
    one ncclGather and one assembly launch per batch; two batches in flight (RT_FLAG_PIPELINE:
    batch b's gather overlaps batch b+1's render).  Default: 32 at N=1; at N>1 the K timed
    frames go in at least 4 batches (ceil(K/4), 4..32: 5 for K=20) so that gathers overlap
    renders inside the region (default_batch).
  * Untimed frames for --clock-warmup-ms (default 50 ms) of wall time so the GPU is at its
    sustained clock (it needs ~30 ms of load to leave idle: 143 → 45 µs per C2 frame,
    tools/clock_ramp.py), then W untimed frames, then exactly K timed frames bracketed by
    barrier + synchronize on both sides (each rank's clock runs from the opening barrier to its
    own closing synchronize); the max over ranks is the time; rank 0 prints ONE JSON line.
  * `--gpus N` > 1 without an outer launcher (no WORLD_SIZE): the N ranks are started here, as
    ONE `torch.distributed.run` child before any GPU call; this process exits with its status.
  * After the timed region the line's `parity` certifies the timed path's output (the assembled
    frame's Reinhard bytes against the reference's SHA-256, every rank's f64 rows against a
    one-launch render); a failed check exits 3.

Extra fields (each outside the headline's timed region, with its own timing): `per_rank`
(render / gather / assembly per frame on every rank), `roofline` (HBM-write bound of the trace
kernel from live per-launch HIP events; traffic and VALU counters from the committed PMC
summaries), `single_launch` (one launch per frame, the round-3 headline path), `weak_frames`
(every rank its own whole frames), `c4_tiled` (BASELINE config 4: the 7680×4320 frame through
the same path), and at N=1 `roofline_f32` (the north star's float3 framebuffer),
`moving_camera` (a new camera position every frame), `d2h` (the drop-in RenderImage() with
its device-to-host copy), `reference_main_c1` (BASELINE config 1 as the reference main()
renders it) and `cpu_baseline` (the unmodified reference renderer, oracle/_ref, on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
FP64_VALU_PEAK_TF = 78.6  # FP64 vector FMA-counted peak (1024 SIMDs x 2.4 GHz x 32)
HDR_BYTES = {"f64": 24, "f32": 12}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256,
                    help="timed frames (default: 8 full batches of 32)")
    ap.add_argument("--warmup", type=int, default=32, help="untimed frames after the clock warm-up")
    ap.add_argument("--config", default="c2",
                    help="c1..c5 (BASELINE configs), mirror, glass, mesh, bigmesh; default c2")
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per rt_render_gather_batch call (up to 32 per launch; default "
                         "32 at N=1, ceil(steps/4) clamped to 4..32 at N>1: default_batch)")
    ap.add_argument("--tonemap", default="reinhard_simple",
                    help="fused LDR operator (the gathered bytes)")
    ap.add_argument("--row-block", type=int, default=8,
                    help="rows per block of the block-cyclic split (N>1); 8 = one packet-kernel "
                         "wave row: at 8 ranks of 1080 rows, 16-row blocks give the slowest "
                         "rank 144 rows against a mean of 135 (and pad every rank's gather to "
                         "144), 8-row blocks 136 (profiles/r06_inflight_block8.txt)")
    ap.add_argument("--hdr", choices=["f64", "f32"], default="f64",
                    help="the rank-local HDR framebuffer: f64 = the reference's std::vector<Vec3>")
    ap.add_argument("--root-weight", default="1",
                    help="N>1: rank 0's share of the row split (rt_comm_set_root_weight): an "
                         "integer (default 1: the equal split), or 'auto' = chosen from an "
                         "untimed equal-split probe of the ranks' render and gather times (opt-in: "
                         "the weighted P2P path has not run on a multi-GPU node yet, DESIGN §6)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="gather on the render stream (no overlap of batch b's gather with "
                         "batch b+1's render)")
    ap.add_argument("--clock-warmup-ms", type=float, default=50.0,
                    help="untimed frames for this much wall time before the W warmup frames, so "
                         "that the K timed frames run at the GPU's sustained clock")
    ap.add_argument("--event-every", type=int, default=None,
                    help="bracket every n-th timed batch with per-batch HIP events (render / "
                         "gather / assembly per rank); 0: none — the kernel time then comes from "
                         "the HIP events on the launch stream around the whole timed region.  "
                         "Default: 0 at N=1 (in-region event records cost ~30 us of a 20-frame "
                         "region, tools/host_overhead.py), 4 at N>1")
    ap.add_argument("--no-extras", action="store_true",
                    help="headline only (no extra fields)")
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


def launcher_command(args_list, gpus: int, port: int):
    """The one child that runs `--gpus N > 1` when no outer launcher set WORLD_SIZE: N ranks of
    this same script under torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1), with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__), *args_list]


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """`python bench.py --gpus N` (N > 1) run plainly: start the N ranks as ONE child process
    (torch.distributed.run), before this process makes any GPU call and without exec — rank 0's
    JSON line reaches the same stdout — and return the child's exit status.  Under an outer
    launcher (WORLD_SIZE set) nothing is started.  RE/Scene.h:318-325 is the loop the ranks
    split."""
    import subprocess
    cmd = launcher_command(list(sys.argv[1:] if argv is None else argv), args.gpus, free_port())
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def needs_launcher(args, environ=None) -> bool:
    env = os.environ if environ is None else environ
    return args.gpus > 1 and "WORLD_SIZE" not in env


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
    """Per-process state: the rank, a torch stream the library launches on, the rank's
    communicator (a one-rank RCCL communicator at N=1), timing helpers."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={self.world}")
        torch.cuda.set_device(self.local_rank)
        if self.world > 1:
            dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank))
        from raytracingengine_amd import capi
        self.capi = capi
        self.ctx = capi.Context(self.local_rank)
        self.stream = torch.cuda.Stream()
        self.ctx.set_stream(self.stream.cuda_stream)
        if self.world > 1:
            uid = [capi.comm_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            uid = uid[0]
        else:
            uid = capi.comm_unique_id()
        self.comm = capi.Comm(self.ctx, self.world, self.rank, uid)

    def solo_comm(self):
        """A one-rank communicator on this GPU (every rank its own whole frames)."""
        if self.world == 1:
            return self.comm
        if not hasattr(self, "_solo"):
            self._solo = self.capi.Comm(self.ctx, 1, 0, self.capi.comm_unique_id())
        return self._solo

    def close(self):
        if hasattr(self, "_solo"):
            self._solo.close()
        self.comm.close()
        self.ctx.close()
        if self.world > 1:
            self.dist.destroy_process_group()

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

    def timed(self, step, frames, warmup, batch, warm_step=None, region_events=False,
              sync=None, prime=None):
        """Untimed work for `--clock-warmup-ms` of wall time (the GPU leaves its idle clock only
        after ~30 ms of sustained load: tools/clock_ramp.py, C2 143 → 54 → 45 µs/frame over the
        first 30 ms), then `warmup` untimed frames, then `frames` timed frames between barrier +
        synchronize.  step(first_frame, nframes, timed) enqueues nframes frames (≤ batch).
        Returns (elapsed seconds max over ranks, HIP-event region ms on the launch stream).
        `warm_step` (default `step`) is what the clock warm-up runs: it must not be a
        collective, since each rank warms up for its own wall time.  Frame indices (what a
        moving camera derives its position from) run on across the phases: the warmup has
        [0, warmup), the timed frames [warmup, warmup + frames), so no timed frame revisits a
        warmup position.  `sync` (the communicator's deadline-guarded wait) runs before the
        device synchronisation that closes the timed region.  `prime` (the split's first
        collective call: RCCL sets up its peer connections there) runs once on every rank after
        the clock warm-up, so that even --warmup 0 keeps the setup out of the timed region."""
        torch = self.torch
        warm = warm_step or step
        t_end = time.perf_counter() + self.args.clock_warmup_ms / 1e3
        k = 0
        while time.perf_counter() < t_end:
            for _ in range(4):
                warm(-1000000 - k, batch, False)
                k += batch
            torch.cuda.synchronize()
        if prime is not None:
            prime()
            torch.cuda.synchronize()

        def run(n, timed, first=0):
            for f0 in range(0, n, batch):
                step(first + f0, min(batch, n - f0), timed)

        run(warmup, False)
        # drain this rank's work (its RCCL gathers included) before the process group's own
        # collective: two communicators' kernels are never in flight together
        torch.cuda.synchronize()
        self.barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(self.stream)   # on the stream the trace kernel is launched on
        run(frames, True, first=warmup)
        ev1.record(self.stream)
        if sync is not None:
            sync()
        torch.cuda.synchronize()
        # this rank's time ends when its own work is done (rank 0's includes the gathered rows'
        # arrival and assembly); the barrier then closes the bracket, and the job's time is the
        # maximum over the ranks, which all left the opening barrier together
        elapsed = time.perf_counter() - t0
        self.barrier()
        region_ms = ev0.elapsed_time(ev1) if region_events else None
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

    def rank_plan(self, H, block, rank=None):
        """rt_render_opts of a rank's block-cyclic rows (its share of every frame; this rank's
        by default)."""
        o = self.capi.default_opts(tonemap=-1)
        if self.world > 1:
            o.row_begin, o.row_end = (self.rank if rank is None else rank) * block, H
            o.row_block, o.row_cycle = block, self.world
        return o


# ------------------------------------------------------------------------------ the headline
def choose_root_weight(n, render_ms, gather_ms, max_weight=16, margin=0.9):
    """Weight of rank 0's share (rt_comm_set_root_weight) from an equal-split probe: render_ms
    per rank and frame (≈ T/n each, T the whole frame on one GPU) and the ranks' gather times
    per frame (a peer's 1/n of the frame over its link: ≈ L/n, L the whole frame's bytes over one
    link, when the gather is link-bound; the fastest peer's, since a gather also waits for the
    other side to be ready).  With weight w the frame is dealt over V = w + n − 1
    row sets: rank 0 renders w/V of it (its rows never cross a link), a peer renders 1/V and
    sends 1/V.  Predicted frame time max(T·w/V, max(T, L)/V); w > 1 only when it beats the
    equal split's max(T/n, L/n) by the margin."""
    if n <= 1 or not render_ms or min(render_ms) <= 0:
        return 1
    T = sum(render_ms)
    peers = [g for g in gather_ms[1:] if g > 0] if gather_ms else []
    L = min(peers) * n if peers else 0.0
    equal = max(T / n, L / n)
    best_w, best_t = 1, equal
    for w in range(2, max_weight + 1):
        V = w + n - 1
        t = max(T * w / V, max(T, L) / V)
        if t < best_t:
            best_w, best_t = w, t
    return best_w if best_t < margin * equal else 1


def split_frames(R: Runner, sc, frames, warmup, batch, hdr="f64", tonemap=1, block=16,
                 pipeline=True, event_every=4, camera_step=None, gather=True, weight=1):
    """Frames of `sc` split over the ranks (block-cyclic rows), `batch` frames per
    rt_render_gather_batch call: this rank's rows of the HDR framebuffer stay on the rank, the
    fused bytes are gathered to rank 0 (one gather per batch; none at N=1) and assembled.
    gather=False: every rank renders whole frames of its own (weak scaling; same call on a
    one-rank view).  camera_step(base, frames) -> a new camera position per frame ([n, 3], one
    vectorised call per batch: the positions of the batch that opens the timed region are formed
    inside it, before its launch, while the GPU waits).
    weight > 1: rank 0 renders `weight` of the weight + N − 1 row sets (rt_comm_set_root_weight)."""
    torch, capi = R.torch, R.capi
    W, H = sc.camera.width, sc.camera.height
    dscene = R.ctx.scene(sc)
    split = gather and R.world > 1
    weight = weight if split else 1
    V = weight + R.world - 1 if split else 1
    # this rank's row sets ("slots") of the V-slot split: rank 0 slots [0, weight), rank r ≥ 1
    # slot weight + r − 1
    def slot_plan(s):
        o = capi.default_opts(tonemap=-1)
        o.row_begin, o.row_end, o.row_block, o.row_cycle = s * block, H, block, V
        return o
    if split:
        my_slots = list(range(weight)) if R.rank == 0 else [weight + R.rank - 1]
        slot_plans = [slot_plan(s) for s in my_slots]
        plan = slot_plans[0]
    else:
        slot_plans = [capi.default_opts(tonemap=-1)]
        plan = slot_plans[0]
    slot_rows = [capi.rendered_rows(p, H) if p.row_begin < H else 0 for p in slot_plans]
    rows = sum(slot_rows)
    # rt_render_gather_batch lays every row set's frames max_rows rows apart (the largest set's)
    max_rows = max(capi.rendered_rows(slot_plan(s), H) for s in range(V)
                   if s * block < H) if split else rows
    rays_rank = sum(R.count_rays(dscene, p) for p, r in zip(slot_plans, slot_rows) if r)
    comm = R.comm if split else R.solo_comm()
    if split:
        comm.set_root_weight(weight)
    # two sets of buffers (the pipelined slots): batch b writes set b mod 2
    hdr_dtype = torch.float64 if hdr == "f64" else torch.float32
    local = [torch.empty(max(max_rows, 1) * W * 3 * batch * len(slot_plans), dtype=hdr_dtype,
                         device="cuda") for _ in range(2)]
    root = R.rank == 0 or not split
    ldr = [torch.empty(H * W * 3 * batch if root else 1, dtype=torch.uint8, device="cuda")
           for _ in range(2)]
    pf = capi.RT_FLAG_PIPELINE if pipeline else 0
    opts = capi.default_opts(tonemap=tonemap, row_block=block if split else 0, flags=pf)
    topts = capi.default_opts(tonemap=tonemap, row_block=block if split else 0,
                              flags=pf | capi.RT_FLAG_TIME_KERNEL)
    base = dscene.camera["position"][0].copy()
    static_cams = dscene.cameras([base] * batch)
    nb, nt, nev = [0], [0], [0]
    last_n = [0, 0]  # frames of the call that last wrote buffer set 0 / 1

    # a moving camera's records for the timed frames, formed before the timed region like the
    # static camera's (the camera path is an input of the workload, as the scene is)
    timed_cams = None if camera_step is None else \
        dscene.cameras(camera_step(base, np.arange(warmup, warmup + frames)))

    def cams_for(f0, n):
        if camera_step is None:
            return static_cams[:n]
        if warmup <= f0 and f0 + n <= warmup + frames:
            return timed_cams[f0 - warmup:f0 - warmup + n]
        return dscene.cameras(camera_step(base, np.arange(f0, f0 + n)))

    def step(f0, n, timed):
        b = nb[0]
        nb[0] += 1
        # HIP events around every event_every-th TIMED batch, the first one included
        ev = timed and event_every > 0 and nt[0] % event_every == 0
        if timed:
            nt[0] += 1
        if ev:
            nev[0] += 1
        kw = {"rank_hdr64": local[b & 1].data_ptr()} if hdr == "f64" else \
             {"rank_hdr32": local[b & 1].data_ptr()}
        last_n[b & 1] = n
        comm.render_gather_batch(dscene, cams_for(f0, n), topts if ev else opts, capi.RT_OUT_LDR,
                                 d_ldr=ldr[b & 1].data_ptr(), **kw)

    # the clock warm-up renders this rank's rows without the gather (no collective)
    wopts = capi.default_opts(tonemap=tonemap)
    for f, _ in capi.RenderOpts._fields_:
        if f.startswith("row_"):
            setattr(wopts, f, getattr(plan, f))

    def warm_step(f0, n, timed):
        if rows:
            dscene.render_batch(static_cams[:n], local[0].data_ptr() if hdr == "f64" else None,
                                local[0].data_ptr() if hdr == "f32" else None,
                                ldr[0].data_ptr() if root else local[1].data_ptr(), wopts)

    comm.timing(reset=True)
    elapsed, region_ms = R.timed(step, frames, warmup, batch,
                                 warm_step=warm_step if split else None,
                                 region_events=True, sync=comm.synchronize if split else None,
                                 prime=(lambda: step(-2000000, batch, False)) if split else None)
    t = comm.timing(reset=True)
    if split and weight != 1:
        comm.set_root_weight(1)
    per_frame = [t.render_ms / max(t.frames, 1), t.gather_ms / max(t.frames, 1),
                 t.assemble_ms / max(t.frames, 1), float(rows), float(rays_rank), float(t.frames),
                 float(nev[0]), t.render_ms,
                 # the HIP events on the launch stream around the whole timed region, per frame
                 # (this rank's render time when no batch carried events of its own)
                 (region_ms / frames) if region_ms and frames else 0.0]
    ranks = R.gather_rows(per_frame)
    (rays_all,) = R.sum_over_ranks(float(rays_rank))
    dscene.close()
    return {"elapsed": elapsed, "rays": rays_all, "rays_rank": rays_rank, "ranks": ranks,
            "px": W * H, "rows": rows, "frames": frames, "batch": batch,
            "gather_bytes_per_frame": max_rows * W * 3 if split else 0, "root_weight": weight,
            "region_ms": region_ms, "launches": -(-frames // batch), "bufs": (local, ldr),
            "split": split, "V": V, "block": block, "weight": weight,
            "slots": my_slots if split else [0], "slot_rows": slot_rows, "max_rows": max_rows,
            "last_n": last_n, "last_set": (nb[0] - 1) & 1, "hdr": hdr,
            "static": camera_step is None}


def kernel_ms_per_frame(res, event_every):
    """Rank 0's render time per frame: per-batch HIP events (event_every > 0) or the HIP events
    on the launch stream around the whole timed region."""
    if event_every > 0:
        return res["ranks"][0][0]
    return res["region_ms"] / max(res["frames"], 1)


def per_rank_summary(res):
    ranks = res["ranks"]
    gb = res.get("gather_bytes_per_frame", 0)
    def entry(i, r):
        e = {"rank": i, "rows": int(r[3]), "rays_per_frame": int(r[4])}
        if int(r[5]) > 0:   # per-batch HIP events (render / gather / assembly)
            e.update({"render_ms_per_frame": round(r[0], 6),
                      "gather_ms_per_frame": round(r[1], 6),
                      "assemble_ms_per_frame": round(r[2], 6), "timed_frames": int(r[5]),
                      "timing": "HIP events around the event-timed batches"})
        else:               # no batch carried events: the region's HIP events
            e.update({"render_ms_per_frame": round(r[8], 6), "timed_frames": res["frames"],
                      "timing": "HIP events on the launch stream around the whole timed region "
                                "(render, gather and assembly together, launch gaps included)"})
        return e

    render = [r[0] if int(r[5]) > 0 else r[8] for r in ranks]
    mean = sum(render) / len(render)
    out = {
        "per_rank": [entry(i, r) for i, r in enumerate(ranks)],
        "render_imbalance": round(max(render) / mean, 4) if mean > 0 else None,
    }
    if gb and len(ranks) > 1:
        # bytes each rank sends per frame (its padded rows of Reinhard bytes) and the rate its
        # gather reached, from the end of its render to the end of the gather (the link rate
        # the row split depends on: DESIGN §6)
        out["gather_bytes_per_rank_frame"] = gb
        out["gather_GBps_per_rank"] = [round(gb / (r[1] * 1e-3) / 1e9, 2) if r[1] > 0 else None
                                       for r in ranks]
    return out


def golden_entry(sc, config: str):
    """The reference's full-frame record of this config (tests/golden/golden_meta.json, made by
    the reference compiled in the build container), when the bench's scene is the one it was
    made from (same scene text, same size); else None."""
    import hashlib
    path = os.path.join(HERE, "tests", "golden", "golden_meta.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        info = json.load(fh)["scenes"].get(f"{config}_full")
    if not info or (info["width"], info["height"]) != (sc.camera.width, sc.camera.height):
        return None
    if hashlib.sha256(sc.to_text().encode()).hexdigest() != info["scene_sha256"]:
        return None
    return info


def block_cyclic_rows(H: int, block: int, V: int, slot: int):
    """Image rows of row set `slot` of V (blocks of `block` rows, RE/Scene.h:318-325 split by
    rows), in the order the library packs them."""
    rows = []
    for b0 in range(slot * block, H, V * block):
        rows.extend(range(b0, min(b0 + block, H)))
    return rows


def frame_parity(R: Runner, sc, res, config: str, tonemap: int, tonemap_name: str):
    """Untimed certification of the timed path's output (after the timed region):
    * ldr_sha_ok (rank 0): SHA-256 of one assembled frame's tonemapped bytes (frame 0 of the
      last timed call; static camera) == the reference's (golden_meta.json);
    * ldr_equals_single_gpu (rank 0): the same bytes == a one-launch whole-frame render here;
    * hdr_rows_ok (every rank, AND over ranks): this rank's rank-local HDR rows of that frame ==
      the same rows of the whole-frame render on this GPU;
    * hdr_single_sha_ok (rank 0, f64): that whole-frame render's SHA == the reference's.
    None = not applicable (no golden for the scene, or a moving camera)."""
    import hashlib
    torch, capi = R.torch, R.capi
    W, H = sc.camera.width, sc.camera.height
    local, ldr = res["bufs"]
    info = golden_entry(sc, config)
    torch.cuda.synchronize()
    bs = res["last_set"]  # the buffer set of the last (timed) call
    out = {"golden": f"tests/golden/golden_meta.json scenes.{config}_full" if info else None,
           "frame": "frame 0 of the last timed call (static camera)"}
    if not res["static"]:
        return out
    # the whole frame on this GPU, one launch (rt_render_device), same outputs
    dscene = R.ctx.scene(sc)
    hdr_t = torch.float64 if res["hdr"] == "f64" else torch.float32
    ref_h = torch.empty(H * W * 3, dtype=hdr_t, device="cuda")
    ref_l = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
    with torch.cuda.stream(R.stream):
        dscene.render_device(ref_h.data_ptr() if res["hdr"] == "f64" else None,
                             ref_h.data_ptr() if res["hdr"] == "f32" else None,
                             ref_l.data_ptr(), capi.default_opts(tonemap=tonemap))
    torch.cuda.synchronize()
    dscene.close()
    # this rank's rows, every row set it renders (rank-local outputs: set k at
    # k * nframes * max_rows * W * 3, nframes = the frames of that call)
    nf, mr = res["last_n"][bs], res["max_rows"]
    ok = True
    for k, slot in enumerate(res["slots"]):
        rows = block_cyclic_rows(H, res["block"], res["V"], slot) if res["split"] else \
            list(range(H))
        if not rows:
            continue
        off = k * nf * mr * W * 3
        got = local[bs][off:off + len(rows) * W * 3].view(len(rows), W * 3)
        idx = torch.tensor(rows, dtype=torch.long, device="cuda")
        want = ref_h.view(H, W * 3).index_select(0, idx)
        ok = ok and bool(torch.equal(got, want))
    (worst,) = R.max_over_ranks(0.0 if ok else 1.0)
    out["hdr_rows_ok"] = worst == 0.0
    if R.rank == 0:
        frame = ldr[bs][:H * W * 3]
        out["ldr_equals_single_gpu"] = bool(torch.equal(frame, ref_l))
        if info:
            sha = hashlib.sha256(frame.cpu().numpy().tobytes()).hexdigest()
            want = info["ldr_sha256"].get(tonemap_name)
            out["ldr_sha_ok"] = (sha == want) if want else None
            if res["hdr"] == "f64":
                out["hdr_single_sha_ok"] = hashlib.sha256(
                    ref_h.cpu().numpy().tobytes()).hexdigest() == info["image_sha256"]
    return out


def parity_failed(p) -> bool:
    return any(p.get(k) is False for k in ("ldr_sha_ok", "ldr_equals_single_gpu", "hdr_rows_ok",
                                           "hdr_single_sha_ok"))


def single_launch_frames(R: Runner, sc, frames, warmup, tonemap=1):
    """One launch per frame (rt_render_device of the whole frame, f64 + bytes), the round-3
    headline path: returns (Mrays/s, ms per frame, HIP-event ms per launch)."""
    torch, capi = R.torch, R.capi
    W, H = sc.camera.width, sc.camera.height
    dscene = R.ctx.scene(sc)
    h = torch.empty(H * W * 3, dtype=torch.float64, device="cuda")
    l = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
    opts = capi.default_opts(tonemap=tonemap)
    rays = R.count_rays(dscene, opts)

    def step(f0, n, timed):
        for _ in range(n):
            dscene.render_device(h.data_ptr(), None, l.data_ptr(), opts)

    elapsed, region = R.timed(step, frames, warmup, 1, region_events=True)
    dscene.close()
    return rays * frames / elapsed / 1e6, elapsed / frames * 1e3, region / frames


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


def default_batch(world, steps):
    """Frames per call when --batch is not given.  N=1: 32 (one launch holds the driver's 20
    frames; nothing to gather).  N>1: the region's K frames in at least 4 batches, so batch
    b's gather overlaps batch b+1's render (RT_FLAG_PIPELINE, two batches in flight); with ONE
    batch the K frames' render and gather run back to back.  Model: time ≈
    K·max(R, G) + b·min(R, G) + (K/b)·c for render R and gather G per frame and a per-call cost
    c (~15 µs of RCCL stream time per gather, ramp and drain per launch), smallest near
    b = sqrt(K·c / min(R, G)) ≈ 4-8 frames for K = 20 at N = 2-8; 4 frames per launch is where the
    8-rank rank-frame stays within 1.4x of full/8 (tools/inflight_balance.py)."""
    if world <= 1:
        return 32
    return max(4, min(32, -(-steps // 4)))


def workload_text(sc, world, block, batch, hdr, tonemap_name):
    W, H = sc.camera.width, sc.camera.height
    return (f"{sc.name}: {W}x{H}, {len(sc.spheres)} spheres, {len(sc.planes)} planes, "
            f"{len(sc.lights)} point lights, AA=1, static camera; a step = one frame: every "
            f"rank renders its block-cyclic {block}-row blocks ({hdr} Vec3 HDR rows kept on the "
            f"rank + fused {tonemap_name} u8), one ncclGather per batch moves the u8 rows to "
            f"rank 0, which assembles the frame (N=1: the one rank renders the whole frame "
            f"straight into it); {batch} frames per call")


def tiled_roofline(t, W, render_ms):
    """§8(d)'s framebuffer-write roofline of a tiled config's render on rank 0: its rows'
    bytes per frame (15 B/px = float3 + u8, §8(d); 27 B/px = the f64 Vec3 + u8 written) / its
    render time per frame (HIP events around every timed batch)."""
    rows = int(t["ranks"][0][3])
    if render_ms <= 0:
        return None
    out = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "kernel_ms_per_frame": round(render_ms, 6)}
    for tag, bpp in (("15B", 15), ("27B", 27)):
        a = rows * W * bpp / (render_ms / 1e3) / 1e9
        out[f"achieved_{tag}"] = round(a, 2)
        out[f"frac_{tag}"] = round(a / HBM_PEAK_GBS, 5)
    return out


def _extras(R: Runner, args, sc, line, res, tonemap, batch):
    """The extra fields of the line (each with its own timing, outside the headline's)."""
    capi = R.capi
    from raytracingengine_amd.configs import make_config
    steps_x = min(args.steps, 96)
    # one launch per frame: the round-3 headline path
    v1, ms1, k1 = single_launch_frames(R, sc, steps_x, args.warmup, tonemap)
    (v1,) = R.sum_over_ranks(v1)
    line["single_launch"] = {"value": round(v1, 3), "ms_per_frame": round(ms1, 5),
                             "kernel_ms_per_launch": round(k1, 6),
                             "note": "every rank its own whole frames, one launch each "
                                     "(rt_render_device)"}
    # weak scaling: every rank its own whole frames, batched
    wk = split_frames(R, sc, steps_x, args.warmup, batch, args.hdr, tonemap, gather=False,
                      event_every=args.event_every)
    (rays_w,) = R.sum_over_ranks(float(wk["rays_rank"]))
    line["weak_frames"] = {
        "value": round(rays_w * steps_x / wk["elapsed"] / 1e6, 3),
        "ms_per_step": round(wk["elapsed"] / steps_x * 1e3, 5), "scaling": "weak",
        "workload": f"{sc.name} whole frames on every rank ({args.hdr} HDR + u8), "
                    f"{batch} per call"}
    if R.world == 1:
        f32 = split_frames(R, sc, steps_x, args.warmup, batch, "f32", tonemap,
                           event_every=args.event_every)
        k32 = kernel_ms_per_frame(f32, args.event_every)
        b32 = res["px"] * 15
        a32 = b32 / (k32 / 1e3) / 1e9 if k32 > 0 else 0.0
        line["roofline_f32"] = {
            "achieved": round(a32, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(a32 / HBM_PEAK_GBS, 5), "alg_bytes_per_frame": b32,
            "kernel_ms_per_frame": round(k32, 6),
            "value": round(f32["rays"] * steps_x / f32["elapsed"] / 1e6, 3)}
        mv = split_frames(R, sc, steps_x, args.warmup, batch, args.hdr, tonemap,
                          event_every=args.event_every,
                          camera_step=lambda base, i: base + np.outer(i * 1e-7, (1, 0, 0)))
        line["moving_camera"] = {
            "ms_per_step": round(mv["elapsed"] / steps_x * 1e3, 5),
            "kernel_ms_per_frame": round(kernel_ms_per_frame(mv, args.event_every), 6),
            "value": round(mv["rays"] * steps_x / mv["elapsed"] / 1e6, 3),
            "note": "camera x moved by 1e-7 every frame: no frame reuses a cached per-camera "
                    "packet image (one small launch per batch forms every frame's image "
                    "before the batch launch, DESIGN §4); rays counted at the first "
                    "position"}
        sc1 = make_config("c1", aa=32)
        v, ms, k = single_launch_frames(R, sc1, 10, 2, capi.TONEMAPS.index("aces"))
        line["reference_main_c1"] = {
            "workload": "c1: the reference main() box (5 mirrored axis planes, 2 point "
                        "lights), 1000x1000, AA=32, f64 Vec3 HDR + fused ACES u8",
            "ms_per_frame": round(ms, 4), "kernel_ms_per_launch": round(k, 4),
            "value": round(v, 3), "unit": "Mrays/s"}
        line["d2h"] = d2h_frames(R, sc, min(args.steps, 20), tonemap)
    # BASELINE config 3 (SURVEY §8e asks for scaling runs on C2, C3 and C4): the 4K frame,
    # 128 spheres, 4 point lights, row-tiled through the same path
    sc3 = make_config("c3", aa=1)
    n3 = min(args.steps, 32)
    t3 = split_frames(R, sc3, n3, min(args.warmup, 8), 8, "f64", tonemap, args.row_block,
                      not args.no_pipeline, 1)
    line["c3_tiled"] = {
        "value": round(t3["rays"] * n3 / t3["elapsed"] / 1e6, 3),
        "ms_per_frame": round(t3["elapsed"] / n3 * 1e3, 5),
        "frames": n3,
        "workload": "c3 3840x2160, 128 spheres, 4 planes, 4 point lights, f64 HDR rows on "
                    "each rank + Reinhard u8 gathered, 8 frames per call",
        "roofline": tiled_roofline(t3, sc3.camera.width, t3["ranks"][0][0]),
        **per_rank_summary(t3)}
    del t3
    # BASELINE config 4: the 8K frame row-tiled through the same path
    sc4 = make_config("c4", aa=1)
    t4 = split_frames(R, sc4, min(args.steps, 16), min(args.warmup, 2), 2, "f64", tonemap,
                      args.row_block, not args.no_pipeline, 1)
    line["c4_tiled"] = {
        "value": round(t4["rays"] * min(args.steps, 16) / t4["elapsed"] / 1e6, 3),
        "ms_per_frame": round(t4["elapsed"] / min(args.steps, 16) * 1e3, 5),
        "workload": "c4 7680x4320, 256 spheres, 8 lights, f64 HDR rows on each rank + "
                    "Reinhard u8 gathered, 2 frames per call",
        "roofline": tiled_roofline(t4, sc4.camera.width, t4["ranks"][0][0]),
        **per_rank_summary(t4)}


# ------------------------------------------------------------------------------ main
def main(argv=None):
    args = parse_args(argv)
    if needs_launcher(args):
        # --gpus N > 1 without an outer launcher: the N ranks run in ONE child process tree,
        # started before this process touches the GPU
        return launch_ranks(args, argv)
    R = Runner(args)
    if args.event_every is None:
        args.event_every = 0 if R.world == 1 else 4
    capi = R.capi
    from raytracingengine_amd.configs import make_config

    tonemap = capi.TONEMAPS.index(args.tonemap)
    sc = make_config(args.config, aa=1)
    W, H = sc.camera.width, sc.camera.height
    extras = not args.no_extras
    batch = max(1, args.batch) if args.batch else default_batch(R.world, args.steps)

    weight, probe = 1, None
    if R.world > 1 and args.root_weight != "1":
        if args.root_weight == "auto":
            # untimed equal-split probe: every batch timed with events
            pr = split_frames(R, sc, 8 * batch, batch, batch, args.hdr, tonemap, args.row_block,
                              not args.no_pipeline, 1)
            render = [r[0] for r in pr["ranks"]]
            gath = [r[1] for r in pr["ranks"]]
            (w,) = R.max_over_ranks(float(choose_root_weight(R.world, render, gath)))
            weight = int(w)
            probe = {"render_ms_per_frame": [round(x, 6) for x in render],
                     "gather_ms_per_frame": [round(x, 6) for x in gath], "chosen": weight}
        else:
            weight = max(1, int(args.root_weight))
    res = split_frames(R, sc, args.steps, args.warmup, batch, args.hdr, tonemap, args.row_block,
                       not args.no_pipeline, args.event_every, weight=weight)
    elapsed = res["elapsed"]
    value = res["rays"] * args.steps / elapsed / 1e6
    # untimed: the timed path's assembled frame and rank-local rows vs the reference's SHA and a
    # one-launch whole-frame render (every rank takes part)
    parity = frame_parity(R, sc, res, args.config, tonemap, args.tonemap)
    summ = per_rank_summary(res)
    r0 = res["ranks"][0]
    # the trace kernel: rank 0's render per frame — from HIP events around every
    # event_every-th timed batch launch, or (event_every 0, the N=1 default) from the HIP events
    # on the launch stream around the whole timed region (launch gaps included)
    if args.event_every > 0:
        render_ms = r0[0]
        ev_launches = max(int(r0[6]), 1)
        frames_per_launch = r0[5] / ev_launches   # the frames the event-timed launches held
        launch_ms = r0[7] / ev_launches           # measured per launch, not render_ms x batch
        timing_src = (f"HIP events around every {args.event_every}-th timed batch launch on the "
                      f"launch stream; those launches held {frames_per_launch:g} frames each")
    else:
        render_ms = res["region_ms"] / args.steps
        frames_per_launch = args.steps / res["launches"]
        launch_ms = res["region_ms"] / res["launches"]
        timing_src = (f"HIP events on the launch stream around the whole timed region "
                      f"({res['launches']} launch(es) of up to {batch} frames, "
                      f"{frames_per_launch:g} frames per launch on average; gaps between "
                      f"launches included)")
    bytes_per_frame = int(r0[3]) * W * (HDR_BYTES[args.hdr] + 3)
    achieved = bytes_per_frame / (render_ms / 1e3) / 1e9 if render_ms > 0 else 0.0
    # §8(d)'s FLOP roofline: F_ray = 25·Ns + 14·Np FP64 flops per ray of the reference's
    # brute-force IntersectClosest, rank 0's rays per frame / its render time per frame
    f_ray = 25 * len(sc.spheres) + 14 * len(sc.planes)
    flops_frame = res["rays_rank"] * f_ray if R.world == 1 else r0[4] * f_ray
    flops_tf = flops_frame / (render_ms / 1e3) / 1e12 if render_ms > 0 else 0.0
    # PMC traffic of a 32-frame batch launch (tools/pmc_passes.sh), scaled per frame to the
    # frames the timed launch held
    traffic, traffic_src = load_profile(f"pmc_{args.config}_batch32.json")
    traffic_launch = None
    if traffic and R.world == 1:
        traffic_launch = traffic["hbm_bytes_per_launch"] / 32 * frames_per_launch
    valu, valu_src = None, None
    for rnd in ("r06", "r05", "r04", "r03"):
        valu, valu_src = load_profile(f"{rnd}_{args.config}_valu.json")
        if valu is not None:
            break
    # committed counter summaries are from an earlier run: stale when the sources they were
    # taken from (their recorded rt_build_info digest) are not the ones this run loaded
    build = {k: v for k, v in capi.build_info().items() if k in
             ("source_sha256", "matches_tree", "arch", "hipcc")}

    def stale(prof):
        return prof is None or prof.get("source_sha256") != build.get("source_sha256")
    if valu is not None:
        valu = {k: v for k, v in valu.items() if k not in ("counters", "definitions")} | {
            "definitions": valu.get("definitions"), "stale": stale(valu)}
    line = {
        "metric": "Mrays/sec (primary+shadow) at 1920x1080" if args.config == "c2"
                  else f"Mrays/sec (primary+shadow), config {args.config}",
        "value": round(value, 3), "unit": "Mrays/s", "n_gpus": R.world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": workload_text(sc, R.world, args.row_block, batch, args.hdr,
                                      args.tonemap),
            "global_batch": args.steps, "resolution": [W, H],
            "parallelism": (f"block-cyclic rows ({args.row_block}-row blocks) x{R.world} + one "
                            f"ncclGather per batch of frames" if weight == 1 else
                            f"block-cyclic rows ({args.row_block}-row blocks) in {weight + R.world - 1} "
                            f"row sets, {weight} on rank 0 + one on each other rank, one group of "
                            f"P2P sends to rank 0 per batch of frames"),
            "root_weight": weight,
            "frames_per_call": batch, "rays_per_frame": int(res["rays"]),
        },
        "frames_per_sec": round(args.steps / elapsed, 3),
        # the library this run loaded: the sources it was compiled from (rt_build_info) and
        # whether they are the sources of this tree
        "build": build,
        "root_weight_probe": probe,
        "clock_warmup_ms": args.clock_warmup_ms,
        "kernel_ms_per_frame": round(render_ms, 6),
        "kernel_ms_per_launch": round(launch_ms, 6),
        "frames_per_timed_launch": round(frames_per_launch, 3),
        **summ,
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": round(traffic_launch) if traffic_launch else None,
            "alg_bytes_per_launch": round(bytes_per_frame * frames_per_launch),
            "alg_bytes_per_frame": bytes_per_frame,
            "traffic_source": traffic_src if R.world == 1 else None,
            "traffic_stale": stale(traffic) if traffic_launch else None,
            # SURVEY §8(d)'s own per-pixel figure: float3 + u8 = 15 B/px (the line's `frac`
            # counts the bytes this workload writes: the f64 Vec3 framebuffer + u8)
            "frac_sec8d_15B": round(int(r0[3]) * W * 15 / (render_ms / 1e3) / 1e9 /
                                    HBM_PEAK_GBS, 5) if render_ms > 0 else None,
            "traffic_note": ("PMC FETCH_SIZE x2 + WRITE_SIZE of a 32-frame launch of this "
                             "config (committed summary), per frame x the frames of the timed "
                             "launch") if traffic_launch else None,
            "flops_alg_per_frame": flops_frame,
            "flops_alg_tflops": round(flops_tf, 3),
            "flops_alg_frac": round(flops_tf / FP64_VALU_PEAK_TF, 5),
            "flops_note": (f"SURVEY §8(d): rays x F_ray (25*Ns + 14*Np = {f_ray} FP64 flops of "
                           "the reference's brute-force IntersectClosest per ray) / render time "
                           f"/ {FP64_VALU_PEAK_TF} TF; culling skips most of that work, so this "
                           "is the reference algorithm's rate, not counted flops (valu)"),
            "note": "rank 0's batch launch: its rows' framebuffer bytes (HDR + u8) per frame / "
                    f"its render time per frame ({timing_src})",
        },
        "parity": parity,
        "valu": valu if R.world == 1 else None,
        "valu_source": valu_src if R.world == 1 else None,
        "cpu_baseline": None,
    }
    if parity_failed(parity):
        # a wrong frame is not a measurement: print the line (it says which check failed), exit
        # non-zero, skip the extras
        extras = False
    if extras:
        _extras(R, args, sc, line, res, tonemap, batch)
    if R.world == 1 and not args.no_cpu_baseline and not parity_failed(parity):
        try:
            line["cpu_baseline"] = cpu_baseline(sc, res["rays_rank"], args.cpu_frames)
        except Exception as e:  # a reported baseline, never the product path
            line["cpu_baseline"] = {"error": repr(e)}
    if R.rank == 0:
        print(json.dumps(line), flush=True)
    R.close()
    return 3 if parity_failed(parity) else 0


if __name__ == "__main__":
    sys.exit(main())
