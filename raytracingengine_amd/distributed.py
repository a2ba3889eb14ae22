"""Row-tiled multi-GPU frames: one process per GPU, each renders its rows of the
frame, rank 0 assembles the frame with ONE gather collective.

Two row plans: contiguous tiles (`block=0`), or block-cyclic rows (`block=b`: blocks of b rows
dealt round-robin to the ranks).  Contiguous tiles of the BASELINE scenes are badly balanced
(the slowest of 8 tiles takes 1.7x the mean on C3/C4, tools/tile_balance.py, because spheres
cluster in the middle rows); block-cyclic rows even that out and are the default.

On MI355X the process group is ``torch.distributed`` with backend ``"nccl"`` (= RCCL over
xGMI); the gather is point-to-point into the root, so the peers' tiles arrive in parallel on
their own xGMI links.  The same code runs on ``gloo`` for the CPU tests, with the tile
renderer injected (the C oracle there; the HIP library on a GPU).

Pixels are independent (Scene::RenderImage has no cross-pixel dependency, Scene.h:318-325), so
a tiled frame is byte-identical to a single-GPU frame.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


def row_tile(rank: int, world: int, height: int) -> tuple[int, int]:
    """Contiguous rows [r0, r1) of `rank`; tile heights differ by at most one row."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return rank * height // world, (rank + 1) * height // world


DEFAULT_BLOCK = 16  # rows per block of the block-cyclic plan (a 16-row packet-kernel tile)


def row_ranges(rank: int, world: int, height: int, block: int = DEFAULT_BLOCK
               ) -> list[tuple[int, int]]:
    """The image rows of `rank` as [r0, r1) ranges, in the order its tile stores them:
    one contiguous tile (block == 0 or world == 1), or blocks of `block` rows starting at
    rank*block, rank*block + world*block, ... (rt_render_opts row_block / row_cycle)."""
    if block <= 0 or world == 1:
        return [row_tile(rank, world, height)]
    if not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return [(b, min(b + block, height)) for b in range(rank * block, height, world * block)]


def plan_rows(ranges: list[tuple[int, int]]) -> int:
    return sum(b - a for a, b in ranges)


def weighted_slots(rank: int, world: int, weight: int) -> list[int]:
    """Row sets ("slots") of `rank` in the weighted split (rt_comm_set_root_weight): the blocks
    are dealt over weight + world − 1 sets, rank 0 owns sets [0, weight), rank r ≥ 1 set
    weight + r − 1."""
    if weight < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world/weight")
    return list(range(weight)) if rank == 0 else [weight + rank - 1]


def gather_frames_weighted(slots: list[torch.Tensor], nframes: int, height: int, width: int,
                           weight: int, channels: int = 3, group=None,
                           block: int = DEFAULT_BLOCK) -> torch.Tensor | None:
    """The weighted split of rt_render_gather_batch with weight > 1 (rt_multi.cpp): `slots`
    holds this rank's row sets (weighted_slots), each [nframes * rows_of_set, width, channels]
    with the frames back to back.  Rank 0's own sets stay in place; every other rank sends its
    one set, padded to max_rows rows per frame, with a point-to-point send (one group of equal
    counts, as ncclSend / ncclRecv), and rank 0 writes every set's rows into image order —
    [nframes, height, width, channels] there, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    V = weight + world - 1
    sets = [row_ranges(s, V, height, block) for s in range(V)]
    max_rows = max(plan_rows(p) for p in sets)
    mine = weighted_slots(rank, world, weight)
    if len(slots) != len(mine):
        raise ValueError(f"rank {rank}: {len(slots)} row sets, expected {len(mine)}")

    def padded(t, s):
        rows = plan_rows(sets[s])
        if t.shape[0] != nframes * rows:
            raise ValueError(f"set {s}: {t.shape[0]} rows, expected {nframes} x {rows}")
        out = torch.zeros((nframes, max_rows, width, channels), dtype=t.dtype)
        out[:, :rows] = t.reshape(nframes, rows, width, channels)
        return out

    if rank != 0:
        dist.send(padded(slots[0], mine[0]).contiguous(), dst=0, group=group)
        return None
    recv = [None] * V
    for j, s in enumerate(mine):
        recv[s] = padded(slots[j], s)
    for r in range(1, world):
        buf = torch.empty((nframes, max_rows, width, channels), dtype=slots[0].dtype)
        dist.recv(buf, src=r, group=group)
        recv[weight + r - 1] = buf
    frames = torch.empty((nframes, height, width, channels), dtype=slots[0].dtype)
    for f in range(nframes):
        for s in range(V):
            k = 0
            for a, b in sets[s]:
                frames[f, a:b] = recv[s][f, k: k + (b - a)]
                k += b - a
    return frames


def gather_rows(tile: torch.Tensor, height: int, width: int, channels: int = 3,
                group=None, block: int = 0) -> torch.Tensor | None:
    """Gather every rank's [rows, width, channels] tile to rank 0 and return the full
    [height, width, channels] frame there (None elsewhere).  Tiles are padded to the tallest
    tile because the collective moves equal-sized buffers; rank 0 places each rank's rows with
    the same plan (`block`, see row_ranges)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    plans = [row_ranges(r, world, height, block) for r in range(world)]
    max_rows = max(plan_rows(p) for p in plans)
    if tile.shape[0] != plan_rows(plans[rank]):
        raise ValueError(f"rank {rank}: tile has {tile.shape[0]} rows, "
                         f"expected {plan_rows(plans[rank])}")
    send = tile
    if tile.shape[0] != max_rows:
        send = torch.zeros((max_rows, width, channels), dtype=tile.dtype, device=tile.device)
        send[: tile.shape[0]] = tile
    recv = None
    if rank == 0:
        recv = [torch.empty_like(send) for _ in range(world)]
    dist.gather(send.contiguous(), recv, dst=0, group=group)
    if rank != 0:
        return None
    frame = torch.empty((height, width, channels), dtype=tile.dtype, device=tile.device)
    for r, buf in enumerate(recv):
        k = 0
        for a, b in plans[r]:
            frame[a:b] = buf[k:k + (b - a)]
            k += b - a
    return frame


def gather_frames(packed: torch.Tensor, nframes: int, height: int, width: int,
                  channels: int = 3, group=None, block: int = DEFAULT_BLOCK
                  ) -> torch.Tensor | None:
    """A batch of frames: every rank's rows of `nframes` frames gathered to rank 0 with ONE
    gather and assembled there into [nframes, height, width, channels] (None elsewhere).  The
    layout of rt_render_gather_batch (rt_multi.cpp): each rank's frames lie max_rows rows apart
    (max_rows = the largest rank's row count; the rows past a rank's own are padding the
    assembly never reads), the gather moves the rank's nframes·max_rows rows at once and rank 0
    receives [world][nframes][max_rows] rows.  `packed` holds either that padded layout
    (nframes·max_rows rows, what the rank-local outputs of rt_render_gather_batch hold) or the
    frames back to back (nframes·rows rows, rt_render_batch's)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    plans = [row_ranges(r, world, height, block) for r in range(world)]
    max_rows = max(plan_rows(p) for p in plans)
    rows = plan_rows(plans[rank])
    if packed.shape[0] == nframes * max_rows:
        send = packed.reshape(nframes, max_rows, width, channels)
    elif packed.shape[0] == nframes * rows:
        send = torch.zeros((nframes, max_rows, width, channels), dtype=packed.dtype,
                           device=packed.device)
        send[:, :rows] = packed.reshape(nframes, rows, width, channels)
    else:
        raise ValueError(f"rank {rank}: {packed.shape[0]} packed rows, expected "
                         f"{nframes} x {rows} or {nframes} x {max_rows}")
    send = send.contiguous()
    recv = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, recv, dst=0, group=group)
    if rank != 0:
        return None
    frames = torch.empty((nframes, height, width, channels), dtype=packed.dtype,
                         device=packed.device)
    for f in range(nframes):
        for r in range(world):
            k = 0
            for a, b in plans[r]:
                frames[f, a:b] = recv[r][f, k: k + (b - a)]
                k += b - a
    return frames


def render_frame_tiled(render_rows: Callable[[list[tuple[int, int]]], torch.Tensor],
                       height: int, width: int, channels: int = 3, group=None,
                       block: int = DEFAULT_BLOCK) -> torch.Tensor | None:
    """Render this rank's rows with `render_rows(ranges)` (a [rows, width, channels] tensor of
    the ranges' rows, in order) and assemble the frame on rank 0."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    tile = render_rows(row_ranges(rank, world, height, block))
    return gather_rows(tile, height, width, channels, group, block=block)


def render_opts_for(ranges: list[tuple[int, int]], rank: int, world: int, height: int,
                    block: int, **kw):
    """rt_render_opts selecting exactly `ranges` (row_ranges of this rank) in one launch."""
    from . import capi

    if block <= 0 or world == 1:
        (r0, r1), = ranges
        return capi.default_opts(row_begin=r0, row_end=r1, **kw)
    return capi.default_opts(row_begin=rank * block, row_end=height, row_block=block,
                             row_cycle=world, **kw)


def hip_tile_renderer(dscene, rank: int, world: int, block: int = DEFAULT_BLOCK,
                      tonemap: int | None = None, dtype=torch.float32):
    """`render_rows` for a librtamd DeviceScene: renders this rank's rows in ONE launch into a
    device tensor on the context's stream (HDR float32, or the uint8 tonemap when `tonemap`
    is given)."""
    width = dscene.data.camera.width
    height = dscene.data.camera.height

    def render_rows(ranges: list[tuple[int, int]]) -> torch.Tensor:
        rows = plan_rows(ranges)
        if rows == 0:  # a rank past the last block (H < world·block): nothing to launch
            kind = torch.float32 if tonemap is None else torch.uint8
            out = torch.empty((0, width, 3), dtype=kind, device="cuda")
            return out if dtype is None or tonemap is not None else out.to(dtype)
        opts = render_opts_for(ranges, rank, world, height, block,
                               tonemap=-1 if tonemap is None else tonemap)
        if tonemap is None:
            out = torch.empty((rows, width, 3), dtype=torch.float32, device="cuda")
            dscene.render_device(None, out.data_ptr(), None, opts)
        else:
            out = torch.empty((rows, width, 3), dtype=torch.uint8, device="cuda")
            dscene.render_device(None, None, out.data_ptr(), opts)
        dscene.ctx.synchronize()
        return out if dtype is None or tonemap is not None else out.to(dtype)

    return render_rows
