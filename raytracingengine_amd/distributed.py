"""Row-tiled multi-GPU frames: one process per GPU, each renders a contiguous
row tile of the frame, rank 0 assembles the frame with ONE gather collective.

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


def gather_rows(tile: torch.Tensor, height: int, width: int, channels: int = 3,
                group=None) -> torch.Tensor | None:
    """Gather every rank's [rows, width, channels] tile to rank 0 and return the full
    [height, width, channels] frame there (None elsewhere).  Tiles are padded to the tallest
    tile because the collective moves equal-sized buffers."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    max_rows = -(-height // world)
    r0, r1 = row_tile(rank, world, height)
    if tile.shape[0] != r1 - r0:
        raise ValueError(f"rank {rank}: tile has {tile.shape[0]} rows, expected {r1 - r0}")
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
    parts = []
    for r, buf in enumerate(recv):
        a, b = row_tile(r, world, height)
        parts.append(buf[: b - a])
    return torch.cat(parts, dim=0)


def render_frame_tiled(render_rows: Callable[[int, int], torch.Tensor], height: int, width: int,
                       channels: int = 3, group=None) -> torch.Tensor | None:
    """Render this rank's tile with `render_rows(r0, r1)` and assemble the frame on rank 0."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    r0, r1 = row_tile(rank, world, height)
    tile = render_rows(r0, r1)
    return gather_rows(tile, height, width, channels, group)


def hip_tile_renderer(dscene, tonemap: int | None = None, dtype=torch.float32):
    """`render_rows` for a librtamd DeviceScene: renders [r0, r1) into a device tensor on the
    context's stream (HDR float32, or the uint8 tonemap when `tonemap` is given)."""
    from . import capi

    width = dscene.data.camera.width

    def render_rows(r0: int, r1: int) -> torch.Tensor:
        rows = r1 - r0
        opts = capi.default_opts(tonemap=-1 if tonemap is None else tonemap, row_begin=r0,
                                 row_end=r1)
        if tonemap is None:
            out = torch.empty((rows, width, 3), dtype=torch.float32, device="cuda")
            dscene.render_device(None, out.data_ptr(), None, opts)
        else:
            out = torch.empty((rows, width, 3), dtype=torch.uint8, device="cuda")
            dscene.render_device(None, None, out.data_ptr(), opts)
        dscene.ctx.synchronize()
        return out if dtype is None or tonemap is not None else out.to(dtype)

    return render_rows
