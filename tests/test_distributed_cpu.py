"""Multi-process row tiling on CPU (gloo): tiles rendered by separate ranks and gathered to
rank 0 reassemble the single-process frame byte for byte (the C oracle renders the tiles
here; on the GPU the HIP library does, through the same gather code)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raytracingengine_amd.distributed import plan_rows, row_ranges, row_tile


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, w, h, outdir, block):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import pyoracle as po
    from raytracingengine_amd.configs import make_config
    from raytracingengine_amd.distributed import render_frame_tiled

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = make_config(name, w, h)

    def render_rows(ranges):
        parts = [po.render(sc, rows=(r0, r1), nthreads=1)[0] for r0, r1 in ranges]
        if not parts:  # a rank past the last block
            return torch.empty((0, w, 3), dtype=torch.float64)
        return torch.from_numpy(np.concatenate(parts))

    frame = render_frame_tiled(render_rows, h, w, block=block)
    if rank == 0:
        np.save(os.path.join(outdir, "frame.npy"), frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,name,w,h,block", [(2, "c2", 96, 54, 0), (3, "mirror", 40, 23, 0),
                                                  (2, "c2", 96, 54, 16), (3, "mirror", 40, 23, 4),
                                                  # rank 2 owns no rows (H < world·block)
                                                  (3, "c2", 48, 24, 16)])
def test_tiled_gather_equals_full_frame(tmp_path, world, name, w, h, block):
    from oracle import pyoracle as po
    from raytracingengine_amd.configs import make_config
    mp.start_processes(_worker, args=(world, _free_port(), name, w, h, str(tmp_path), block),
                       nprocs=world, join=True, start_method="spawn")
    frame = np.load(tmp_path / "frame.npy")
    full, _, _ = po.render(make_config(name, w, h))
    assert np.array_equal(frame, full)


def _batch_worker(rank, world, port, name, w, h, outdir, block, nframes, padded):
    import dataclasses
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import pyoracle as po
    from raytracingengine_amd.configs import make_config
    from raytracingengine_amd.distributed import gather_frames

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = make_config(name, w, h)
    ranges = row_ranges(rank, world, h, block)
    parts = []
    for f in range(nframes):  # this rank's rows of frame f (camera f), packed frame by frame
        cam = dataclasses.replace(sc.camera, position=_batch_position(sc, f))
        scf = dataclasses.replace(sc, camera=cam)
        parts += [po.render(scf, rows=(r0, r1), nthreads=1)[0] for r0, r1 in ranges]
    packed = torch.from_numpy(np.concatenate(parts)) if parts else \
        torch.empty((0, w, 3), dtype=torch.float64)
    if padded:  # the rank-local layout of rt_render_gather_batch: frames max_rows rows apart
        rows = plan_rows(ranges)
        max_rows = max(plan_rows(row_ranges(r, world, h, block)) for r in range(world))
        pad = torch.full((nframes, max_rows, w, 3), float("nan"), dtype=torch.float64)
        pad[:, :rows] = packed.reshape(nframes, rows, w, 3)
        packed = pad.reshape(nframes * max_rows, w, 3)
    frames = gather_frames(packed, nframes, h, w, block=block)
    if rank == 0:
        np.save(os.path.join(outdir, "frames.npy"), frames.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _batch_position(sc, f):
    x, y, z = sc.camera.position
    return (x + 0.25 * f, y - 0.125 * f, z + 0.5 * f)


@pytest.mark.parametrize("world,name,w,h,block,nframes,padded", [
    (2, "c2", 64, 40, 16, 3, False),
    (3, "c2", 48, 37, 8, 2, True),
    (3, "c2", 40, 24, 16, 2, False),   # rank 2 owns no rows
    (3, "c2", 40, 24, 16, 3, True)])
def test_batched_gather_equals_full_frames(tmp_path, world, name, w, h, block, nframes, padded):
    """A batch of frames (one camera each) split over the ranks, ONE gather of the whole batch
    with the send / receive layout of rt_render_gather_batch (each rank's frames max_rows rows
    apart, NaN padding that the assembly must never read): rank 0's frames equal the
    single-process frames."""
    import dataclasses
    from oracle import pyoracle as po
    from raytracingengine_amd.configs import make_config
    mp.start_processes(_batch_worker,
                       args=(world, _free_port(), name, w, h, str(tmp_path), block, nframes,
                             padded),
                       nprocs=world, join=True, start_method="spawn")
    frames = np.load(tmp_path / "frames.npy")
    sc = make_config(name, w, h)
    for f in range(nframes):
        cam = dataclasses.replace(sc.camera, position=_batch_position(sc, f))
        full, _, _ = po.render(dataclasses.replace(sc, camera=cam))
        assert np.array_equal(frames[f], full), f


def test_row_tile_partition():
    for H in (1, 7, 54, 1080, 4320):
        for world in (1, 2, 3, 4, 8):
            tiles = [row_tile(r, world, H) for r in range(world)]
            assert tiles[0][0] == 0 and tiles[-1][1] == H
            assert all(a[1] == b[0] for a, b in zip(tiles, tiles[1:]))
            sizes = [b - a for a, b in tiles]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        row_tile(2, 2, 10)


def test_block_cyclic_partition():
    """Every row belongs to exactly one rank's block-cyclic plan; ranks differ by <= 1 block."""
    for H in (1, 7, 54, 123, 1080, 4320):
        for world in (1, 2, 3, 8):
            for block in (1, 5, 16):
                plans = [row_ranges(r, world, H, block) for r in range(world)]
                rows = sorted(y for p in plans for a, b in p for y in range(a, b))
                assert rows == list(range(H))
                sizes = [plan_rows(p) for p in plans]
                assert max(sizes) - min(sizes) <= block


def _weighted_worker(rank, world, port, name, w, h, outdir, block, nframes, weight):
    import dataclasses
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import pyoracle as po
    from raytracingengine_amd.configs import make_config
    from raytracingengine_amd.distributed import gather_frames_weighted, weighted_slots

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = make_config(name, w, h)
    V = weight + world - 1
    slots = []
    for s in weighted_slots(rank, world, weight):  # each row set: its rows of every frame
        ranges = row_ranges(s, V, h, block)
        parts = []
        for f in range(nframes):
            cam = dataclasses.replace(sc.camera, position=_batch_position(sc, f))
            scf = dataclasses.replace(sc, camera=cam)
            parts += [po.render(scf, rows=(r0, r1), nthreads=1)[0] for r0, r1 in ranges]
        slots.append(torch.from_numpy(np.concatenate(parts)) if parts else
                     torch.empty((0, w, 3), dtype=torch.float64))
    frames = gather_frames_weighted(slots, nframes, h, w, weight, block=block)
    if rank == 0:
        np.save(os.path.join(outdir, "frames.npy"), frames.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,name,w,h,block,nframes,weight", [
    (2, "c2", 64, 40, 8, 2, 3),
    (3, "c2", 48, 37, 8, 2, 2),
    (3, "c2", 40, 24, 16, 2, 2)])   # some row sets own no rows
def test_weighted_gather_equals_full_frames(tmp_path, world, name, w, h, block, nframes, weight):
    """The weighted split (rt_comm_set_root_weight) with gloo: rank 0 renders `weight` of the
    weight + world − 1 row sets, every other rank one, sent point to point to rank 0 (equal,
    padded counts) — rank 0's frames equal the single-process frames."""
    import dataclasses
    from oracle import pyoracle as po
    from raytracingengine_amd.configs import make_config
    mp.start_processes(_weighted_worker,
                       args=(world, _free_port(), name, w, h, str(tmp_path), block, nframes,
                             weight),
                       nprocs=world, join=True, start_method="spawn")
    frames = np.load(tmp_path / "frames.npy")
    sc = make_config(name, w, h)
    for f in range(nframes):
        cam = dataclasses.replace(sc.camera, position=_batch_position(sc, f))
        full, _, _ = po.render(dataclasses.replace(sc, camera=cam))
        assert np.array_equal(frames[f], full), f
