"""bench.py at N > 1 without an outer launcher, and the certification its line carries.

* `python bench.py --gpus N` run plainly (no WORLD_SIZE) starts ONE child,
  `python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>`, before it makes
  any GPU call (it does not even import torch), and exits with the child's status.
* The parity block compares one assembled frame with the reference's SHA in
  tests/golden/golden_meta.json: the bench's scene must be the one those SHAs were made from,
  and the row sets it checks must tile the frame (RE/Scene.h:318-325 split by rows)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CHILD = r"""
import json, os, subprocess, sys
sys.path.insert(0, %r)
seen = {}
def fake_run(cmd, env=None, **kw):
    seen["cmd"] = cmd
    seen["world"] = (env or {}).get("WORLD_SIZE")
    return subprocess.CompletedProcess(cmd, 7)
subprocess.run = fake_run
import bench
rc = bench.main(["--gpus", "2", "--steps", "64", "--warmup", "8"])
print(json.dumps({"rc": rc, "cmd": seen.get("cmd"), "world": seen.get("world"),
                  "torch": "torch" in sys.modules}))
"""


def test_gpus2_without_world_size_starts_one_launcher_child():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True,
                         text=True, timeout=120, check=True)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["rc"] == 7                      # the child's status is the bench's
    assert r["torch"] is False               # no torch (hence no GPU state) in the parent
    assert r["world"] is None
    cmd = r["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    assert any(a.startswith("--master-port=") for a in cmd)
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "2", "--steps", "64", "--warmup", "8"]


def test_outer_launcher_or_one_gpu_starts_nothing():
    a = bench.parse_args(["--gpus", "8"])
    assert bench.needs_launcher(a, {})
    assert not bench.needs_launcher(a, {"WORLD_SIZE": "8"})
    assert not bench.needs_launcher(bench.parse_args([]), {})


@pytest.mark.parametrize("H,block,V", [(1080, 16, 1), (1080, 16, 2), (1080, 16, 8),
                                       (4320, 16, 8), (2160, 16, 9), (1000, 7, 3)])
def test_row_sets_tile_the_frame(H, block, V):
    sets = [bench.block_cyclic_rows(H, block, V, s) for s in range(V)]
    flat = [r for s in sets for r in s]
    assert sorted(flat) == list(range(H))
    for s in sets:
        assert s == sorted(s)


@pytest.mark.parametrize("name", ["c2", "c3", "c4"])
def test_golden_applies_to_the_bench_scene(name):
    from raytracingengine_amd.configs import make_config
    sc = make_config(name, aa=1)
    info = bench.golden_entry(sc, name)
    assert info is not None, "the bench's scene drifted from the golden scene"
    assert "reinhard_simple" in info["ldr_sha256"]
    assert bench.golden_entry(make_config(name, 96, 54), name) is None


def test_parity_failed():
    assert not bench.parity_failed({"ldr_sha_ok": True, "hdr_rows_ok": True})
    assert not bench.parity_failed({"ldr_sha_ok": None, "hdr_rows_ok": True})
    assert bench.parity_failed({"ldr_sha_ok": True, "hdr_rows_ok": False})
    assert bench.parity_failed({"ldr_equals_single_gpu": False})


@pytest.mark.parametrize("world,steps,want", [
    (1, 20, 32), (1, 256, 32), (2, 20, 5), (8, 20, 5), (8, 8, 4), (4, 1, 4), (8, 256, 32),
    (2, 100, 25)])
def test_default_batch_splits_the_region_at_n_gt_1(world, steps, want):
    # N>1: at least 4 batches in the timed region so gathers overlap renders; N=1: 32
    b = bench.default_batch(world, steps)
    assert b == want
    if world > 1 and steps >= 16:
        assert -(-steps // b) >= 4


@pytest.mark.parametrize("H,block,V", [(1080, 8, 2), (1080, 8, 8), (1080, 16, 9), (270, 16, 3),
                                       (40, 16, 4), (123, 5, 4)])
def test_parity_rows_are_the_split_the_kernels_render(H, block, V):
    # bench.frame_parity reads a rank's rows in block_cyclic_rows order; that is the row order of
    # distributed.row_ranges, which test_block_cyclic_rows_equal_full_frame holds to the kernels
    from raytracingengine_amd.distributed import row_ranges
    for s in range(V):
        want = [r for a, b in row_ranges(s, V, H, block) for r in range(a, b)]
        assert bench.block_cyclic_rows(H, block, V, s) == want
