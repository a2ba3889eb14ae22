"""The RCCL gather across processes — one process per GPU, the bench's own call
(rt_render_gather_batch: block-cyclic rows, ONE ncclGather per batch, or with a root weight > 1
the grouped ncclSend / ncclRecv of the weighted split), pipelined and not: rank 0's assembled
frames equal rt_render_batch of the whole frames on one GPU, HDR and bytes (RE/Scene.h:318-325).

Needs at least two GPUs (RCCL allows one rank per GPU), so it is skipped on the one-GPU test box;
on a multi-GPU node it is the check that the cross-process RCCL paths deliver the frames
(they had not run on hardware when this test was written)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_WORKER = r'''
import json, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["RT_ROOT"])
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(rank)
dist.init_process_group("gloo")  # the unique id and the verdicts only; the frames go over RCCL
ctx = capi.Context(rank)
uid = [capi.comm_unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, src=0)
comm = capi.Comm(ctx, world, rank, uid[0], timeout_ms=60000)
W, H, nf, block = 320, 180, 5, 16
sc = make_config("c2", W, H)
ds = ctx.scene(sc)
base = ds.camera["position"][0].copy()
pos = np.array([base + (0.05 * f, -0.02 * f, 0.03 * f) for f in range(nf)])
cams = ds.cameras(pos)
ok, notes = True, []
ref64 = ref8 = None
if rank == 0:  # the whole frames on this GPU alone
    r64 = torch.empty(nf * H * W * 3, dtype=torch.float64, device="cuda")
    r8 = torch.empty(nf * H * W * 3, dtype=torch.uint8, device="cuda")
    ds.render_batch(cams, r64.data_ptr(), None, r8.data_ptr(), capi.default_opts(tonemap=1))
    ctx.synchronize()
    ref64, ref8 = r64.cpu().numpy(), r8.cpu().numpy()
for weight in (1, 2):
    comm.set_root_weight(weight)
    for pipeline in (False, True):
        opts = capi.default_opts(tonemap=1, row_block=block,
                                 flags=capi.RT_FLAG_PIPELINE if pipeline else 0)
        d64 = torch.full((nf * H * W * 3,), -1.0, dtype=torch.float64, device="cuda")
        d8 = torch.zeros(nf * H * W * 3, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for _ in range(2):  # two batches in a row through the pipelined slots
            comm.render_gather_batch(ds, cams, opts, capi.RT_OUT_LDR | capi.RT_OUT_HDR64,
                                     d_hdr64=d64.data_ptr(), d_ldr=d8.data_ptr())
        comm.synchronize()
        if rank == 0:
            same = (np.array_equal(d64.cpu().numpy(), ref64) and
                    np.array_equal(d8.cpu().numpy(), ref8))
            ok = ok and same
            notes.append({"weight": weight, "pipeline": pipeline, "equal": same})
comm.set_root_weight(1)
ds.close()
comm.close()
ctx.close()
if rank == 0:
    print("RESULT " + json.dumps({"ok": ok, "cases": notes}), flush=True)
dist.barrier()
dist.destroy_process_group()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (one RCCL rank each)")
def test_rccl_gather_batch_across_processes_is_the_frames(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(_WORKER)
    env = dict(os.environ, RT_ROOT=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script)]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["ok"], res
