"""Dev micro-benchmark: host enqueue cost and GPU time of one ncclGather on a one-rank RCCL
communicator (the per-frame gather of rt_multi.cpp at the 8-rank C2 size: 135 rows x 1920 x 3 B
per rank), to size the per-frame host budget of a row-split frame.
    python tools/micro/rccl_host.py [bytes] [iters]"""
import ctypes
import sys
import time

import torch

nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 136 * 1920 * 3
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
lib = ctypes.CDLL("/opt/rocm/lib/librccl.so")


class UID(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


uid = UID()
assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
comm = ctypes.c_void_p()
torch.cuda.set_device(0)
assert lib.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
s = torch.cuda.Stream()
src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
st = ctypes.c_void_p(s.cuda_stream)
lib.ncclGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                           ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]


def gather():
    lib.ncclGroupStart()
    r = lib.ncclGather(src.data_ptr(), dst.data_ptr(), nbytes, 0, 0, comm, st)
    lib.ncclGroupEnd()
    return r


for _ in range(50):
    assert gather() == 0
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    gather()
host = (time.perf_counter() - t0) / iters * 1e6
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record(s)
for _ in range(iters):
    gather()
e1.record(s)
torch.cuda.synchronize()
print({"bytes": nbytes, "host_us_per_gather": round(host, 2),
       "stream_us_per_gather": round(e0.elapsed_time(e1) / iters * 1e3, 2)})
# a batch: 16 gathers in one group (rt_render_gather_batch) vs one gather of 16x the bytes
big_src = torch.empty(16 * nbytes, dtype=torch.uint8, device="cuda")
big_dst = torch.empty(16 * nbytes, dtype=torch.uint8, device="cuda")


def group16():
    lib.ncclGroupStart()
    for f in range(16):
        lib.ncclGather(big_src.data_ptr() + f * nbytes, big_dst.data_ptr() + f * nbytes, nbytes,
                       0, 0, comm, st)
    lib.ncclGroupEnd()


def one_big():
    lib.ncclGroupStart()
    lib.ncclGather(big_src.data_ptr(), big_dst.data_ptr(), 16 * nbytes, 0, 0, comm, st)
    lib.ncclGroupEnd()


for fn, name in ((group16, "group_of_16_gathers"), (one_big, "one_gather_of_16x")):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(200):
        fn()
    e1.record(s)
    host = (time.perf_counter() - t0) / 200 * 1e6
    torch.cuda.synchronize()
    print({name: {"host_us_per_call": round(host, 2),
                  "stream_us_per_call": round(e0.elapsed_time(e1) / 200 * 1e3, 2)}})
# the empty ctypes call, for scale
t0 = time.perf_counter()
for _ in range(iters):
    lib.ncclGroupStart()
    lib.ncclGroupEnd()
print({"host_us_group_only": round((time.perf_counter() - t0) / iters * 1e6, 2)})
lib.ncclCommDestroy(comm)
