"""Build recipe for the HIP library (gfx950 only) and the C++ drop-in archive.

``python -m raytracingengine_amd.build`` compiles, in-tree (so the .so travels to the GPU box):

* ``raytracingengine_amd/librtamd.so`` — the kernels (rt_trace.hip) and the C-ABI
  (rt_capi.cpp) with ``hipcc --offload-arch=gfx950 -ffp-contract=off``.

Floating-point flags are part of the parity contract: ``-ffp-contract=off`` keeps every
multiply and add separately rounded, as in the reference's SSE2 build.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

HIP_FLAGS = ["-O3", "-std=c++20", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC",
             "-Wall", "-Wno-unused-result"]
SOURCES = ["rt_trace.hip", "rt_trace_lean.hip", "rt_packet.hip", "rt_packet_area.hip",
           "rt_wavefront.hip", "rt_wavefront_lean.hip", "rt_assemble.hip", "rt_box.hip", "rt_capi.cpp",
           "rt_multi.cpp", "rt_queue.cpp", "rt_bvh.cpp"]
# RCCL (multi-GPU frames, rt_multi.cpp).  Inside a PyTorch process the loader reuses torch's
# librccl.so.1 (same soname, loaded first by capi.load_library), so one RCCL serves both.
LINK_LIBS = ["-L/opt/rocm/lib", "-lrccl"]
# per-source extra flags: the packet kernel schedules for ILP (measured 1-2 % faster on C1-C5;
# the generic kernels are not: mesh/glass 1-5 % slower)
EXTRA_FLAGS = {"rt_packet.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}
OBJ_DIR = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(HERE, "librtamd.so")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = False) -> str:
    # the recipe itself is a dependency: a change of HIP_FLAGS / EXTRA_FLAGS / SOURCES rebuilds.
    # Objects are rebuilt per source: a source's object is stale when the source, any header
    # (csrc/*.hpp, include/rt_capi.h) or this recipe is newer.
    # (.hip sources also depend on the other .hip files: rt_trace_lean.hip includes rt_trace.hip)
    common = [os.path.join(ROOT, "include", "rt_capi.h"), os.path.abspath(__file__)]
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    hip_files = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip")]
    os.makedirs(OBJ_DIR, exist_ok=True)
    inc = f"-I{os.path.join(ROOT, 'include')}"
    procs, objs = [], []
    for src in SOURCES:  # one hipcc per stale source, in parallel
        obj = os.path.join(OBJ_DIR, src + ".o")
        objs.append(obj)
        deps = [os.path.join(CSRC, src)] + headers + common + (hip_files if src.endswith(".hip") else [])
        if not force and not _stale(obj, deps):
            continue
        cmd = [HIPCC, *HIP_FLAGS, *EXTRA_FLAGS.get(src, []), inc, "-c", "-o", obj,
               os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((cmd, subprocess.Popen(cmd)))
    for cmd, p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    if not force and not procs and not _stale(LIB, objs):
        return LIB
    cmd = [HIPCC, *HIP_FLAGS, "-shared", "-o", LIB, *objs, *LINK_LIBS]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return LIB


API_DIR = os.path.join(HERE, "api")
CPP_LIB = os.path.join(HERE, "librtamd_cpp.so")
CPP_FLAGS = ["-std=c++20", "-O2", "-fPIC", "-ffp-contract=off", "-Wall", "-Wextra",
             f"-I{API_DIR}", f"-I{os.path.join(ROOT, 'include')}"]
EXAMPLES = {"box_demo": "box_demo.cpp", "render_scenefile": "render_scenefile.cpp"}


def build_cpp_api(force: bool = False, verbose: bool = False) -> str:
    """The drop-in C++20 API (api/rtamd/*.cpp) as librtamd_cpp.so over librtamd.so, plus the
    example programs under examples/ (bin in examples/bin, rpath to the package dir)."""
    build_library(force=force, verbose=verbose)
    srcs = [os.path.join(API_DIR, "rtamd", f) for f in ("scene.cpp", "image.cpp", "obj.cpp")]
    hdrs = [os.path.join(API_DIR, "rtamd", f) for f in os.listdir(os.path.join(API_DIR, "rtamd"))]
    link = [f"-L{HERE}", "-lrtamd", f"-Wl,-rpath,{HERE}", "-Wl,-rpath,$ORIGIN"]
    cxx = os.environ.get("CXX", "g++")
    if force or _stale(CPP_LIB, srcs + hdrs + [LIB, os.path.abspath(__file__)]):
        cmd = [cxx, *CPP_FLAGS, "-shared", "-o", CPP_LIB, *srcs, *link]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    bindir = os.path.join(ROOT, "examples", "bin")
    os.makedirs(bindir, exist_ok=True)
    for exe, src in EXAMPLES.items():
        src = os.path.join(ROOT, "examples", src)
        target = os.path.join(bindir, exe)
        if force or _stale(target, [src, CPP_LIB] + hdrs):
            cmd = [cxx, *CPP_FLAGS, "-o", target, src, f"-L{HERE}", "-lrtamd_cpp", "-lrtamd",
                   f"-Wl,-rpath,{HERE}", "-Wl,-rpath,$ORIGIN/../../raytracingengine_amd"]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    return CPP_LIB


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    print(build_library(force="--force" in argv, verbose=True))
    print(build_cpp_api(force="--force" in argv, verbose=True))


if __name__ == "__main__":
    main()
