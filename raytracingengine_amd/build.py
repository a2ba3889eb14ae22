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
SOURCES = ["rt_trace.hip", "rt_capi.cpp"]
LIB = os.path.join(HERE, "librtamd.so")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [
        os.path.join(ROOT, "include", "rt_capi.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = [HIPCC, *HIP_FLAGS, "-shared", f"-I{os.path.join(ROOT, 'include')}", "-o", LIB,
           *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return LIB


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    print(build_library(force="--force" in argv, verbose=True))


if __name__ == "__main__":
    main()
