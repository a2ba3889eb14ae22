"""Register budgets of the built gfx950 kernels (CPU: reads the code objects' metadata).

Occupancy is the lever measured most in DESIGN.md §4: the single-sample packet kernels run at
5 waves/SIMD (≤ 96 VGPRs + AGPRs; C2's and the area-only one at 6, ≤ 80), the lean reflection-chain kernels at 3 (≤ 168: C1 -19 %,
mirror -23 % against 2) and the other generic / breadth-first trace kernels at 2 (≤ 256).
An unrelated change once pushed the breadth-first level kernel into AGPRs and 1 wave/SIMD
(glass +35 %); this pins the budgets on the objects `build()` produced."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "build", "obj")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(src):
    obj = os.path.join(OBJ, src + ".o")
    if not os.path.exists(obj):
        pytest.skip(f"{obj} not built")
    tmp = os.path.join(OBJ, "_meta_" + src)
    os.makedirs(tmp, exist_ok=True)
    fb, co = os.path.join(tmp, "fatbin"), os.path.join(tmp, "gfx950.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                    os.path.join(tmp, "host.o")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    out = {}
    for entry in re.split(r"\n  - \.", notes):  # kernel records (argument records are deeper)
        name = re.search(r"\n    \.name:\s+(\S+)", entry)
        v = re.search(r"vgpr_count:\s+(\d+)", entry)
        a = re.search(r"^agpr_count:\s+(\d+)", entry)
        if name and v and a and "_kernel" in name.group(1):
            out[name.group(1)] = int(v.group(1)) + int(a.group(1))
    assert out, "no kernel metadata found"
    return out


def _waves(regs):
    return min(8, 512 // max(8, -(-regs // 8) * 8))


def test_packet_single_sample_kernels_run_at_5_waves():
    ks = {**_kernels("rt_packet.hip"), **_kernels("rt_packet_area.hip")}
    # packet_direct_kernel<MAXC, FEAT, COUNT=false, MULTI=false, WGY>, FEAT 0 (lean), 2 (area)
    # or 16 (plane cull)
    lean = {n: r for n, r in ks.items()
            if re.search(r"packet_direct_kernelILi[14]ELi(0|2|16|34)ELb0ELb0E", n)}
    assert len(lean) == 14, sorted(lean)
    assert all(_waves(r) >= 5 for r in lean.values()), lean
    # <= 64 spheres and point lights only (C2): 6, its light records read through the scalar cache
    small = {n: r for n, r in lean.items() if re.search(r"packet_direct_kernelILi1ELi0ELb0ELb0E", n)}
    assert small and all(_waves(r) >= 6 for r in small.values()), small
    # the area-only variant (FEAT 34 = area light, no planes / point lights: C5) runs at 6
    area_only = {n: r for n, r in lean.items() if "ELi34E" in n}
    assert len(area_only) == 2 and all(_waves(r) >= 6 for r in area_only.values()), area_only


@pytest.mark.parametrize("src", ["rt_trace.hip", "rt_trace_lean.hip", "rt_wavefront.hip"])
def test_generic_trace_kernels_run_at_2_waves(src):
    ks = _kernels(src)
    heavy = {n: r for n, r in ks.items() if "trace_kernel" in n or "wf_level_kernel" in n}
    assert heavy
    assert all(_waves(r) >= 2 for r in heavy.values()), heavy


def test_lean_chain_kernels_run_at_3_waves():
    """trace_kernel<PATH = chain, COUNT, LDS, MINW = 3, SINGLE, NOSPH, SPAR> of rt_trace_lean.hip
    (C1, mirror; NOSPH: the sphere-free instantiations C1 takes; SPAR: one thread per sample)."""
    ks = _kernels("rt_trace_lean.hip")
    chain = {n: r for n, r in ks.items() if re.search(r"trace_kernelILi1ELb[01]ELb[01]ELi3E", n)}
    assert len(chain) == 24, sorted(ks)
    assert all(_waves(r) >= 3 for r in chain.values()), chain
