"""Dev tool: build an A/B library whose rt_packet.hip device code has every VOP2
`v_cndmask_b32_e32 …, vcc` re-encoded as VOP3 (`v_cndmask_b32_e64`): on gfx950 the VOP2 select
measured 23 cycles per wave-instruction against 4.4 for the VOP3 one (tools/micro/valu_rates.hip,
profiles/r05_valu_rates.txt).  Same operation, same operands (src0 a VGPR or an inline constant,
so the VOP3 form needs no second constant-bus read); the assembler rejects anything else.

    python tools/vop3_build.py NAME [source.hip]     -> tools/variants/NAME.so

Pipeline (what hipcc runs, with the patch in the middle): device assembly (--cuda-device-only -S)
-> patch -> assemble -> lld -> clang-offload-bundler -> host compile with the bundle embedded
(-fcuda-include-gpubinary) -> link with the in-tree objects of the other sources."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from raytracingengine_amd import build as B  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"
PAT = re.compile(r"^(\s*)v_cndmask_b32_e32 (v\d+), (v\d+|-?\d+|0x[0-9a-f]+|[-0-9.e]+), (v\d+), vcc\s*$")
INLINE_INT = set(str(i) for i in range(-16, 65))
INLINE_F = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0"}


def patch_asm(text: str) -> tuple[str, int, int]:
    out, n, skipped = [], 0, 0
    for line in text.splitlines(keepends=True):
        m = PAT.match(line)
        if m and (m.group(3).startswith("v") or m.group(3) in INLINE_INT or m.group(3) in INLINE_F):
            out.append(f"{m.group(1)}v_cndmask_b32_e64 {m.group(2)}, {m.group(3)}, {m.group(4)}, vcc\n")
            n += 1
        else:
            if "v_cndmask_b32_e32" in line:
                skipped += 1
            out.append(line)
    return "".join(out), n, skipped


def compile_patched(src: str, obj: str, tmp: str) -> None:
    flags = [*B.HIP_FLAGS, *B.EXTRA_FLAGS.get(os.path.basename(src), []),
             f"-I{os.path.join(B.ROOT, 'include')}"]
    dev_s = os.path.join(tmp, "dev.s")
    subprocess.run([B.HIPCC, *flags, "--cuda-device-only", "-S", "-o", dev_s, src], check=True)
    text, n, skipped = patch_asm(open(dev_s).read())
    print(f"{os.path.basename(src)}: {n} VOP2 selects re-encoded as VOP3, {skipped} left", flush=True)
    dev_p = os.path.join(tmp, "dev_patched.s")
    open(dev_p, "w").write(text)
    dev_o = os.path.join(tmp, "dev.o")
    subprocess.run([f"{LLVM}/clang", "-target", "amdgcn-amd-amdhsa", f"-mcpu={B.ARCH}", "-c",
                    dev_p, "-o", dev_o], check=True)
    hsaco = os.path.join(tmp, "dev.hsaco")
    subprocess.run([f"{LLVM}/ld.lld", "-flavor", "gnu", "-m", "elf64_amdgpu", "--no-undefined",
                    "-shared", "-o", hsaco, dev_o], check=True)
    fb = os.path.join(tmp, "dev.hipfb")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "-type=o", "-bundle-align=4096",
                    f"-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--{B.ARCH}",
                    "-input=/dev/null", f"-input={hsaco}", f"-output={fb}"], check=True)
    subprocess.run([B.HIPCC, *flags, "--cuda-host-only", "-Xclang", "-fcuda-include-gpubinary",
                    "-Xclang", fb, "-c", "-o", obj, src], check=True)


def main():
    name = sys.argv[1]
    srcname = sys.argv[2] if len(sys.argv) > 2 else "rt_packet.hip"
    B.build_library()
    tmp = tempfile.mkdtemp()
    obj = os.path.join(tmp, srcname + ".o")
    compile_patched(os.path.join(B.CSRC, srcname), obj, tmp)
    objs = [obj if os.path.basename(o) == srcname + ".o" else o
            for o in [os.path.join(B.OBJ_DIR, s + ".o") for s in B.SOURCES]]
    objs.append(os.path.join(B.OBJ_DIR, "rt_build_info.cpp.o"))
    out_dir = os.path.join(B.ROOT, "tools", "variants")
    os.makedirs(out_dir, exist_ok=True)
    lib = os.path.join(out_dir, name + ".so")
    subprocess.run([B.HIPCC, *B.HIP_FLAGS, "-shared", "-o", lib, *objs, *B.LINK_LIBS], check=True)
    print(lib)


if __name__ == "__main__":
    main()
