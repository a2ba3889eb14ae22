"""Dev tool: build an A/B (or ablation) library from a patched copy of one source.

    python tools/build_variant.py NAME FILE 'old text' 'new text' ['old' 'new' ...] [-D MACRO ...]
        [--flags "extra hipcc flags replacing the source's in-tree extras"] [--src a.hip,b.hip]

FILE is a source under raytracingengine_amd/csrc; the copy (with every replacement applied,
each must match) is compiled with the in-tree flags and linked with the in-tree objects of the
other sources into tools/variants/NAME.so (git-ignored).  Ablation builds render wrong images;
time them with tools/ab_time.py / tools/pmc_ab.sh only.
"""
import os, shutil, subprocess, sys, tempfile
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from raytracingengine_amd import build as B

args = sys.argv[1:]
srcs = None  # --src a.hip,b.hip: the sources to recompile (when FILE is a header)
if "--src" in args:
    i = args.index("--src")
    srcs = args[i + 1].split(",")
    del args[i:i + 2]
extra = None  # --flags "...": replaces the in-tree per-source extra flags of the patched file(s)
if "--flags" in args:
    i = args.index("--flags")
    extra = args[i + 1].split()
    del args[i:i + 2]
defs = []
while "-D" in args:
    i = args.index("-D")
    defs.append("-D" + args[i + 1])
    del args[i:i + 2]
name, fname, reps = args[0], args[1], args[2:]
assert len(reps) % 2 == 0
B.build_library()
tmp = tempfile.mkdtemp()
src_dir = os.path.join(tmp, "csrc")
shutil.copytree(B.CSRC, src_dir)
path = os.path.join(src_dir, fname)
text = open(path).read()
for old, new in zip(reps[::2], reps[1::2]):
    assert old in text, f"patch text not found: {old[:60]!r}"
    text = text.replace(old, new)
open(path, "w").write(text)
inc = f"-I{os.path.join(B.ROOT, 'include')}"
rebuilt = {}
for src in srcs or [fname]:
    obj = os.path.join(tmp, src + ".o")
    flags = B.EXTRA_FLAGS.get(src, []) if extra is None else extra
    r = subprocess.run([B.HIPCC, *B.HIP_FLAGS, *flags, *defs, inc, "-c",
                        "-o", obj, os.path.join(src_dir, src)], stderr=subprocess.PIPE, text=True)
    if r.returncode:  # the errors only (the warnings of these sources are known)
        sys.exit("\n".join(l for l in r.stderr.splitlines() if "error" in l) or r.stderr[-4000:])
    rebuilt[src] = obj
objs = [rebuilt.get(s, os.path.join(B.OBJ_DIR, s + ".o")) for s in B.SOURCES]
objs.append(os.path.join(B.OBJ_DIR, "rt_build_info.cpp.o"))  # the in-tree build record
out_dir = os.path.join(B.ROOT, "tools", "variants")
os.makedirs(out_dir, exist_ok=True)
out = os.path.join(out_dir, name + ".so")
subprocess.check_call([B.HIPCC, *B.HIP_FLAGS, "-shared", "-o", out, *objs, *B.LINK_LIBS])
shutil.rmtree(tmp)
print(out)
