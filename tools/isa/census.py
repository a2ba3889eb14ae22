#!/usr/bin/env python3
"""Static ISA census of one kernel in a `hipcc --cuda-device-only -S` listing (dev tool).

    python tools/isa/census.py /tmp/pk.s 'packet_direct_kernelILi1ELi0ELb0ELb0ELi1E' [--blocks]

Counts the instructions of the kernel by class (FP64 / FP32 / int VALU, v_cndmask, v_mov,
v_cmp, SALU, LDS, global, branches), and with --blocks prints every basic block with its size
and class counts, so that the blocks of the hot path can be attributed to source phases."""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_cndmask"):
        return "v_cndmask"
    if op.startswith(("v_mov", "v_readlane", "v_readfirstlane", "v_writelane")):
        return "v_mov/lane"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "v_cmp_f64" if "f64" in op else "v_cmp_other"
    if op.startswith("v_"):
        if "f64" in op:
            if any(k in op for k in ("rcp", "rsq", "sqrt", "div_scale", "div_fmas", "div_fixup",
                                     "ldexp", "frexp", "trig", "class")):
                return "v_f64_special"
            return "v_f64_arith"
        if "f32" in op or "f16" in op:
            return "v_f32"
        if "dpp" in op:
            return "v_dpp"
        return "v_int/bit"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_barrier"):
        return "s_wait/nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem:" + ("scratch" if op.startswith("scratch") or "buffer" in op else "global")
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and name in l and l.rstrip().endswith(":") or (l.startswith("_Z") and name in l and ": ;" in l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    for l in lines[start + 1:end]:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            m = re.match(r"^(\.LBB\d+_\d+):", s)
            if m:
                cur = m.group(1)
                blocks[cur] = []
            continue
        op = s.split()[0]
        blocks[cur].append(op)
    total = Counter(classify(o) for b in blocks.values() for o in b)
    n = sum(total.values())
    print(f"{name}: {n} instructions in {len(blocks)} blocks")
    for k, v in total.most_common():
        print(f"  {k:16s} {v:6d}")
    if "--blocks" in sys.argv:
        for b, ops in blocks.items():
            c = Counter(classify(o) for o in ops)
            print(f"{b:14s} {len(ops):5d}  " + " ".join(f"{k}={v}" for k, v in c.most_common(6)))


if __name__ == "__main__":
    main()
