"""Dev tool: per-kernel VGPRs / AGPRs / scratch / occupancy of the in-tree HIP sources (compiler
remarks, -Rpass-analysis=kernel-resource-usage).   python tools/kernel_resources.py [src ...]"""
import os, re, subprocess, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from raytracingengine_amd import build as B

for src in sys.argv[1:] or [s for s in B.SOURCES if s.endswith(".hip")]:
    r = subprocess.run([B.HIPCC, *B.HIP_FLAGS, *B.EXTRA_FLAGS.get(src, []),
                        f"-I{os.path.join(B.ROOT, 'include')}", "-c", "-o", os.devnull,
                        os.path.join(B.CSRC, src), "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
    cur = None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            if cur:
                print(src, *cur)
            cur = [v[:70]]
        else:
            cur.append(f"{k.split()[0]}={v}")
    if cur:
        print(src, *cur)
