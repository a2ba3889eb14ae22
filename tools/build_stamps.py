"""Dev tool: build the per-wave timestamp variant of the packet kernel (tools/stamps_patch.txt,
read by tools/wave_timeline.py), optionally with further replacements in rt_packet.hip.

    python tools/build_stamps.py NAME ['old text' 'new text' ...]

Writes tools/variants/NAME.so (git-ignored)."""
import os, subprocess, sys

here = os.path.dirname(os.path.abspath(__file__))
parts = open(os.path.join(here, "stamps_patch.txt")).read().split("@@@\n")
assert len(parts) % 2 == 0
pairs = [p.rstrip("\n") for p in parts]
name, extra = sys.argv[1], sys.argv[2:]
subprocess.check_call([sys.executable, os.path.join(here, "build_variant.py"), name,
                       "rt_packet.hip", *pairs, *extra])
