"""Dev tool: turn the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_passes.sh into the per-launch
HBM byte count bench.py reports as roofline.traffic (profiles/pmc_<config>_frames.json).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): the derived counters are
in KiB; on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so it is doubled; WRITE_SIZE is
taken as is."""
import json, sys
src, dst, config, alg = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
sub = sys.argv[5] if len(sys.argv) > 5 else None  # kernel name substring (several variants ran)
d = json.load(open(src))
k = [n for n in d if not n.startswith("_") and (sub in n if sub else ("packet_direct_kernel" in n or "trace_kernel" in n))]
assert len(k) == 1, k
c = d[k[0]]
fetch = c["FETCH_SIZE"] * 1024 * 2
write = c["WRITE_SIZE"] * 1024
out = {"config": config, "kernel": k[0], "FETCH_SIZE_KiB": c["FETCH_SIZE"],
       "WRITE_SIZE_KiB": c["WRITE_SIZE"], "fetch_bytes_corrected": fetch, "write_bytes": write,
       "hbm_bytes_per_launch": fetch + write, "alg_bytes_per_launch": alg,
       "traffic_over_alg": (fetch + write) / alg,
       "source_sha256": d.get("_build", {}).get("source_sha256"),
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                 "tools/profile_kernel.py, averaged per dispatch; FETCH doubled (gfx950)"}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
