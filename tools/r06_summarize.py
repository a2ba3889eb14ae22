"""Dev tool: turn a tools/profile_round6.sh output directory into the committed round-6 profile
files (kernel-trace excerpts, VALU and HBM-traffic summaries with the build digest).
    python tools/r06_summarize.py gpurun_out/<tag>"""
import csv, glob, json, os, subprocess, sys
from collections import defaultdict

OUT = sys.argv[1]
PROF = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")


def trace(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def gz(r):
    return int(r.get("Grid_Size_Z") or r.get("Grid_Z") or 1)


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


rows = trace(f"{OUT}/stats/run_kernel_trace.csv")
pk = [r for r in rows if "packet" in r["Kernel_Name"]]
# the timed region: the last 20-frame packet launch and the fix-up after it
i = max(k for k, r in enumerate(pk) if gz(r) == 20 and "packet_direct" in r["Kernel_Name"])
timed = pk[i:i + 2]
b = json.load(open(f"{OUT}/bench_prof.json"))
out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 --warmup 5 "
                  "--no-cpu-baseline --no-extras",
       "note": "the timed region is ONE 20-frame packet launch + its fix-up launch; the earlier "
               "32-frame launches are the clock warm-up and warm-up frames",
       "timed_launches": [{"kernel": r["Kernel_Name"][:60], "grid_z": gz(r),
                           "duration_us": dur(r) / 1e3} for r in timed],
       "bench_value": b["value"], "bench_ms_per_step": b["ms_per_step"],
       "bench_kernel_ms_per_launch": b["kernel_ms_per_launch"], "bench_parity": b["parity"]}
json.dump(out, open(f"{PROF}/r06_s20_timed_launch.json", "w"), indent=1)
print(json.dumps(out["timed_launches"]))
os.system(f"cp {OUT}/stats/run_kernel_stats.csv {PROF}/r06_c2_kernel_stats_s20.csv")
os.system(f"cp {OUT}/kt32/kt_kernel_stats.csv {PROF}/r06_c2_batch32_kernel_stats.csv")
os.system(f"cp {OUT}/pmc_c2/summary.json {PROF}/r06_pmc_c2_batch32_summary.json")
k32 = [dur(r) for r in trace(f"{OUT}/kt32/kt_kernel_trace.csv")
       if "packet_direct_kernel" in r["Kernel_Name"] and gz(r) == 32]
d32 = sum(k32) / len(k32)
here = os.path.dirname(os.path.abspath(__file__))
subprocess.run([sys.executable, f"{here}/valu_summary.py", f"{OUT}/pmc_c2/summary.json",
                "packet_direct_kernel<1, 128", str(d32), f"{PROF}/r06_c2_valu.json"], check=True)
subprocess.run([sys.executable, f"{here}/traffic_summary.py", f"{OUT}/pmc_c2/summary.json",
                f"{PROF}/pmc_c2_batch32.json", "c2", str(32 * 2073600 * 27),
                "packet_direct_kernel<1, 128"], check=True, capture_output=True)
subprocess.run([sys.executable, f"{here}/traffic_summary.py",
                f"{OUT}/tr_c5/librtamd/summary.json", f"{PROF}/r06_c5_traffic.json", "c5",
                str(20 * 8294400 * 27), "1, 34, false, false"], check=True, capture_output=True)
# glass: every kernel of the frame summed, per frame
base = f"{OUT}/tr_glass/librtamd"
tot, disp = defaultdict(float), defaultdict(set)
for p, name in (("p1", "FETCH_SIZE"), ("p2", "WRITE_SIZE")):
    for f in glob.glob(f"{base}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name:
                continue
            tot[(r["Kernel_Name"][:70], name)] += float(r["Counter_Value"])
            disp[(r["Kernel_Name"][:70], name)].add(r["Dispatch_Id"])
frames = len(disp[[k for k in disp if "wf_final_kernel" in k[0] and k[1] == "FETCH_SIZE"][0]])
fetch = sum(v for (k, n), v in tot.items() if n == "FETCH_SIZE") * 2048 / frames
write = sum(v for (k, n), v in tot.items() if n == "WRITE_SIZE") * 1024 / frames
alg = 2073600 * 27
g = {"config": "glass", "frames": frames, "fetch_bytes_corrected_per_frame": fetch,
     "write_bytes_per_frame": write, "hbm_bytes_per_frame": fetch + write,
     "alg_bytes_per_frame": alg, "traffic_over_alg": (fetch + write) / alg,
     "source_sha256": json.load(open(f"{base}/summary.json")).get("_build", {}).get("source_sha256"),
     "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
               "tools/profile_kernel.py glass (tools/traffic_passes.sh via "
               "tools/profile_round6.sh), every dispatch of the frame's kernels summed, per frame "
               "(frames = wf_final_kernel dispatches); FETCH doubled (gfx950)"}
json.dump(g, open(f"{PROF}/r06_glass_traffic.json", "w"), indent=1)
for f in ("r06_c2_valu.json", "pmc_c2_batch32.json", "r06_c5_traffic.json"):
    d = json.load(open(f"{PROF}/{f}"))
    print(f, {k: d.get(k) for k in ("valu_per_wave", "valu_issue_frac", "clock_ghz_measured",
                                     "traffic_over_alg", "source_sha256") if k in d})
print("glass traffic_over_alg", g["traffic_over_alg"])
