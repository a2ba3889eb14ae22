"""Dev tool: counter-derived VALU roofline of one kernel, from the rocprofv3 counter passes of
tools/pmc_passes.sh (summary.json) and the kernel's measured duration.

    python tools/valu_summary.py SUMMARY.json KERNEL_SUBSTR DURATION_NS OUT.json [FP64_RATES.txt]

SQ_ACTIVE_INST_VALU and SQ_WAVE_CYCLES count quad-cycles (MI355X_MICROARCH.md, constants
table); the capacity is 1024 SIMDs x duration x 2.4 GHz (the clock the FP64 peak is quoted at;
under load the chip runs lower, so fractions against 2.4 GHz are conservative).  Issue costs per
wave64 instruction: FP64 add/mul/fma 4 cycles, FP64 transcendental 16, other VALU 2 (SIMD-32),
from tools/micro/fp64_rates.hip on MI355X (profiles/r02_fp64_rates.txt)."""
import json
import sys

SIMDS, CLOCK = 1024, 2.4e9
FP64_PEAK_TFLOPS = 78.6  # 1024 SIMDs x 16 lanes x 2 flops x 2.4 GHz (FMA); FP32 vector / 2


def main():
    summ, sub, dur_ns, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    d = json.load(open(summ))
    (name, c), = [(k, v) for k, v in d.items() if sub in k and not k.startswith("_")]
    cap = SIMDS * dur_ns * 1e-9 * CLOCK
    # the clock the chip ran at during the passes: GRBM_GUI_ACTIVE (GPU-busy cycles, summed
    # over the 8 XCDs) / 8 / duration; the SIMD capacity at that clock is what the issue
    # cycles are measured against
    clk = c["GRBM_GUI_ACTIVE"] / 8 / (dur_ns * 1e-9) if c.get("GRBM_GUI_ACTIVE") else CLOCK
    cap_clk = SIMDS * dur_ns * 1e-9 * clk
    f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_FMA_F64"]
    trans = c["SQ_INSTS_VALU_TRANS_F64"]
    other = c["SQ_INSTS_VALU"] - f64 - trans
    issue = 4 * f64 + 16 * trans + 2 * other
    flops = 64 * (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"]) + \
        128 * c["SQ_INSTS_VALU_FMA_F64"]
    waves = c["SQ_WAVES"]
    res = {
        "kernel": name, "duration_ns": dur_ns, "waves": waves,
        "valu_per_wave": round(c["SQ_INSTS_VALU"] / waves, 1),
        "salu_per_wave": round(c["SQ_INSTS_SALU"] / waves, 1),
        "fp64_share_of_valu": round((f64 + trans) / c["SQ_INSTS_VALU"], 4),
        "clock_ghz_measured": round(clk / 1e9, 4),
        "valu_issue_frac": round(issue / cap_clk, 4),
        "valu_issue_frac_at_2p4ghz": round(issue / cap, 4),
        "active_inst_valu_ratio": round(4 * c["SQ_ACTIVE_INST_VALU"] / cap_clk, 4),
        "valu_lane_activity": (round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_INSTS_VALU"]), 4)
                               if c.get("SQ_THREAD_CYCLES_VALU") else None),
        "fp64_counted_tflops": round(flops / (dur_ns * 1e-9) / 1e12, 3),
        "fp64_counted_frac": round(flops / (dur_ns * 1e-9) / 1e12 / FP64_PEAK_TFLOPS, 4),
        "definitions": {
            "valu_issue_frac": "issue cycles (4 x FP64 add/mul/fma + 16 x FP64 transcendental + "
                               "2 x other VALU wave-instructions, the per-class costs measured "
                               "by tools/micro) / SIMD cycles (1024 SIMDs x duration x the "
                               "measured clock, clock_ghz_measured = GRBM_GUI_ACTIVE / 8 / "
                               "duration): the share of SIMD cycles the kernel's VALU "
                               "instructions occupy, a fraction <= 1",
            "valu_issue_frac_at_2p4ghz": "the same issue cycles against the 2.4 GHz peak clock",
            "active_inst_valu_ratio": "4 x SQ_ACTIVE_INST_VALU / the measured-clock SIMD cycles: "
                                      "NOT a busy fraction (the counter is not SIMD-busy cycles; "
                                      "it exceeds 1 on saturated kernels), kept for comparison "
                                      "with earlier rounds' valu_busy_frac",
            "valu_lane_activity": "SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU): the mean share of "
                                  "a wave's 64 lanes active per VALU instruction (divergence)",
            "clock_note": "GRBM_GUI_ACTIVE also counts the dispatch around a short kernel, so for "
                          "kernels of tens of us (the glass level kernels' deeper levels) "
                          "clock_ghz_measured overstates the clock; valu_issue_frac_at_2p4ghz "
                          "is the bound there",
            "fp64_counted_tflops": "64 flops per FP64 add/mul and 128 per FMA wave-instruction "
                                   "(all lanes counted) / duration, against 78.6 TF",
        },
        "counters": c,
        "source_sha256": d.get("_build", {}).get("source_sha256"),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("counters", "definitions")}))


if __name__ == "__main__":
    main()
