"""VALU roofline inputs of the injection kernels -> profiles/inject_valu.json.

Counters (rocprofv3 --pmc passes of tools/inject_pmc.py and of the VALU
microbenchmark tools/exp/run_valu_rate2.py, QUICK=1: tools/gpu_r06e.sh):

  SQ_INSTS_VALU          wave-level VALU instructions issued
  SQ_ACTIVE_INST_VALU2   quad-cycles in which a SIMD issued TWO VALU instructions
                         (gfx950 dual issue)
  SQ_BUSY_CYCLES         cycles with waves present, per shader engine (32 SEs):
                         the launch's length in shader clocks, at the clock it ran

A SIMD issues one wave64 VALU instruction per quad-cycle; some opcodes pair up
(dual issue, two in one quad-cycle).  So the VALU issue slots a launch used are
INSTS - VALU2, and the VALU-busy fraction is

    (INSTS - VALU2) / (SIMDs * SQ_BUSY_CYCLES / SEs / 4)

-- the counters and the launch's own clock, independent of the instruction count
the roofline's `achieved` comes from.  (gfx950's SQ_ACTIVE_INST_VALU equals
SQ_INSTS_VALU and SQ_THREAD_CYCLES_VALU equals 64 x SQ_INSTS_VALU for full waves:
neither measures cycles; round 5's "valu_busy" was 2 x the issue fraction.)

The peak the bench prices injection at is the issue-slot rate at the spec clock
for the kernel's own pairing: SIMDs * 2.4e9 / 4 / (1 - VALU2/INSTS) wave-
instructions per second.  The microbenchmark's pure single-opcode streams
calibrate the busy fraction a VALU-only loop reaches (its loop's scalar
instructions and the launch's ramp cost it ~10 %).

usage: python tools/inject_summary.py gpurun_out/r06e [profiles/r06]
"""
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M, V = 8 * 4096 * 32 * 43, 8 * 4096 * 32 * 128
SIMDS, SES, CLK = 256 * 4, 32, 2.4e9


def dispatches(d):
    """{dispatch id: {"name", counters..., "dur"}} of one rocprofv3 --pmc output directory."""
    per = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            e = per.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = int(r["Dispatch_Id"])
            if k in per:
                per[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return per


def busy(e):
    """VALU issue-slot busy fraction and the launch's clock from one dispatch's counters."""
    cycles = e["SQ_BUSY_CYCLES"] / SES
    slots = e["SQ_INSTS_VALU"] - e["SQ_ACTIVE_INST_VALU2"]
    return slots / (SIMDS * cycles / 4), cycles / e["dur"] if e.get("dur") else None


def summarise(per, match):
    es = [e for e in per.values() if match(e["name"]) and "SQ_ACTIVE_INST_VALU2" in e]
    if not es:
        return None
    med = {c: statistics.median(e[c] for e in es) for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU2",
                                                          "SQ_BUSY_CYCLES")}
    b = [busy(e) for e in es]
    return {"dispatches": len(es), "counters_median": med,
            "dual_issue_frac": med["SQ_ACTIVE_INST_VALU2"] / med["SQ_INSTS_VALU"],
            "valu_busy": statistics.median(x[0] for x in b),
            "clock_hz": statistics.median(x[1] for x in b if x[1]),
            "duration_s_under_pmc": statistics.median(e["dur"] for e in es if "dur" in e)}


OPS = ["v_add_u32", "v_xor_b32", "v_mul_lo_u32", "v_mul_hi_u32", "v_lshlrev_b32", "v_add3_u32",
       "v_bitop3_b32", "v_add_f32", "v_and_b32", "v_lshrrev_b32"]


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else None
    inj = dispatches(os.path.join(src, "inj_pmc3"))
    res = {"source": f"{src}: rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES "
                     "(+ SQ_THREAD_CYCLES_VALU) of tools/inject_pmc.py and tools/exp/run_valu_rate2.py",
           "kernels": {}}
    for name, golay in (("inject_kernel<int, 24, false, true>", True), ("inject_kernel<unsigned char, 8, false, true>", False)):
        s = summarise(inj, lambda n, name=name: name in n)
        if s is None:
            continue
        philox = M * 24 if golay else V * 8
        s["philox_per_launch"] = philox
        s["valu_insts_per_philox"] = s["counters_median"]["SQ_INSTS_VALU"] * 64 / philox
        s["issue_peak_wave_instr_per_s"] = SIMDS * CLK / 4 / (1 - s["dual_issue_frac"])
        res["kernels"][name] = s
    gol = res["kernels"].get("inject_kernel<int, 24, false, true>")
    if gol:
        res.update({"valu_insts_per_philox": gol["valu_insts_per_philox"], "valu_busy": gol["valu_busy"],
                    "dual_issue_frac": gol["dual_issue_frac"],
                    "issue_peak_wave_instr_per_s": gol["issue_peak_wave_instr_per_s"],
                    "nominal_peak_wave_instr_per_s": SIMDS * CLK / 2,
                    "peak_basis": "one wave64 VALU instruction per quad-cycle per SIMD at 2.4 GHz, dual-issued "
                                  "pairs (SQ_ACTIVE_INST_VALU2) sharing a slot; the nominal 2-cycle rate "
                                  "assumes every instruction pairs"})
    micro = dispatches(os.path.join(src, "valu_pmc3"))
    cal = {}
    for a in range(len(OPS)):
        for b in range(len(OPS)):
            tag = f"valu2_kernel<{a}, {b}, 16>"
            s = summarise(micro, lambda n, tag=tag: tag in n)
            if s:
                cal[OPS[a] if a == b else f"{OPS[a]}+{OPS[b]}"] = {
                    "dual_issue_frac": round(s["dual_issue_frac"], 4), "valu_busy": round(s["valu_busy"], 4),
                    "clock_hz": s["clock_hz"]}
    res["microbenchmark_W8_CH16"] = cal
    rates = os.path.join(src, "valu_rate2.json")
    if os.path.exists(rates):
        res["chains_sweep"] = json.load(open(rates))["summary"]
    out = json.dumps(res, indent=1)
    print(out)
    if dst:
        os.makedirs(dst, exist_ok=True)
        with open(os.path.join(dst, "inject_valu.json"), "w") as f:
            f.write(out)
        with open(os.path.join(REPO, "profiles", "inject_valu.json"), "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
