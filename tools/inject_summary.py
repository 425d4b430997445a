"""VALU roofline inputs of the injection kernels from rocprofv3 counter passes
(tools/gpu_r05.sh, tools/inject_pmc.py) -> profiles/inject_valu.json.

SQ_INSTS_VALU counts wave-level VALU instructions; a wave instruction covers
64 lanes, so lane-instructions per Philox = SQ_INSTS_VALU * 64 / Philox per
launch (Golay: M * 24, Hamming(8,4): V * 8).  SQ_ACTIVE_INST_VALU counts the
quad-cycles in which a SIMD issued VALU work, so VALU-busy = 4 *
SQ_ACTIVE_INST_VALU / (SIMDs * cycles of the launch), the cycles taken from the
launch's kernel-trace duration at the 2.4 GHz shader clock.

usage: python tools/inject_summary.py gpurun_out/<tag> [profiles/<round>]"""
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M, V = 8 * 4096 * 32 * 43, 8 * 4096 * 32 * 128
SIMDS, CLK = 256 * 4, 2.4e9


def rows(d):
    out = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        out += list(csv.DictReader(open(p)))
    return out


KERNEL = "_ZN5kvecc13inject_kernelIiLi24ELb0ELb1EEEvPKT_PS1_PhNS_10InjectArgsEPm"  # inject_kernel<int, 24, false, true>


def isa_mix():
    """Opcode shares of the Golay injection kernel's VALU instructions, from its
    gfx950 disassembly (hipcc -S of csrc/inject.hip)."""
    import collections
    import subprocess
    import tempfile
    pkg = os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd")
    with tempfile.TemporaryDirectory() as t:
        asm = os.path.join(t, "inject.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                               "-I" + os.path.join(REPO, "include"), "--cuda-device-only", "-S",
                               os.path.join(pkg, "csrc", "inject.hip"), "-o", asm],
                              stderr=subprocess.DEVNULL)
        text = open(asm).read()
    body = text[text.index(KERNEL + ":"):]
    body = body[:body.index(".Lfunc_end")]
    ops = collections.Counter(ln.split()[0].split("_e32")[0].split("_e64")[0]
                              for ln in map(str.strip, body.splitlines()) if ln.startswith("v_"))
    tot = sum(ops.values())
    return {k: v / tot for k, v in ops.most_common()}


def mix_peak(mix, rates):
    """Wave-instructions per second the chip issues for this opcode mix: every
    opcode at its measured issue cost (tools/exp/run_valu_rate.py), opcodes
    not measured at the 4-cycle cost of the 32-bit integer VOP3 ops."""
    cyc = {k.split("(")[0]: v["cycles_per_wave_instr_per_simd"] for k, v in rates.items()}
    per = sum(share * cyc.get(op, 4.15) for op, share in mix.items())
    return SIMDS * CLK / per, per


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else None
    rates_path = os.path.join(REPO, "profiles", "r05", "valu_rate.json")
    per = {}  # (dispatch id) -> {counter: value, name, dur}
    for d in sorted(glob.glob(os.path.join(src, "inj_pmc*"))):
        for r in rows(d):
            if "inject" not in r["Kernel_Name"]:
                continue
            key = (os.path.basename(d), int(r["Dispatch_Id"]))
            e = per.setdefault(key, {"name": r["Kernel_Name"]})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    trace = {}
    for p in glob.glob(os.path.join(src, "inj_trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if "inject" in r["Kernel_Name"]:
                trace.setdefault(r["Kernel_Name"], []).append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    res = {"source": f"{src} (rocprofv3 --pmc passes of tools/inject_pmc.py)", "kernels": {}}
    for name in sorted({e["name"] for e in per.values()}):
        es = [e for e in per.values() if e["name"] == name]
        golay = "inject_kernel<int" in name
        philox = M * 24 if golay else V * 8
        med = {c: statistics.median(e[c] for e in es if c in e)
               for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVES", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES",
                         "SQ_BUSY_CYCLES") if any(c in e for e in es)}
        k = {"philox_per_launch": philox, "counters_median": med}
        if "SQ_INSTS_VALU" in med:
            k["valu_insts_per_philox"] = med["SQ_INSTS_VALU"] * 64 / philox
        durs = [t for n, ts in trace.items() if n == name for t in ts]
        if durs:
            dur = statistics.median(durs)
            k["duration_s"] = dur
            if "SQ_ACTIVE_INST_VALU" in med:
                k["valu_busy"] = 4 * med["SQ_ACTIVE_INST_VALU"] / (SIMDS * dur * CLK)
            if "SQ_INSTS_VALU" in med:
                k["valu_issue_frac"] = med["SQ_INSTS_VALU"] / dur / (SIMDS * CLK / 2)
        res["kernels"][name.split("(")[0]] = k
    gol = [k for n, k in res["kernels"].items() if "inject_kernel<int" in n]
    if gol and "valu_insts_per_philox" in gol[0]:
        res["valu_insts_per_philox"] = gol[0]["valu_insts_per_philox"]
        res["valu_busy"] = gol[0].get("valu_busy")
    if os.path.exists(rates_path):
        mix = isa_mix()
        peak, cyc = mix_peak(mix, json.load(open(rates_path)))
        res["isa_mix"] = {k: round(v, 4) for k, v in mix.items() if v >= 0.002}
        res["mix_cycles_per_wave_instr"] = cyc
        res["mix_peak_wave_instr_per_s"] = peak
        res["nominal_peak_wave_instr_per_s"] = SIMDS * CLK / 2
        res["valu_rates"] = rates_path
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
