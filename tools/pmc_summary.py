"""Summarise a tools/gpu_check.sh run into profiles/<round>/ and profiles/traffic.json.

HBM traffic per launch = FETCH_SIZE * 2 (gfx950 tallies 128-B streaming reads
at 64 B, MI355X_MICROARCH.md section HBM) + WRITE_SIZE, both in KiB, from two
separate --pmc passes.  The median over the profiled launches of each kernel
is reported next to the kernel's algorithmic bytes.

usage: python tools/pmc_summary.py gpurun_out/r01c profiles/r01
       python tools/pmc_summary.py --variants gpurun_out/<tag> profiles/<round>/fused_variants
"""

from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M = 8 * 4096 * 32 * 43  # codewords of the bench workload
ALGO = {"golay_decode_kernel": 8 * M, "golay_encode_kernel": 7 * M,
        "golay_decode_packed_kernel": 4.625 * M, "golay_decode_packed_staged_kernel": 4.625 * M,
        "golay_decode_packed_wave_kernel": 4.625 * M,
        "golay_encode_packed_kernel": 4.5 * M,
        # per-head rows: 128 nibble bytes + 43 codewords per row
        "golay_encode_rows_reg_kernel": 300 * (M // 43), "golay_decode_rows_reg_kernel": 300 * (M // 43),
        # fused shim read, K+V token rows: int32 (172 + 4 + 256 B) then packed (129 + 4 + 256 B)
        "shim_read_golay_tiles_kernel[int32]": 432 * 2 * (M // 43),
        "shim_read_golay_tiles_kernel[packed]": 389 * 2 * (M // 43),
        # fused shim read, Hamming(8,4) K+V token rows: 128 + 4 + 256 B
        "shim_read_bytes_tiles_kernel": 388 * 2 * (M // 43),
        "shim_read_h84_interp_kernel": 388 * 2 * (M // 43)}
# kernels the bench launches in two configurations under one (truncated) name:
# the first half of the launches is the first configuration
SPLIT = {"shim_read_golay_tiles_kernel": ("[int32]", "[packed]")}


def counters(path):
    per = {}
    for r in sorted(csv.DictReader(open(path)), key=lambda r: int(r.get("Dispatch_Id", 0) or 0)):
        per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    for name, tags in SPLIT.items():
        if name in per:
            v = per.pop(name)
            h = len(v) // 2
            per[name + tags[0]], per[name + tags[1]] = v[:h], v[h:]
    return per


# fused-read variants traced one per run (tools/gpu_read_variants.sh): the
# variant's algorithmic bytes per launch (K+V token rows of [8,4096,32,128])
VARIANTS = {"golay": ("shim_read_golay_tiles_kernel", 432), "golay_packed": ("shim_read_golay_tiles_kernel", 389),
            "hamming84": ("shim_read_bytes_tiles_kernel", 388), "hamming84_interp": ("shim_read_h84_interp_kernel", 388)}


def variants(src, dst):
    os.makedirs(dst, exist_ok=True)
    out = {"source": src, "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1",
           "driver": "tools/exp/run_read_ab.py, one variant per rocprofv3 run", "variants": {}}
    for var, (kern, per_row) in VARIANTS.items():
        d = os.path.join(src, var)
        if not os.path.isdir(d):
            continue
        fetch = counters(glob.glob(os.path.join(d, "pmc_fetch", "*counter_collection.csv"))[0])
        write = counters(glob.glob(os.path.join(d, "pmc_write", "*counter_collection.csv"))[0])
        stats_csv = glob.glob(os.path.join(d, "prof", "*kernel_stats.csv"))[0]
        shutil.copy(stats_csv, os.path.join(dst, var + "_kernel_stats.csv"))
        stats = {r["Name"]: r for r in csv.DictReader(open(stats_csv))}
        name = next(k for k in stats if kern in k)
        fk = next(k for k in fetch if kern in k)
        wk = next(k for k in write if kern in k)
        f = statistics.median(fetch[fk]) * 1024 * 2
        w = statistics.median(write[wk]) * 1024
        algo = per_row * 2 * (M // 43)
        ns = float(stats[name]["AverageNs"])
        # the timed launches alone: the trace's last ROUNDS dispatches (the
        # average above also counts the driver's warm-up calls)
        trace = glob.glob(os.path.join(d, "prof", "*kernel_trace.csv"))[0]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                for r in sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Dispatch_Id"]))
                if kern in r["Kernel_Name"]]
        rounds = int(os.environ.get("ROUNDS", "20"))
        timed = durs[-rounds:]
        med = statistics.median(timed)
        out["variants"][var] = {"kernel": name, "avg_ns": ns, "calls": int(stats[name]["Calls"]),
                                "median_ns_timed": med, "timed_launches": len(timed),
                                "frac_of_8tbs_timed": algo / med / 8e3,
                                "algorithmic_bytes": algo, "fetch_bytes": f, "write_bytes": w,
                                "hbm_bytes_per_launch": f + w, "traffic_over_algorithmic": (f + w) / algo,
                                "achieved_tbs": algo / ns / 1e3, "frac_of_8tbs": algo / ns / 8e3}
    with open(os.path.join(dst, "pmc_variants.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


def main():
    if sys.argv[1] == "--variants":
        return variants(sys.argv[2], sys.argv[3])
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    fetch = counters(glob.glob(os.path.join(src, "pmc_fetch", "*counter_collection.csv"))[0])
    write = counters(glob.glob(os.path.join(src, "pmc_write", "*counter_collection.csv"))[0])
    stats_csv = glob.glob(os.path.join(src, "prof", "*kernel_stats.csv"))[0]
    shutil.copy(stats_csv, os.path.join(dst, "kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(stats_csv))}
    out = {"source": src, "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1",
           "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        f = statistics.median(fetch[k]) * 1024 * 2
        w = statistics.median(write[k]) * 1024
        entry = {"fetch_bytes": f, "write_bytes": w, "hbm_bytes_per_launch": f + w}
        if k in ALGO:
            entry["algorithmic_bytes"] = ALGO[k]
            entry["traffic_over_algorithmic"] = (f + w) / ALGO[k]
        base = k.split("[")[0]
        if base in stats:  # (a split kernel's stats cover both configurations)
            entry["avg_ns"] = float(stats[base]["AverageNs"])
            entry["calls"] = int(stats[base]["Calls"])
        out["kernels"][k] = entry
    with open(os.path.join(dst, "pmc_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    dec = out["kernels"].get("golay_decode_kernel", {})
    if dec:
        with open(os.path.join(REPO, "profiles", "traffic.json"), "w") as fh:
            json.dump({"golay_decode_bytes_per_launch": dec["hbm_bytes_per_launch"],
                       "source": os.path.join(dst, "pmc_summary.json")}, fh, indent=1)
    for name in ("bench.log", "status.txt"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, name))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
