"""Per-kernel counter table from rocprofv3 --pmc passes (one directory per pass).

Each kernel (full name, template arguments included, so experiment variants in
one library stay apart) gets every counter's per-dispatch value summed over the
agent's blocks and averaged over its dispatches; with a --kernel-trace --stats
directory the average duration is added.  FETCH_SIZE / WRITE_SIZE are KiB;
hbm_bytes = 2 * FETCH_SIZE + WRITE_SIZE KiB (MI355X_MICROARCH.md, HBM section:
gfx950 tallies 128-B streaming reads at 64 B).

usage: python tools/pmc_table.py OUT.json PASS_DIR [PASS_DIR ...] [--stats STATS_DIR] [--match SUBSTR]
"""

from __future__ import annotations

import collections
import csv
import glob
import json
import sys


def load_pass(d, match):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = collections.defaultdict(dict)
    for (k, c), v in agg.items():
        out[k][c] = v / len(disp[(k, c)])
        out[k]["dispatches"] = len(disp[(k, c)])
    return out


def main():
    args = sys.argv[1:]
    stats_dir, match = None, None
    if "--stats" in args:
        i = args.index("--stats")
        stats_dir = args[i + 1]
        del args[i:i + 2]
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        del args[i:i + 2]
    out, dirs = args[0], args[1:]
    table = collections.defaultdict(dict)
    for d in dirs:
        for k, v in load_pass(d, match).items():
            table[k].update(v)
    if stats_dir:
        for f in glob.glob(f"{stats_dir}/**/*kernel_trace.csv", recursive=True):
            durs = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if match and match not in k:
                    continue
                durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for k, v in durs.items():
                table[k]["avg_ns"] = sum(v) / len(v)
                table[k]["calls"] = len(v)
    for k, v in table.items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            v["hbm_bytes"] = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
        if "SQ_LDS_BANK_CONFLICT" in v and "SQ_LDS_IDX_ACTIVE" in v:
            v["lds_conflict_share"] = v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1)
        if "SQ_WAIT_INST_ANY" in v and "SQ_WAVE_CYCLES" in v:
            v["wait_inst_any_share"] = v["SQ_WAIT_INST_ANY"] / max(v["SQ_WAVE_CYCLES"], 1)
    with open(out, "w") as f:
        json.dump({"source": dirs, "stats": stats_dir, "kernels": table}, f, indent=1, sort_keys=True)
    print(f"{len(table)} kernels -> {out}")


if __name__ == "__main__":
    main()
