"""Evidence summary: every roofline figure in the bench line against the
rocprofv3 kernel trace (and HBM counters) of the same bench.py command
(tools/gpu_session.sh steps bench, prof, pmc).

The trace is taken WITHOUT name truncation, so template instances that share a
kernel name (the int32 and packed fused Golay reads, interp_tile_kernel<false>
and <true>, fp16 and fp32 decode+dequantize) are separate entries: no entry
carries another configuration's average.  HBM traffic per launch = FETCH_SIZE
x 2 (gfx950 tallies 128-B streaming reads at 64 B, MI355X_MICROARCH.md, HBM
section) + WRITE_SIZE, each from its own --pmc pass.

usage: python tools/rocprof_summary.py gpurun_out/<tag> profiles/<round>/<name>
  expects <tag>/bench.log (the JSON line), <tag>/prof/*kernel_trace.csv and
  optionally <tag>/pmc_fetch, <tag>/pmc_write counter collections.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import statistics
import sys

# bench-line path -> (kernel-name fragment, algorithmic bytes key in the line)
SECTIONS = {
    "roofline": ("golay_decode_kernel<true, true>", ("roofline", "bytes_per_launch"), ("kernel_ms", "decode")),
    "encode": ("golay_encode_kernel(", None, ("kernel_ms", "encode")),
    "fused_golay_decode": ("shim_read_golay_tiles_kernel<__half, true, false, 0, 0>", ("fused_golay_decode", "bytes_per_launch"),
                           ("fused_golay_decode", "kernel_ms")),
    "fused_golay_decode.packed": ("shim_read_golay_tiles_kernel<__half, true, true, 0, 0>",
                                  ("fused_golay_decode", "packed", "bytes_per_launch"),
                                  ("fused_golay_decode", "packed", "kernel_ms")),
    "fused_h84.plain": ("shim_read_bytes_tiles_kernel<__half, 2, true>",
                        ("fused_golay_decode", "hamming84", "plain", "bytes_per_launch"),
                        ("fused_golay_decode", "hamming84", "plain", "kernel_ms")),
    "fused_h84.interp": ("shim_read_h84_interp_kernel<__half, true, 2>",
                         ("fused_golay_decode", "hamming84", "interp", "bytes_per_launch"),
                         ("fused_golay_decode", "hamming84", "interp", "kernel_ms")),
    "golay_rows.decode": ("golay_decode_rows_reg_kernel<true", ("golay_rows", "bytes_per_launch"),
                          ("golay_rows", "kernel_ms", "decode")),
    "golay_rows.encode": ("golay_encode_rows_full_kernel", ("golay_rows", "bytes_per_launch"),
                          ("golay_rows", "kernel_ms", "encode")),
    "interp": ("interp_tile_kernel<false>", ("interp", "bytes_per_launch"), ("interp", "kernel_ms")),
    # the API call: the recording pass, then the fix-up launch -- from the first's start to the
    # second's end per call, as the bench's events around the calls see it
    "interp.api": (("interp_tile_kernel<true>", "interp_fixup_kernel"), ("interp", "api", "bytes_per_launch"),
                   ("interp", "api", "kernel_ms")),
    "interp.rec": ("interp_tile_kernel<true>", ("interp", "api", "bytes_per_launch"), None),
    "quantize_encode": ("quantize_encode_tile_kernel<__half", ("fused_quant", "quantize_encode", "bytes_per_launch"),
                        ("fused_quant", "quantize_encode", "kernel_ms")),
    "decode_dequant": ("decode_dequant_tile_kernel<__half>", ("fused_quant", "decode_dequant", "bytes_per_launch"),
                       ("fused_quant", "decode_dequant", "kernel_ms")),
    "decode_dequant_fp32": ("decode_dequant_tile_kernel<float>",
                            ("fused_quant", "decode_dequant_fp32", "bytes_per_launch"),
                            ("fused_quant", "decode_dequant_fp32", "kernel_ms")),
    "inject": ("inject_kernel<int, 24, false, true>", None, ("inject", "ms")),
}


def get(d, path):
    if path is None:
        return None
    for k in path:
        if d is None:
            return None
        d = d.get(k)
    return d


def trace_spans(src):
    spans = {}
    for p in glob.glob(os.path.join(src, "prof", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            spans.setdefault(r["Kernel_Name"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for v in spans.values():
        v.sort()
    return spans


def call_spans(spans, first, then):
    """Per launch of `first`: from its start to the end of the next `then` launch
    (a call of two kernels on one stream, timed as the bench times it)."""
    import bisect
    nxt = spans[then]
    starts = [a for a, _ in nxt]
    out = []
    for a, b in spans[first]:
        i = bisect.bisect_left(starts, b)
        if i < len(nxt):
            out.append(nxt[i][1] - a)
    return out


def counters(src, sub):
    per = {}
    for p in glob.glob(os.path.join(src, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return per


def pick(names, frag):
    hits = [n for n in names if frag in n]
    return hits[0] if len(hits) == 1 else (None if not hits else min(hits, key=len))


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    line = None
    for ln in open(os.path.join(src, "bench.log")):
        if ln.startswith("{"):
            line = json.loads(ln)
    spans = trace_spans(src)
    durs = {k: [b - a for a, b in v] for k, v in spans.items()}
    fetch, write = counters(src, "pmc_fetch"), counters(src, "pmc_write")
    out = {"source": src, "bench_line": os.path.join(dst, "bench.log"),
           "note": "rocprofv3 --kernel-trace without name truncation; median and mean over every launch of the "
                   "instance in the traced bench.py run (warm-up launches included); the bench line's figures "
                   "are means of dispatch-stamped launches, so rocprof_mean_vs_bench is the like-for-like check", "sections": {}}
    for sec, (frag, bytes_path, ms_path) in SECTIONS.items():
        if isinstance(frag, tuple):  # a call of two kernels: first start -> second end, per call
            names = [pick(durs, f) for f in frag]
            if None in names:
                continue
            d = call_spans(spans, names[0], names[1])
            name = " -> ".join(x.split("(")[0] for x in names)
            frag = frag[0]
        else:
            name = pick(durs, frag)
            if name is None:
                continue
            d = durs[name]
        bench_ms = get(line, ms_path)
        nbytes = get(line, bytes_path) if bytes_path else None
        if sec == "encode":
            nbytes = 7 * line["config"]["codewords_per_gpu"]
        e = {"kernel": name.split("(")[0], "launches": len(d), "median_us": statistics.median(d) / 1e3,
             "mean_us": statistics.fmean(d) / 1e3, "bench_us": bench_ms * 1e3 if bench_ms else None}
        if " -> " in e["kernel"]:
            e["note"] = ("a call of two launches: the trace's span from the first's start to the second's end "
                         "carries rocprofv3's per-dispatch completion gaps, which the un-profiled bench does not; "
                         "the recording kernel alone is the 'interp.rec' entry")
        if bench_ms:
            e["rocprof_median_vs_bench"] = statistics.median(d) / 1e6 / bench_ms - 1.0
            e["rocprof_mean_vs_bench"] = statistics.fmean(d) / 1e6 / bench_ms - 1.0
        if nbytes:
            e["algorithmic_bytes"] = nbytes
            e["frac_rocprof_median"] = nbytes / (statistics.median(d) * 1e-9) / 8e12
            e["frac_bench"] = nbytes / (bench_ms * 1e-3) / 8e12 if bench_ms else None
        fk, wk = pick(fetch, frag), pick(write, frag)
        if fk and wk:
            f = statistics.median(fetch[fk]) * 1024 * 2
            w = statistics.median(write[wk]) * 1024
            e.update({"fetch_bytes": f, "write_bytes": w, "hbm_bytes_per_launch": f + w})
            if nbytes:
                e["traffic_over_algorithmic"] = (f + w) / nbytes
        out["sections"][sec] = e
    for p in glob.glob(os.path.join(src, "prof", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(p, os.path.join(dst, "kernel_stats.csv"))
    for name in ("bench.log", "status.txt"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, name))
    with open(os.path.join(dst, "bench_vs_rocprof.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for sec, e in out["sections"].items():
        dm, da = e.get("rocprof_median_vs_bench"), e.get("rocprof_mean_vs_bench")
        print(f"{sec:28s} bench {e['bench_us'] or 0:8.2f} us  rocprof median {e['median_us']:8.2f} "
              f"({'' if dm is None else f'{dm * 100:+.1f}%'}) mean {e['mean_us']:8.2f} "
              f"({'' if da is None else f'{da * 100:+.1f}%'})  traffic/algo {e.get('traffic_over_algorithmic', 0):.3f}")
    dec = out["sections"].get("roofline", {})
    if "hbm_bytes_per_launch" in dec:
        with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                               "traffic.json"), "w") as fh:
            json.dump({"golay_decode_bytes_per_launch": dec["hbm_bytes_per_launch"],
                       "source": os.path.join(dst, "bench_vs_rocprof.json")}, fh, indent=1)


if __name__ == "__main__":
    main()
