"""Store-shape ceiling study (tools/exp/store_ceiling.hip).

Write-only streams of 537 MB (the fused Golay read's output size) and the fused
read's own byte mix (2816 B read + 4096 B written per 16-row tile, 131,072
tiles), across store width per lane (4/8/16 B), nt vs plain stores, workgroup
size, waves per CU (persistent grids, or full grids capped by dynamic LDS) and
unit shape (grid-stride 64·W bytes vs 4 KiB per wave).

Per configuration: median over 5 repetitions of 8 back-to-back launches timed
with HIP events.  Prints one line per configuration and the best of each group;
writes JSON to argv[1] if given.
"""
import ctypes
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
VP, U32, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
lib = ctypes.CDLL(os.path.join(HERE, "libstore.so"))
lib.store_probe.argtypes = [VP, VP, U32, U32, U32, I, I, I, I, I, I, VP]
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream()
sp = VP(stream.cuda_stream)
NCU = torch.cuda.get_device_properties(0).multi_processor_count
WBYTES = 131072 * 4096
src = torch.empty(131072 * 2816, dtype=torch.uint8, device=dev).random_(0, 256)
dst = torch.empty(WBYTES, dtype=torch.uint8, device=dev)
LDS_CU = 160 * 1024


def run(rch, wch, units, w, nt, pf, bs, grid, lds, reps=8, rounds=5):
    args = (VP(src.data_ptr()), VP(dst.data_ptr()), rch, wch, units, w, nt, pf, bs, grid, lds, sp)
    rc = lib.store_probe(*args)
    if rc:
        return None
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            lib.store_probe(*args)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return statistics.median(ts)


def geometries(bs, waves_total):
    """(label, grid, lds): persistent grids at 8/16/32 waves per CU, and full
    grids (one wave per unit) with workgroups per CU capped through LDS."""
    wpw = bs // 64
    out = []
    for wpc in (8, 16, 32):
        if wpc >= wpw:
            out.append((f"persist {wpc:2d}w/CU", NCU * wpc // wpw, 0))
    full = min((waves_total + wpw - 1) // wpw, 1 << 20)
    for wpc in (8, 16):
        wg = max(1, wpc // wpw)
        out.append((f"full    {wpc:2d}w/CU", full, (LDS_CU // wg) & ~1023))
    out.append(("full    hw  w/CU", full, 0))
    return out


results = []


def case(kind, rch, wch, w, nt, pf, bs):
    units = WBYTES // wch
    for label, grid, lds in geometries(bs, units):
        if grid > 1 << 20:
            continue
        us = run(rch, wch, units, w, nt, pf, bs, grid, lds)
        if us is None:
            print(f"{kind} skip w{w} nt{nt} bs{bs} {label} (launch failed)", flush=True)
            continue
        byts = units * (rch + wch)
        rate = byts / us / 1e3
        rec = dict(kind=kind, rch=rch, wch=wch, w=w, nt=nt, pf=pf, bs=bs, geom=label, grid=grid, lds=lds,
                   us=round(us, 2), gbps=round(rate, 1))
        results.append(rec)
        print(f"{kind:5s} W={w:2d} nt={nt} pf={pf} wch={wch:5d} bs={bs:4d} {label} grid={grid:6d}: "
              f"{us:7.1f} us {rate:6.0f} GB/s", flush=True)


for w in (4, 8, 16):
    for nt in (1, 0):
        for wch in sorted({64 * w, 4096}):
            for bs in (256, 512, 1024):
                case("write", 0, wch, w, nt, 0, bs)
for w in (16, 8, 4):
    for pf in (1, 0):
        for bs in (256, 512):
            case("mix", 2816, 4096, w, 1, pf, bs)

for kind in ("write", "mix"):
    rs = sorted((r for r in results if r["kind"] == kind), key=lambda r: -r["gbps"])
    print(f"--- best {kind}:")
    for r in rs[:8]:
        print("   ", r)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump(dict(ncu=NCU, results=results), f, indent=1)
