"""Fused-read byte mix (2816 B read + 4096 B written per 16-row tile, 131,072
tiles) by work distribution (tools/exp/store_ceiling.hip):

- stride: persistent grid, wave w takes tiles w, w + nwaves, ... (the fused
  read kernels' scheme until round 3);
- chunk P: wave w takes the P consecutive tiles [w P, w P + P), grid sized to
  cover every tile once (workgroups retire and are replaced in dispatch order);

each with and without a 32 KiB table copied into LDS per workgroup (the fused
Golay read's spread tables), at 8 and 16 waves per CU (dynamic LDS caps the
workgroups per CU).  16-B nt stores, next tile's loads issued before stores.
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
lib.store_probe_mode.argtypes = [U32, U32, VP]
dev = torch.device("cuda:0")
sp = VP(torch.cuda.current_stream().cuda_stream)
NCU = torch.cuda.get_device_properties(0).multi_processor_count
UNITS, RCH, WCH = 131072, 2816, 4096
src = torch.empty(UNITS * RCH, dtype=torch.uint8, device=dev).random_(0, 256)
dst = torch.empty(UNITS * WCH, dtype=torch.uint8, device=dev)
table = torch.empty(32768, dtype=torch.uint8, device=dev).random_(0, 256)
LDS_CU = 160 * 1024


def timed(args, reps=8, rounds=5):
    if lib.store_probe(*args):
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


lib.store_probe_fix.argtypes = [VP, VP, U32, U32, I, I, VP]
results = []


def timed_fix(per, grid, lds, reps=8, rounds=5):
    args = (VP(src.data_ptr()), VP(dst.data_ptr()), UNITS, per, grid, lds, sp)
    if lib.store_probe_fix(*args):
        return None
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            lib.store_probe_fix(*args)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return statistics.median(ts)


# fixed VMEM count per iteration (probe_fix): the loop waits for its loads only
for wpc in (8, 12, 16, 24, 32):
    wg = wpc // 4
    lds = (LDS_CU // wg) & ~1023
    for per in (0, 1, 2, 4, 8, 16):
        waves = NCU * wpc if per == 0 else (UNITS + per - 1) // per
        grid = (waves + 3) // 4
        us = timed_fix(per, grid, lds)
        gbps = UNITS * (RCH + WCH) / us / 1e3
        mode = "stride " if per == 0 else f"chunk{per:2d}"
        results.append(dict(fix=1, bs=256, wpc=wpc, per=per, grid=grid, lds=lds, us=round(us, 2), gbps=round(gbps, 1)))
        print(f"FIX bs=256 {wpc:2d}w/CU {mode} grid={grid:6d}: {us:7.1f} us {gbps:6.0f} GB/s", flush=True)
if os.environ.get("FIXONLY"):
    TABS = ()
else:
    TABS = (0, 32768)
for tab in TABS:
    for bs in (256, 512):
        wpw = bs // 64
        for wpc in (8, 16):
            wg = max(1, wpc // wpw)
            lds = max(tab, (LDS_CU // wg) & ~1023)
            for per in (0, 1, 2, 4, 8, 16, 32):
                waves = NCU * wpc if per == 0 else (UNITS + per - 1) // per
                grid = (waves + wpw - 1) // wpw
                lib.store_probe_mode(per, tab, VP(table.data_ptr()))
                us = timed((VP(src.data_ptr()), VP(dst.data_ptr()), RCH, WCH, UNITS, 16, 1, 1, bs, grid, lds, sp))
                mode = "stride " if per == 0 else f"chunk{per:2d}"
                if us is None:
                    print(f"tab={tab:5d} bs={bs} {wpc:2d}w/CU {mode}: launch failed", flush=True)
                    continue
                gbps = UNITS * (RCH + WCH) / us / 1e3
                results.append(dict(tab=tab, bs=bs, wpc=wpc, per=per, grid=grid, lds=lds, us=round(us, 2),
                                    gbps=round(gbps, 1)))
                print(f"tab={tab:5d} bs={bs} {wpc:2d}w/CU {mode} grid={grid:6d}: {us:7.1f} us {gbps:6.0f} GB/s",
                      flush=True)
lib.store_probe_mode(0, 0, None)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump(dict(ncu=NCU, results=results), f, indent=1)
