"""VALU issue cost vs independent work in flight (tools/exp/valu_rate2.hip):
cycles per wave-instruction per SIMD (at the 2.4 GHz clock) for chains per lane
CH in {1, 2, 4, 8, 16} x waves per SIMD W in {1, 2, 4, 8}.  A flat value over
the large-CH, large-W corner is the issue cost; the CH=1, W=1 value is latency.
usage (GPU box): python tools/exp/run_valu_rate2.py [out.json]"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libvalu2.so"))
lib.valu2_rate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.valu2_pair.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
OPS = ["v_add_u32", "v_xor_b32", "v_mul_lo_u32", "v_mul_hi_u32", "v_lshlrev_b32", "v_add3_u32",
       "v_bitop3_b32", "v_add_f32", "v_and_b32", "v_lshrrev_b32"]
CUS, SIMDS, CLK = 256, 4, 2.4e9
PER_LANE = 8192  # instructions per lane per launch (iters x chains)
out = torch.empty(CUS * 8 * 256, dtype=torch.int32, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
res = {}
for p in range(lib.valu2_pairs()):
    a, b = ctypes.c_int(), ctypes.c_int()
    lib.valu2_pair(p, ctypes.byref(a), ctypes.byref(b))
    name = OPS[a.value] if a.value == b.value else f"{OPS[a.value]}+{OPS[b.value]}"
    res[name] = {}
    quick = os.environ.get("QUICK") == "1"  # the W8 CH16 corner only (counter passes)
    for w in ((8,) if quick else (1, 2, 4, 8)):
        blocks = CUS * w  # one 256-thread workgroup = one wave per SIMD
        for ch in ((16,) if quick else (1, 2, 4, 8, 16)):
            iters = PER_LANE // ch
            for _ in range(2):
                assert lib.valu2_rate(p, ch, ctypes.c_void_p(out.data_ptr()), blocks, iters, s) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lib.valu2_rate(p, ch, ctypes.c_void_p(out.data_ptr()), blocks, iters, s)
            e1.record()
            torch.cuda.synchronize()
            sec = e0.elapsed_time(e1) / 5 * 1e-3
            instrs = blocks * 4 * iters * ch  # wave-instructions
            cyc = sec * CLK * CUS * SIMDS / instrs
            res[name][f"W{w}_CH{ch}"] = round(cyc, 3)
    row = res[name]
    print(f"{name:28s} " + " ".join(f"{k}={v:5.2f}" for k, v in row.items()), flush=True)
summary = {}
for name, row in ({} if os.environ.get("QUICK") == "1" else res).items():
    corner = [row[f"W{w}_CH{c}"] for w in (4, 8) for c in (4, 8, 16)]
    summary[name] = {"issue_cycles": min(corner), "corner_spread": max(corner) - min(corner),
                     "latency_cycles_W1_CH1": row["W1_CH1"]}
doc = {"what": "cycles per wave64 VALU instruction per SIMD at 2.4 GHz, vs chains per lane (CH) and waves per SIMD (W)",
       "source": "tools/exp/valu_rate2.hip, tools/exp/run_valu_rate2.py", "rates": res, "summary": summary}
print(json.dumps(summary))
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump(doc, f, indent=1)
