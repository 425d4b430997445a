"""A/B: H(8,4) decode+dequant unroll/grid (tools/exp/dequant_exp.hip) vs production, cold cache.
Build: make -C tools/exp libdequant.so    Run (GPU box): python tools/exp/run_dequant.py"""
import ctypes, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import ops
VP = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "libdequant.so"))
lib.dequant_exp.argtypes = [ctypes.c_int, ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_int, VP, VP]
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
rows, d = 8 * 4096 * 32, 128
g = torch.Generator().manual_seed(0)
cw = torch.randint(0, 256, (rows, d), generator=g, dtype=torch.uint8).to(dev)
sc = torch.rand(rows, generator=g).to(dev)
P = lambda t: VP(t.data_ptr())
for dt, fp16 in ((torch.float16, 1), (torch.float32, 0)):
    ref = torch.empty(rows, d, dtype=dt, device=dev)
    ops.decode_dequant_h84_into(cw, sc, ref, True, ops.new_stats(dev))
    out = torch.empty_like(ref)
    cases = {"prod": lambda: ops.decode_dequant_h84_into(cw, sc, out, True, ops.new_stats(dev))}
    for v in (1, 2, 4):
        for grid in (4096, 8192, 16384, 32768):
            cases[f"u{v}_g{grid}"] = (lambda v=v, grid=grid: lib.dequant_exp(
                v, fp16, P(cw), P(sc), P(out), rows, d, grid, P(ops.new_stats(dev)), s))
    ok = {}
    for kk, fn in cases.items():
        out.zero_(); fn(); torch.cuda.synchronize(); ok[kk] = torch.equal(out, ref)
    t = {kk: [] for kk in cases}
    for _ in range(7):
        for kk, fn in cases.items():
            junk.fill_(1)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); fn(); b.record(); torch.cuda.synchronize()
            t[kk].append(a.elapsed_time(b) * 1e3)
    byts = rows * (d * (1 + out.element_size()) + 4)
    print(dt)
    for kk, v in sorted(t.items(), key=lambda kv: statistics.median(kv[1]))[:8]:
        med = statistics.median(v)
        print(f"  {kk:12s} {med:7.1f} us {byts / med / 1e3:6.0f} GB/s ok={ok[kk]}")
    print(f"  prod         {statistics.median(t['prod']):7.1f} us")
