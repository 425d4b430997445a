"""A/B: fp16 quantize+H84 encode variants (tools/exp/quant_exp.hip) vs production, cold cache.
Build: make -C tools/exp libquant.so    Run (GPU box): python tools/exp/run_quant.py"""
import ctypes, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import ops, _lib
VP = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "libquant.so"))
lib.quant_exp.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int, VP]
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
rows, d = 8 * 4096 * 32, 128
g = torch.Generator().manual_seed(0)
x = torch.randn(rows, d, generator=g).to(torch.float16).to(dev)
cw_ref = torch.empty(rows, d, dtype=torch.uint8, device=dev); sc_ref = torch.empty(rows, device=dev)
ops.quantize_encode_rows_into(x, _lib.CODEC_H84, cw_ref, sc_ref, "mul_inv7")
cw = torch.empty_like(cw_ref); sc = torch.empty_like(sc_ref)
P = lambda t: VP(t.data_ptr())
cases = {"prod": lambda: ops.quantize_encode_rows_into(x, _lib.CODEC_H84, cw, sc, "mul_inv7")}
for v in range(7):
    for grid in ((8192, 16384, 32768, 65536) if v in (1, 3) else ()):
        cases[f"v{v}_g{grid}"] = (lambda v=v, grid=grid: lib.quant_exp(v, P(x), P(cw), P(sc), rows, grid, s))
ok = {}
for kk, fn in cases.items():
    cw.zero_(); sc.zero_(); fn(); torch.cuda.synchronize()
    ok[kk] = torch.equal(cw, cw_ref) and torch.equal(sc, sc_ref)
t = {kk: [] for kk in cases}
for _ in range(9):
    for kk, fn in cases.items():
        junk.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize()
        t[kk].append(a.elapsed_time(b) * 1e3)
byts = rows * (3 * d + 4)
for kk, v in sorted(t.items(), key=lambda kv: statistics.median(kv[1])):
    med = statistics.median(v)
    print(f"{kk:12s} {med:7.1f} us {byts / med / 1e3:6.0f} GB/s ok={ok[kk]}")
