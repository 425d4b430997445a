"""A/B: interpolation geometry (tools/exp/interp_exp.hip) vs production, cold cache, interleaved.
Build: make -C tools/exp libinterp.so    Run (GPU box): python tools/exp/run_interp.py"""
import ctypes, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import ops
VP = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "libinterp.so"))
lib.interp_exp.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, VP]
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
B, L, H, D = 8, 4096, 32, 128
g = torch.Generator().manual_seed(0)
q = torch.randint(0, 16, (B, L, H, D), generator=g, dtype=torch.uint8).to(dev)
err = (torch.rand(B, L, H, D, generator=g) < 0.01).to(torch.uint8).mul_(2).to(dev)
n = q.numel(); chunks = H * D // 16
ref = torch.empty_like(q); ops.interpolate_into(q.view(-1), err.view(-1), ref.view(-1), B, L, H * D)
out = torch.empty_like(q)
P = lambda t: VP(t.data_ptr())
cases = {"prod": lambda: ops.interpolate_into(q.view(-1), err.view(-1), out.view(-1), B, L, H * D)}
for v in range(8):
    R = {0: 8, 1: 8, 2: 8, 3: 16, 4: 16, 5: 16, 6: 4, 7: 8}[v]
    items = B * (L // R) * chunks
    for grid in (sorted({items // 256, 4096, 8192, 16384}) if v in (0, 3, 7) else [4096]):
        cases[f"v{v}_g{grid}"] = (lambda v=v, grid=grid: lib.interp_exp(v, P(q), P(err), P(out), B, L, chunks, grid, s))
ok = {}
for kk, fn in cases.items():
    out.zero_(); fn(); torch.cuda.synchronize(); ok[kk] = torch.equal(out, ref)
t = {kk: [] for kk in cases}
for _ in range(9):
    for kk, fn in cases.items():
        junk.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize()
        t[kk].append(a.elapsed_time(b) * 1e3)
for kk, v in sorted(t.items(), key=lambda kv: statistics.median(kv[1])):
    med = statistics.median(v)
    print(f"{kk:14s} {med:7.1f} us {3 * n / med / 1e3:6.0f} GB/s ok={ok[kk]}")
