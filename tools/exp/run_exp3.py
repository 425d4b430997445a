"""A/B: decode refinements (tools/exp/golay_exp3.hip) vs production and exp2 best."""
import ctypes, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
sys.path.insert(0, HERE)
import torch
from run_exp import tables
VP = ctypes.c_void_p
lib3 = ctypes.CDLL(os.path.join(HERE, "libexp3.so"))
lib3.exp3_decode.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, VP, VP, ctypes.c_int, VP]
lib2 = ctypes.CDLL(os.path.join(HERE, "libexp2.so"))
lib2.exp2_golay.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, VP, VP, ctypes.c_int, VP]
from kvecc import ops
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
tab = tables(dev)
g = torch.Generator().manual_seed(0)
x = torch.randint(0, 16, (8, 4096, 32, 128), generator=g, dtype=torch.uint8).to(dev)
trip = torch.zeros(8, 4096, 32, 129, dtype=torch.uint8, device=dev); trip[..., :128] = x; trip = trip.view(-1)
m = trip.numel() // 3
cw = torch.empty(m, dtype=torch.int32, device=dev); ops.golay_encode_into(trip, cw, m)
noisy = torch.empty_like(cw); ops.inject_into(cw, noisy, 1e-2, 24, seed=42)
ref_t = torch.empty(m * 3, dtype=torch.uint8, device=dev); ref_c = torch.empty(m, dtype=torch.uint8, device=dev)
ref_s = ops.new_stats(dev); ops.golay_decode_into(noisy, ref_t, ref_c, ref_s)
out_t = torch.empty_like(ref_t); out_c = torch.empty_like(ref_c)
P = lambda t: VP(t.data_ptr())
cases = {"prod": (lambda st: ops.golay_decode_into(noisy, out_t, out_c, st), "p"),
         "exp2_v3_g8192": (lambda st: lib2.exp2_golay(3, P(noisy), P(out_t), P(out_c), m, P(st), P(tab), 8192, s), "x")}
for v in range(9):
    for grid in (2048, 4096, 8192):
        cases[f"v{v}_g{grid}"] = (lambda st, v=v, grid=grid: lib3.exp3_decode(v, P(noisy), P(out_t), P(out_c), m, P(st), P(tab), grid, s), "x")
ok = {}
for k, (fn, kind) in cases.items():
    out_t.zero_(); out_c.zero_(); st = ops.new_stats(dev)
    r = fn(st); torch.cuda.synchronize()
    ok[k] = torch.equal(out_t, ref_t) and torch.equal(out_c, ref_c) and ops.read_stats(st) == ops.read_stats(ref_s)
times = {k: [] for k in cases}
for _ in range(9):
    for k, (fn, _) in cases.items():
        st = ops.new_stats(dev)
        junk.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(st); b.record(); torch.cuda.synchronize()
        times[k].append(a.elapsed_time(b) * 1e3)
for k, t in sorted(times.items(), key=lambda kv: statistics.median(kv[1])):
    med = statistics.median(t)
    print(f"{k:16s} {med:7.1f} us (min {min(t):6.1f}) {8 * m / med / 1e3:6.0f} GB/s ok={ok[k]}")
