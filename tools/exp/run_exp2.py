"""A/B: Golay decode/encode vs groups-per-lane and block size (tools/exp/golay_exp2.hip)."""
import ctypes, json, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
sys.path.insert(0, HERE)
import torch
from run_exp import tables
VP = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "libexp2.so"))
lib.exp2_golay.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, VP, VP, ctypes.c_int, VP]
from kvecc import ops
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
tab = tables(dev)
g = torch.Generator().manual_seed(0)
x = torch.randint(0, 16, (8, 4096, 32, 128), generator=g, dtype=torch.uint8).to(dev)
trip = torch.zeros(8, 4096, 32, 129, dtype=torch.uint8, device=dev)
trip[..., :128] = x
trip = trip.view(-1)
m = trip.numel() // 3
cw = torch.empty(m, dtype=torch.int32, device=dev)
ops.golay_encode_into(trip, cw, m)
noisy = torch.empty_like(cw)
ops.inject_into(cw, noisy, 1e-2, 24, seed=42)
ref_t = torch.empty(m * 3, dtype=torch.uint8, device=dev)
ref_c = torch.empty(m, dtype=torch.uint8, device=dev)
ops.golay_decode_into(noisy, ref_t, ref_c, ops.new_stats(dev))
out_t = torch.empty_like(ref_t); out_c = torch.empty_like(ref_c); cw2 = torch.empty_like(cw)
cases = {"prod_dec": (lambda: ops.golay_decode_into(noisy, out_t, out_c, ops.new_stats(dev)), 8 * m, None),
         "prod_enc": (lambda: ops.golay_encode_into(trip, cw2, m), 7 * m, None)}
for v in list(range(7)) + list(range(10, 17)):
    for grid in (1024, 2048, 4096, 8192, 16384):
        if v < 10:
            fn = lambda v=v, grid=grid: lib.exp2_golay(v, VP(noisy.data_ptr()), VP(out_t.data_ptr()), VP(out_c.data_ptr()), m, VP(ops.new_stats(dev).data_ptr()), VP(tab.data_ptr()), grid, s)
            cases[f"dec_v{v}_g{grid}"] = (fn, 8 * m, "dec")
        else:
            fn = lambda v=v, grid=grid: lib.exp2_golay(v, VP(cw2.data_ptr()), VP(trip.data_ptr()), VP(0), m, VP(0), VP(tab.data_ptr()), grid, s)
            cases[f"enc_v{v}_g{grid}"] = (fn, 7 * m, "enc")
ok = {}
for k, (fn, _, kind) in cases.items():
    if kind == "dec":
        out_t.zero_(); out_c.zero_(); assert fn() == 0; torch.cuda.synchronize()
        ok[k] = torch.equal(out_t, ref_t) and torch.equal(out_c, ref_c)
    elif kind == "enc":
        cw2.zero_(); assert fn() == 0; torch.cuda.synchronize()
        ok[k] = torch.equal(cw2, cw)
times = {k: [] for k in cases}
for _ in range(7):
    for k, (fn, _, _) in cases.items():
        junk.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize()
        times[k].append(a.elapsed_time(b) * 1e3)
res = {k: (round(statistics.median(t), 1), round(cases[k][1] / statistics.median(t) / 1e3), ok.get(k)) for k, t in times.items()}
for k, v in sorted(res.items(), key=lambda kv: kv[1][0]):
    print(f"{k:20s} {v[0]:7.1f} us {v[1]:6d} GB/s ok={v[2]}")
