"""Historical (round 1): drives libpk_direct.so, a switch build of csrc/packed.hip
(removed in round 4). Round-4 experiments: tools/exp/packed_dec_exp.hip + run_packed_dec_exp.py.

A/B: packed Golay decode, production (LDS-staged) vs the direct 8-byte-load kernel
(libpk_direct.so), cold cache.
Build: make -C tools/exp libpk_direct.so    Run (GPU box): python tools/exp/run_packed.py"""
import ctypes, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import _lib, ops
VP, I64 = ctypes.c_void_p, ctypes.c_int64
libs = {"prod": _lib.load(), "direct": ctypes.CDLL(os.path.join(HERE, "libpk_direct.so"))}
for l in libs.values():
    l.kvecc_golay_decode_packed.argtypes = [VP, VP, VP, I64, VP, VP]
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
m = 8 * 4096 * 32 * 43
g = torch.Generator().manual_seed(0)
nib = torch.randint(0, 256, ((m * 3 + 1) // 2,), generator=g, dtype=torch.uint8).to(dev)
cw3 = ops.golay_encode_packed(nib, m)
noisy = cw3 ^ (torch.rand(cw3.shape, device=dev) < 0.01).to(torch.uint8) * 4
P = lambda t: VP(t.data_ptr())
res = {}
for name, l in libs.items():
    out = torch.empty_like(nib); fl = torch.empty((m + 7) // 8, dtype=torch.uint8, device=dev)
    st = ops.new_stats(dev)
    fn = (lambda l=l, out=out, fl=fl, st=st: l.kvecc_golay_decode_packed(P(noisy), P(out), P(fl), m, P(st), s))
    res[name] = (fn, out, fl, st)
ok = {}
for name, (fn, out, fl, st) in res.items():
    st.zero_(); fn(); torch.cuda.synchronize()
    ok[name] = (out.clone(), fl.clone(), ops.read_stats(st))
t = {k: [] for k in res}
for _ in range(9):
    for name, (fn, *_r) in res.items():
        junk.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize()
        t[name].append(a.elapsed_time(b) * 1e3)
for name in res:
    same = all(torch.equal(x, y) if torch.is_tensor(x) else x == y for x, y in zip(ok[name], ok["prod"]))
    med = statistics.median(t[name])
    print(f"{name:8s} {med:7.1f} us {4.625 * m / med / 1e3:6.0f} GB/s equal={same}")
