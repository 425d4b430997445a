"""Historical (round 1): drives libgl_*.so switch builds of csrc/golay.hip (removed in
round 4; results in profiles/r01/golay).

A/B: Golay encode/decode geometry variants (tools/exp/libgl_*.so) vs production, cold cache,
interleaved.  Build: make -C tools/exp libgl_g1.so libgl_g1deep.so libgl_g2deep.so libgl_b256.so
Env: LIBS (libgl_<name>.so list), WARM=1 (no cache flush between launches), ROUNDS."""
import ctypes, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import _lib, ops
VP, I64 = ctypes.c_void_p, ctypes.c_int64
libs = {"prod": _lib.load()}
for n in os.environ.get("LIBS", "g1,g1deep,g2deep,b256").split(","):
    p = os.path.join(HERE, f"libgl_{n}.so")
    if os.path.exists(p):
        libs[n] = ctypes.CDLL(p)
for l in libs.values():
    l.kvecc_golay_encode.argtypes = [VP, VP, I64, VP]
    l.kvecc_golay_decode.argtypes = [VP, VP, VP, I64, VP, VP]
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
m = 8 * 4096 * 32 * 43
g = torch.Generator().manual_seed(0)
trip = torch.randint(0, 16, (m * 3,), generator=g, dtype=torch.uint8).to(dev)
cw = torch.empty(m, dtype=torch.int32, device=dev)
ops.golay_encode_into(trip, cw, m)
noisy = torch.empty_like(cw)
ops.inject_into(cw, noisy, 1e-2, 24, seed=42)
P = lambda t: VP(t.data_ptr())
ref_t = torch.empty_like(trip); ref_c = torch.empty(m, dtype=torch.uint8, device=dev)
ops.golay_decode_into(noisy, ref_t, ref_c, ops.new_stats(dev))
cases = {}
for name, l in libs.items():
    o_cw = torch.empty_like(cw); o_t = torch.empty_like(trip); o_c = torch.empty_like(ref_c)
    st = ops.new_stats(dev)
    cases[(name, "enc")] = (lambda l=l, o=o_cw: l.kvecc_golay_encode(P(trip), P(o), m, s), o_cw, cw, 7)
    cases[(name, "dec")] = (lambda l=l, ot=o_t, oc=o_c, st=st: l.kvecc_golay_decode(P(noisy), P(ot), P(oc), m, P(st), s),
                            o_t, ref_t, 8)
ok = {}
for k, (fn, out, ref, _) in cases.items():
    out.zero_(); fn(); torch.cuda.synchronize(); ok[k] = torch.equal(out, ref)
t = {k: [] for k in cases}
WARM = os.environ.get("WARM") == "1"  # back-to-back as bench.py runs, instead of cold
for _ in range(int(os.environ.get("ROUNDS", "9"))):
    for k, (fn, *_r) in cases.items():
        if not WARM:
            junk.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize()
        t[k].append(a.elapsed_time(b) * 1e3)
for k in sorted(cases, key=lambda k: (k[1], statistics.median(t[k]))):
    med = statistics.median(t[k])
    print(f"{k[1]} {k[0]:8s} {med:7.1f} us {cases[k][3] * m / med / 1e3:6.0f} GB/s ok={ok[k]}")
