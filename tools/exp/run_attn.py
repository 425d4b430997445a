"""Historical (rounds 1-3): drives libattn_*.so builds of csrc/attention.hip with
-DKVECC_ATTN_* switches, which round 4 removed (results: profiles/r01-r03/attention, attn).
Round-4 attention experiments: tools/exp/attn_exp.hip + run_attn_exp.py.

A/B: paged attention lane widths (tools/exp/libattn_v*.so built with other
KVECC_ATTN_*_VEC) vs production libkvecc.so, interleaved, same inputs, both codecs.
Build: make -C tools/exp libattn_v8.so libattn_v16.so libattn_u16.so   Run (GPU box): python tools/exp/run_attn.py"""
import ctypes, math, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import _lib, ops
VP, I64 = ctypes.c_void_p, ctypes.c_int64
libs = {"prod": _lib.load()}
for name in ("prev", "v2", "v8", "v16", "buf", "nopk", "bufnopk", "u16", "g4", "u2", "u8", "gu1", "gu3", "gu4", "lutf", "expf", "r01", "w8", "w8u2", "w8v2", "h1", "h3", "h2f", "h2w8", "m5w5", "m6w6", "m8w8"):
    path = os.path.join(HERE, f"libattn_{name}.so")
    if os.path.exists(path):
        libs[name] = ctypes.CDLL(path)
for l in libs.values():
    l.kvecc_paged_attention.argtypes = [VP, ctypes.c_int, VP, VP, VP, VP, VP, VP, VP, I64, I64, I64, I64, I64,
                                        I64, I64, I64, I64, I64, ctypes.c_float, ctypes.c_int, VP, I64, VP]
    l.kvecc_paged_attention.restype = ctypes.c_int
    l.kvecc_paged_attention_workspace.argtypes = [I64, I64, I64, I64]
    l.kvecc_paged_attention_workspace.restype = I64
dev = torch.device("cuda:0")
B, H, CTX, BS = 8, 32, 4096, 16
D = int(os.environ.get("D", "128"))
g = torch.Generator(device=dev).manual_seed(0)
nb = CTX // BS
blocks = B * nb
P = lambda t: VP(t.data_ptr())
s = VP(torch.cuda.current_stream().cuda_stream)
ks = torch.rand(blocks, 1, H, BS, device=dev, generator=g)
vs = torch.rand_like(ks)
table = torch.randperm(blocks, device=dev, generator=g).to(torch.int32).view(B, nb)
lens = torch.full((B,), CTX, dtype=torch.int32, device=dev)
q = torch.randn(B, H, D, device=dev, generator=g).half()
ws_n = max(l.kvecc_paged_attention_workspace(B, H, D, CTX) for l in libs.values())
ws = torch.empty(ws_n, dtype=torch.float32, device=dev)
nib = torch.randint(0, 16, (blocks * H * BS * D,), dtype=torch.uint8, device=dev, generator=g)
G = (D + 2) // 3
pad = torch.zeros(blocks * H * BS, G * 3, dtype=torch.uint8, device=dev)
pad[:, :D] = nib.view(-1, D)
caches = {("hamming84", "random"): torch.randint(0, 256, (blocks, 1, H, BS * D), dtype=torch.uint8, device=dev, generator=g),
          ("hamming84", "encoded"): ops.hamming84_encode(nib).view(blocks, 1, H, BS * D),
          ("golay", "encoded"): ops.golay_encode(pad.view(-1, 3)).view(blocks, 1, H, BS * G),
          ("golay", "random"): torch.randint(0, 1 << 24, (blocks, 1, H, BS * G), dtype=torch.int32, device=dev, generator=g)}
RB = _lib.golay_packed_row_bytes(G)  # packed rows: low 3 bytes of each int32 codeword
for kind in ("encoded", "random"):
    w = caches[("golay", kind)].view(-1, G).view(torch.uint8).view(-1, G, 4)[:, :, :3].reshape(-1, 3 * G)
    pk = torch.zeros(w.shape[0], RB, dtype=torch.uint8, device=dev)
    pk[:, :3 * G] = w
    caches[("golay_packed", kind)] = pk.view(blocks, 1, H, BS * RB)
codes = {"hamming84": _lib.CODEC_H84, "golay": _lib.CODEC_GOLAY, "golay_packed": _lib.CODEC_GOLAY_PACKED}
outs = {}
for (codec, kind), kc in caches.items():
    vc = kc.roll(1, 0).contiguous()
    for lname, l in libs.items():
        out = torch.empty_like(q)
        fn = (lambda l=l, out=out, kc=kc, vc=vc, codec=codec: l.kvecc_paged_attention(
            P(q), _lib.F16, P(kc), P(vc), P(table), P(lens), P(ks), P(vs), P(out), B, H, H, D, blocks, 1, 0, BS,
            nb, CTX, 1 / math.sqrt(D), codes[codec], P(ws), ws_n, s))
        outs[(codec, kind, lname)] = (fn, out)
t = {k: [] for k in outs}
for r in range(10):
    for k, (fn, out) in outs.items():
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            rc = fn()
        b.record(); torch.cuda.synchronize()
        assert rc == 0, (k, rc)
        t[k].append(a.elapsed_time(b) * 100)  # us per call
for k in outs:
    med = statistics.median(t[k])
    ref = outs[(k[0], k[1], "prod")][1].float()
    err = float((outs[k][1].float() - ref).abs().max())
    cw_b = caches[k[:2]].numel() * caches[k[:2]].element_size() * 2 + 2 * B * CTX * H * 4
    print(f"{k[0]:10s} {k[1]:8s} {k[2]:5s} {med:7.1f} us {cw_b / med / 1e3:6.0f} GB/s max|diff| vs prod {err:.2e}")
