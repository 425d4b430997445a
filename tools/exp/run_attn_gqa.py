"""Historical (round 3): drives libattn_<name>.so switch builds (removed in round 4;
results in profiles/r03/attn). Round-4 experiments: tools/exp/attn_exp.hip + run_attn_exp.py.

GQA A/B for paged attention: the product library (workgroups share a cache
head across G query heads) against libattn_nogqa.so (KVECC_ATTN_GQA=0, one
workgroup per query head), interleaved, on [B=8, ctx=4096, D=128] with 32
query heads over 32 (MHA), 16 and 8 cache heads, every codec.  Times are
per API call (split + combine kernels, hipEvent markers), median of ROUNDS.
Env: LIBS (other builds, libattn_<name>.so), ROUNDS, CTX, CODECS, HKVS.
usage: python tools/exp/run_attn_gqa.py"""
import ctypes, math, os, statistics, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402
from kvecc import _lib  # noqa: E402
VP, I64 = ctypes.c_void_p, ctypes.c_int64
libs = {"prod": _lib.load()}
for name in [x for x in os.environ.get("LIBS", "nomfma").split(",") if x]:
    libs[name] = ctypes.CDLL(os.path.join(HERE, f"libattn_{name}.so"))
for l in libs.values():
    l.kvecc_paged_attention.argtypes = [VP, ctypes.c_int, VP, VP, VP, VP, VP, VP, VP, I64, I64, I64, I64, I64,
                                        I64, I64, I64, I64, I64, ctypes.c_float, ctypes.c_int, VP, I64, VP]
    l.kvecc_paged_attention_workspace.argtypes = [I64, I64, I64, I64]
    l.kvecc_paged_attention_workspace.restype = I64
ROUNDS = int(os.environ.get("ROUNDS", "30"))
dev = torch.device("cuda:0")
B, H, BS, D = 8, 32, 16, 128
CTX = int(os.environ.get("CTX", "4096"))
CODECS = os.environ.get("CODECS", "hamming84,golay,golay_packed").split(",")
HKVS = [int(x) for x in os.environ.get("HKVS", "32,16,8").split(",")]
g = torch.Generator(device=dev).manual_seed(0)
nb = CTX // BS
blocks = B * nb
s = VP(torch.cuda.current_stream().cuda_stream)
P = lambda t: VP(t.data_ptr())  # noqa: E731
table = torch.randperm(blocks, device=dev, generator=g).to(torch.int32).view(B, nb)
lens = torch.full((B,), CTX, dtype=torch.int32, device=dev)
q = torch.randn(B, H, D, device=dev, generator=g).half()
ws_n = max(l.kvecc_paged_attention_workspace(B, H, D, CTX) for l in libs.values())
ws = torch.empty(ws_n, dtype=torch.float32, device=dev)
G3 = (D + 2) // 3
RB = _lib.golay_packed_row_bytes(G3)
codecs = {"hamming84": (1, D, torch.uint8), "golay": (2, G3, torch.int32), "golay_packed": (3, RB, torch.uint8)}
for codec, (cid, per, dt) in codecs.items():
    if codec not in CODECS:
        continue
    cid = {"hamming84": _lib.CODEC_H84, "golay": _lib.CODEC_GOLAY, "golay_packed": _lib.CODEC_GOLAY_PACKED}[codec]
    for hkv in HKVS:
        shape = (blocks, 1, hkv, BS * per)
        if dt == torch.int32:
            kc = torch.randint(0, 1 << 24, shape, dtype=dt, device=dev, generator=g)
        else:
            kc = torch.randint(0, 256, shape, dtype=dt, device=dev, generator=g)
        vc = kc.roll(1, 0).contiguous()
        ks = torch.rand(blocks, 1, hkv, BS, device=dev, generator=g)
        vs = torch.rand_like(ks)
        outs = {n: torch.empty_like(q) for n in libs}

        def call(n):
            rc = libs[n].kvecc_paged_attention(P(q), 1, P(kc), P(vc), P(table), P(lens), P(ks), P(vs), P(outs[n]),
                                               B, H, hkv, D, blocks, 1, 0, BS, nb, CTX, 1 / math.sqrt(D), cid,
                                               P(ws), ws_n, s)
            assert rc == 0, (n, rc)

        for n in libs:
            for _ in range(20):
                call(n)
        times = {n: [] for n in libs}
        for _ in range(ROUNDS):
            for n in libs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                call(n)
                e1.record()
                times[n].append((e0, e1))
        torch.cuda.synchronize()
        others = [n for n in libs if n != "prod"]
        other = others[0] if others else "prod"
        diff = float((outs["prod"].float() - outs[other].float()).abs().max())
        kv_bytes = 2 * blocks * hkv * BS * (per * kc.element_size() + 4)
        line = " ".join(f"{n} {statistics.median(a.elapsed_time(b) * 1e3 for a, b in t):6.1f} us"
                        for n, t in times.items())
        med = statistics.median(a.elapsed_time(b) * 1e3 for a, b in times["prod"])
        print(f"{codec:12s} ctx={CTX} H={H} Hkv={hkv:2d}: {line}  (prod {kv_bytes / med / 1e3:5.0f} GB/s of K+V cache)"
              f"  max|prod-{other}| {diff:.2e}", flush=True)
