"""Does the K/V buffer offset matter?  Paged attention on identical K/V data,
V placed at different byte offsets after K (adjacent allocations put V one
cache size after K, as SimpleBlockManager's two torch.zeros do)."""
import math, sys, statistics
sys.path.insert(0, "quantized-kv-cache-ecc-protection_amd")
import torch
from kvecc import ops
dev = torch.device("cuda:0")
B, H, D, CTX, BS = 8, 32, 128, 4096, 16
nb = CTX // BS; blocks = B * nb
g = torch.Generator(device=dev).manual_seed(0)
for codec in ("hamming84", "golay", "golay_packed"):
    per = D if codec == "hamming84" else (D + 2) // 3
    if codec == "golay_packed": per = (3 * per + 3) // 4 * 4
    dt = torch.int32 if codec == "golay" else torch.uint8
    n = blocks * H * BS * per
    esz = 4 if dt == torch.int32 else 1
    ks = torch.rand(blocks, 1, H, BS, device=dev, generator=g); vs = torch.rand_like(ks)
    table = torch.randperm(blocks, device=dev, generator=g).to(torch.int32).view(B, nb)
    lens = torch.full((B,), CTX, dtype=torch.int32, device=dev)
    q = torch.randn(B, H, D, device=dev, generator=g).half(); out = torch.empty_like(q)
    for pad_bytes in (0, 4096, 65536 + 4096, 1 << 20, 3 * 4096 + 512):
        pad = pad_bytes // esz
        buf = torch.empty(2 * n + pad + 64, dtype=dt, device=dev)
        if dt == torch.int32:
            buf.random_(0, 1 << 24, generator=g)
        else:
            buf.random_(0, 256, generator=g)
        kc = buf[:n].view(blocks, 1, H, BS * per)
        vc = buf[n + pad:2 * n + pad].view(blocks, 1, H, BS * per)
        vc.copy_(kc)
        call = lambda: ops.paged_attention_into(q, kc, vc, table, lens, ks, vs, out, 0, BS, 1 / math.sqrt(D), codec, CTX)
        for _ in range(3): call()
        ts = []
        for r in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): call()
            e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 100)
        print(f"{codec:13s} V at K + size + {pad_bytes:8d} B: {statistics.median(ts):6.1f} us", flush=True)
        del buf, kc, vc
