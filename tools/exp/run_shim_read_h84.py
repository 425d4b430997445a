"""The shim's fused read for the byte codecs (kvecc_shim_read_batch ->
shim_read_bytes_kernel): Hamming(8,4) with and without double-error
interpolation, H(7,4), raw INT4, on [B=8, L=4096, Hkv=32, D=128] K+V, block 16,
fp16 out.  Bytes per token row and side: 128 codeword bytes + 4 B scale in,
256 B out (interpolation re-reads the two neighbour rows: not counted)."""
import os, statistics, sys
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import ops
B, L, H, D, BS = 8, 4096, 32, 128, 16
dev = torch.device("cuda:0")
nlb = L // BS
nb = B * nlb
gen = torch.Generator().manual_seed(7)
x = torch.randint(0, 16, (2, nb, 1, H, BS * D), generator=gen, dtype=torch.uint8).to(dev)
sc = (torch.rand(2, nb, 1, H, BS, generator=gen) * 0.1 + 0.01).to(dev)
table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
ODT = torch.float32 if os.environ.get("OUT") == "fp32" else torch.float16
outs = (torch.empty(B, H, L, D, dtype=ODT, device=dev), torch.empty(B, H, L, D, dtype=ODT, device=dev))
st = ops.new_stats(dev)
for codec, interp in (("hamming84", False), ("hamming84", True), ("hamming74", False), ("int4", False)):
    enc = {"hamming84": ops.hamming84_encode, "hamming74": ops.hamming74_encode, "int4": lambda t: t.clone()}[codec]
    c = [enc(x[s].reshape(-1)).view(nb, 1, H, BS * D) for s in range(2)]
    if codec != "int4":
        for s in range(2):
            cf = c[s].view(-1)
            ops.inject_into(cf, cf, 1e-3, 8 if codec == "hamming84" else 7, seed=42 + s)
    call = lambda: ops.shim_read_batch(c[0], c[1], sc[0], sc[1], table, L, D, 0, codec, ODT,
                                       stats=st, interp=interp, out=outs)
    for _ in range(20): call()
    ts = []
    for _ in range(30):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); call(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    med = statistics.median(ts)
    nbytes = 2 * B * L * H * (D + 4 + outs[0].element_size() * D)
    print(f"{str(ODT)[6:]:8s} {codec:9s} interp={interp!s:5s}: {med:7.1f} us ({nbytes / med / 1e3:.0f} GB/s, {nbytes / med / 8e4:.1f}% of 8 TB/s)", flush=True)
