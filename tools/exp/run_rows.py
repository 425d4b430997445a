"""A/B of the per-head Golay row kernels (kvecc_golay_encode_rows /
decode_rows) across library builds, interleaved in one process, cold L2/MALL
(1 GiB flush before each launch), on [8,4096,32,128] (1,048,576 rows of 128
nibbles, 43 codewords each).  usage: run_rows.py lib.so [lib.so ...]"""
import ctypes
import os
import statistics
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import _lib, ops  # noqa: E402

ROUNDS = 15
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
x = torch.randint(0, 16, (8, 4096, 32, 128), generator=g, dtype=torch.uint8).to(dev)
rows, d = 8 * 4096 * 32, 128
gs = 43
ref_cw = ops.golay_encode_rows(x)
noisy = ref_cw.clone().view(-1)
ops.inject_into(noisy, noisy, 1e-2, 24, seed=42)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
libs = []
for p in sys.argv[1:]:
    h = ctypes.CDLL(os.path.abspath(p))
    for n in ("kvecc_golay_encode_rows", "kvecc_golay_decode_rows"):
        getattr(h, n).argtypes = _lib.SIGNATURES[n]
        getattr(h, n).restype = ctypes.c_int
    libs.append((os.path.basename(p), h))
# one output pair for every library (where outputs sit in HBM moves times)
shared = (torch.empty_like(ref_cw), torch.empty_like(x))
outs = [(shared[0], shared[1], ops.new_stats(dev)) for _ in libs]


def enc(i):
    assert libs[i][1].kvecc_golay_encode_rows(x.data_ptr(), outs[i][0].data_ptr(), rows, d, stream) == 0


def dec(i):
    assert libs[i][1].kvecc_golay_decode_rows(noisy.data_ptr(), outs[i][1].data_ptr(), rows, d,
                                              outs[i][2].data_ptr(), stream) == 0


ref = None
for i, (name, _) in enumerate(libs):
    shared[0].fill_(-1)
    shared[1].fill_(0xEE)
    enc(i)
    dec(i)
    torch.cuda.synchronize()
    if ref is None:
        ref = (shared[0].clone(), shared[1].clone())
    print(f"{name}: encode equal={torch.equal(shared[0], ref[0])} decode equal="
          f"{torch.equal(shared[1], ref[1])} stats={ops.read_stats(outs[i][2])}", flush=True)
del ref
times = {(i, k): [] for i in range(len(libs)) for k in ("enc", "dec")}
for r in range(ROUNDS):
    for i in range(len(libs)):
        for k, fn in (("enc", enc), ("dec", dec)):
            junk.fill_(1)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn(i)
            b.record()
            times[(i, k)].append((a, b))
torch.cuda.synchronize()
nbytes = x.numel() + 4 * ref_cw.numel()
for i, (name, _) in enumerate(libs):
    for k in ("enc", "dec"):
        us = [a.elapsed_time(b) * 1e3 for a, b in times[(i, k)]]
        med = statistics.median(us)
        print(f"{name} {k}: median {med:.1f} us min {min(us):.1f} ({nbytes / med / 1e3:.0f} GB/s, "
              f"{nbytes / med / 1e3 / 80:.1f}%)", flush=True)
