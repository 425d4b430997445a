"""A/B of kvecc_golay_decode_packed across library builds (product first),
interleaved: M = 8*4096*32*43 codewords (3 B each; the bench's BER-1e-2 encoded
data, DATA=random for random bytes) -> packed nibbles + uncorrectable bits;
outputs must equal the first library's.  Env: SIZES, ROUNDS, DATA.
CODEC=h84: kvecc_hamming84_decode_packed instead, N = 8*4096*32*128 values
(encoded at BER 1e-3, 8 bits; DATA=random for random bytes) -> packed nibbles
+ packed error types, 1.75 B/value.
usage: python tools/exp/run_packed_dec_ab.py lib.so [lib.so ...]"""
import ctypes, os, statistics, sys
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402
from kvecc import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
H84 = os.environ.get("CODEC") == "h84"
libs = []
for p in sys.argv[1:]:
    h = ctypes.CDLL(os.path.abspath(p))
    sym = "kvecc_hamming84_decode_packed" if H84 else "kvecc_golay_decode_packed"
    fn = getattr(h, sym)
    fn.argtypes = _lib.SIGNATURES[sym]
    fn.restype = ctypes.c_int
    libs.append((os.path.basename(p), fn))
s = torch.cuda.current_stream().cuda_stream
FULL = 8 * 4096 * 32 * (128 if H84 else 43)
SIZES = [int(x) for x in os.environ.get("SIZES", f"{FULL},1000003,77").split(",")]
ROUNDS = int(os.environ.get("ROUNDS", "40"))
for m in SIZES:
    if H84:
        cw = torch.randint(0, 16, (m,), dtype=torch.uint8, device=dev)
        cw = ops.hamming84_encode(cw)
        if os.environ.get("DATA") == "random":
            cw.random_(0, 256)
        else:
            ops.inject_into(cw, cw, 1e-3, 8, seed=42)
    elif os.environ.get("DATA") == "random":  # every syndrome random: the LDS worst case
        cw = torch.randint(0, 256, (3 * m,), dtype=torch.uint8, device=dev)
    else:  # the bench's input: encoded triplets at BER 1e-2 (24 bits)
        trip = torch.randint(0, 16, (m, 3), dtype=torch.uint8, device=dev)
        enc = ops.golay_encode(trip)
        ops.inject_into(enc, enc, 1e-2, 24, seed=42)
        cw = torch.stack([(enc >> (8 * k)) & 0xFF for k in range(3)], 1).to(torch.uint8).reshape(-1).contiguous()
        del trip, enc
    # one output pair for every library (where outputs sit in HBM moves times)
    if H84:
        shared = (torch.empty((m + 1) // 2, dtype=torch.uint8, device=dev),
                  torch.empty((m + 3) // 4, dtype=torch.uint8, device=dev))
    else:
        shared = (torch.empty((3 * m + 1) // 2, dtype=torch.uint8, device=dev),
                  torch.empty((m + 7) // 8, dtype=torch.uint8, device=dev))
    outs = [shared for _ in libs]
    sts = [ops.new_stats(dev) for _ in libs]
    call = lambda i: libs[i][1](cw.data_ptr(), outs[i][0].data_ptr(), outs[i][1].data_ptr(), m,  # noqa: E731
                                sts[i].data_ptr(), s)
    same, ref = [], None
    for i in range(len(libs)):
        shared[0].fill_(0xEE)
        shared[1].fill_(0xEE)
        assert call(i) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref = (shared[0].clone(), shared[1].clone())
        same.append(torch.equal(shared[0], ref[0]) and torch.equal(shared[1], ref[1]) and ops.read_stats(sts[i]) == ops.read_stats(sts[0]))
    ts = [[] for _ in libs]
    for _ in range(ROUNDS):
        for i in range(len(libs)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); call(i); b.record()
            ts[i].append((a, b))
    torch.cuda.synchronize()
    nb = (1.75 if H84 else 4.625) * m
    for i, (name, _) in enumerate(libs):
        us = statistics.median(a.elapsed_time(b) * 1e3 for a, b in ts[i])
        print(f"m={m:9d} {name:14s} equal={same[i]} median {us:7.1f} us {nb / us / 1e3:5.0f} GB/s", flush=True)
