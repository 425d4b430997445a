"""A/B of kvecc_golay_decode_packed across library builds (product first),
interleaved: M = 8*4096*32*43 codewords (3 B each) -> packed nibbles +
uncorrectable bits; outputs must equal the first library's.
usage: python tools/exp/run_packed_dec_ab.py lib.so [lib.so ...]"""
import ctypes, os, statistics, sys
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402
from kvecc import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
libs = []
for p in sys.argv[1:]:
    h = ctypes.CDLL(os.path.abspath(p))
    fn = h.kvecc_golay_decode_packed
    fn.argtypes = _lib.SIGNATURES["kvecc_golay_decode_packed"]
    fn.restype = ctypes.c_int
    libs.append((os.path.basename(p), fn))
s = torch.cuda.current_stream().cuda_stream
for m in (8 * 4096 * 32 * 43, 1000003, 77):
    cw = torch.randint(0, 256, (3 * m,), dtype=torch.uint8, device=dev)
    # one output pair for every library (where outputs sit in HBM moves times)
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
        same.append(torch.equal(shared[0], ref[0]) and torch.equal(shared[1], ref[1]) and torch.equal(sts[i], sts[0]))
    ts = [[] for _ in libs]
    for _ in range(40):
        for i in range(len(libs)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); call(i); b.record()
            ts[i].append((a, b))
    torch.cuda.synchronize()
    nb = 4.625 * m
    for i, (name, _) in enumerate(libs):
        us = statistics.median(a.elapsed_time(b) * 1e3 for a, b in ts[i])
        print(f"m={m:9d} {name:14s} equal={same[i]} median {us:7.1f} us {nb / us / 1e3:5.0f} GB/s", flush=True)
