"""A/B of the experimental Golay decode variants (tools/exp/golay_dec_exp.hip,
libgdec.so) against kvecc_golay_decode (the product kernel, same library),
interleaved in one process: the headline's 45,088,768 codewords
([8,4096,32,128] per-head packing), BER 1e-2, counts and statistics on.

usage: python tools/exp/run_golay_dec_exp.py [RUN ...]   RUN = tab:per_cu
  tab 0: the product's uint16 tables, 1: the byte-class tables (golay_bc.h)
Times are the kernels' own dispatch stamps, median over ROUNDS interleaved
rounds; outputs, counts and statistics are compared with the product's.
"""
import ctypes
import os
import statistics
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import _lib, ops  # noqa: E402

M = 8 * 4096 * 32 * 43
ROUNDS = int(os.environ.get("ROUNDS", "40"))
LIB = os.path.join(REPO, "tools", "exp", "libgdec.so")
DEFAULT = ["0:32", "0:8", "0:4", "1:32", "1:16", "1:8", "1:4"]


def main():
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(LIB)
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_gdec.argtypes = [ci, ci, vp, vp, vp, i64, vp, vp]
    lib.kvecc_exp_gdec.restype = ci
    prod = lib.kvecc_golay_decode
    prod.argtypes = _lib.SIGNATURES["kvecc_golay_decode"]
    prod.restype = ci
    tn = lib.kvecc_time_next_launch
    tn.argtypes = [vp, vp]
    runs = sys.argv[1:] or DEFAULT
    gen = torch.Generator().manual_seed(0)
    trip = torch.randint(0, 16, (M * 3,), generator=gen, dtype=torch.uint8).to(dev)
    cw = torch.empty(M, dtype=torch.int32, device=dev)
    ops.golay_encode_into(trip, cw, M)
    noisy = torch.empty_like(cw)
    ops.inject_into(cw, noisy, 1e-2, 24, seed=42)
    del cw
    stream = torch.cuda.current_stream(dev).cuda_stream
    out_t = torch.empty(M * 3, dtype=torch.uint8, device=dev)
    out_c = torch.empty(M, dtype=torch.uint8, device=dev)
    allruns = ["product"] + runs
    stats = {r: ops.new_stats(dev) for r in allruns}

    def call(r, ev=None):
        if ev is not None:
            tn(ev[0].cuda_event, ev[1].cuda_event)
        if r == "product":
            rc = prod(noisy.data_ptr(), out_t.data_ptr(), out_c.data_ptr(), M, stats[r].data_ptr(), stream)
        else:
            tab, per_cu = (int(x) for x in r.split(":"))
            rc = lib.kvecc_exp_gdec(tab, per_cu, noisy.data_ptr(), out_t.data_ptr(), out_c.data_ptr(), M,
                                    stats[r].data_ptr(), stream)
        assert rc == 0, (r, rc)

    for r in allruns:
        for _ in range(20):
            call(r)
    torch.cuda.synchronize()
    for s in stats.values():
        s.zero_()
    ref, same = None, {}
    for r in allruns:
        out_t.fill_(0xEE)
        out_c.fill_(0xEE)
        call(r)
        torch.cuda.synchronize()
        if ref is None:
            ref = (out_t.clone(), out_c.clone())
        same[r] = (torch.equal(out_t, ref[0]) and torch.equal(out_c, ref[1])
                   and ops.read_stats(stats[r]) == ops.read_stats(stats["product"]))
    del ref
    times = {r: [] for r in allruns}
    for _ in range(ROUNDS):
        for r in allruns:
            ev = ops.kernel_timer(dev)
            call(r, ev)
            times[r].append(ev)
    torch.cuda.synchronize()
    nbytes = 8 * M
    for r in allruns:
        us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
        med = statistics.median(us)
        print(f"{r:10s} median {med:6.1f} us  min {min(us):6.1f}  {nbytes / med / 1e3:5.0f} GB/s  "
              f"frac {nbytes / med / 1e3 / 8000:5.3f}  same={same[r]}", flush=True)


if __name__ == "__main__":
    main()
