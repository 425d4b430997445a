"""A/B of packed Hamming(8,4) encode grids (tools/exp/h84_pk_enc_exp.hip,
libh84pke.so) against kvecc_hamming84_encode_packed, interleaved in one
process: V = 8*4096*32*128 values (config 2's tensor, packed nibbles in,
codeword bytes out; 1.5 B per value).  RUN = v:per_cu (v 0 grid-stride, 1 full
grid, 2 full grid two chunks per lane).  Median of ROUNDS kernel stamps."""
import ctypes
import os
import statistics
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import ops  # noqa: E402

N = 8 * 4096 * 32 * 128
ROUNDS = int(os.environ.get("ROUNDS", "60"))


def golay(lib, dev, runs):
    """packed Golay encode: RUN = per_cu (the product 16); M_h codewords"""
    m = 8 * 4096 * 32 * 43
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_gpk_enc.argtypes = [ci, vp, vp, i64, vp]
    prod = lib.kvecc_golay_encode_packed
    prod.argtypes = [vp, vp, i64, vp]
    tn = lib.kvecc_time_next_launch
    tn.argtypes = [vp, vp]
    g = torch.Generator(device=dev).manual_seed(0)
    nib = torch.randint(0, 256, ((3 * m + 1) // 2,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(3 * m, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream

    def call(r, ev=None):
        if ev is not None:
            tn(ev[0].cuda_event, ev[1].cuda_event)
        rc = prod(nib.data_ptr(), out.data_ptr(), m, s) if r == "product" else \
            lib.kvecc_exp_gpk_enc(int(r), nib.data_ptr(), out.data_ptr(), m, s)
        assert rc == 0, r

    allruns = ["product"] + runs
    for r in allruns:
        for _ in range(30):
            call(r)
    call("product")
    torch.cuda.synchronize()
    ref = out.clone()
    same = {}
    for r in allruns:
        out.fill_(0)
        call(r)
        torch.cuda.synchronize()
        same[r] = torch.equal(out, ref)
    times = {r: [] for r in allruns}
    for _ in range(ROUNDS):
        for r in allruns:
            ev = ops.kernel_timer(dev)
            call(r, ev)
            times[r].append(ev)
    torch.cuda.synchronize()
    nbytes = m * 9 // 2
    for r in allruns:
        us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
        med = statistics.median(us)
        print(f"golay {r:8s} median {med:6.2f} us  min {min(us):6.2f}  frac {nbytes / med / 1e3 / 8000:5.3f}  "
              f"same={same[r]}", flush=True)


def main():
    dev = torch.device("cuda:0")
    if sys.argv[1:2] == ["golay"]:
        return golay(ctypes.CDLL(os.path.join(REPO, "tools", "exp", "libh84pke.so")), dev, sys.argv[2:] or ["16", "32", "64"])
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "exp", "libh84pke.so"))
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_h84_pk_enc.argtypes = [ci, ci, vp, vp, i64, vp]
    prod = lib.kvecc_hamming84_encode_packed
    prod.argtypes = [vp, vp, i64, vp]
    tn = lib.kvecc_time_next_launch
    tn.argtypes = [vp, vp]
    runs = sys.argv[1:] or ["0:32", "0:64", "1:0", "2:0"]
    g = torch.Generator(device=dev).manual_seed(0)
    nib = torch.randint(0, 256, (N // 2,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(N, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream

    def call(r, ev=None):
        if ev is not None:
            tn(ev[0].cuda_event, ev[1].cuda_event)
        if r == "product":
            rc = prod(nib.data_ptr(), out.data_ptr(), N, s)
        else:
            v, pc = (int(x) for x in r.split(":"))
            rc = lib.kvecc_exp_h84_pk_enc(v, pc, nib.data_ptr(), out.data_ptr(), N, s)
        assert rc == 0, r

    allruns = ["product"] + runs
    for r in allruns:
        for _ in range(30):
            call(r)
    torch.cuda.synchronize()
    call("product")
    ref = out.clone()
    same = {}
    for r in allruns:
        out.fill_(0)
        call(r)
        torch.cuda.synchronize()
        same[r] = torch.equal(out, ref)
    times = {r: [] for r in allruns}
    for _ in range(ROUNDS):
        for r in allruns:
            ev = ops.kernel_timer(dev)
            call(r, ev)
            times[r].append(ev)
    torch.cuda.synchronize()
    nbytes = N * 3 // 2
    for r in allruns:
        us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
        med = statistics.median(us)
        print(f"{r:8s} median {med:6.2f} us  min {min(us):6.2f}  frac {nbytes / med / 1e3 / 8000:5.3f}  same={same[r]}",
              flush=True)


if __name__ == "__main__":
    main()
