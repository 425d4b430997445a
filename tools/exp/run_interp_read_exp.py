"""A/B of the experimental fused H(8,4) + interpolation reads (interp_read_exp.hip,
libipe.so: ipe_kernel at 1/2/4/8 waves per workgroup, plain and interpolating)
against the product (kvecc_shim_read_batch, interpolating and plain), interleaved
in one process: [B=8, L=4096, Hkv=32, D=128] K+V, block 16, fp16 out, BER
(env, default 1e-3) -- bench.py's fused_golay_decode.hamming84 workload.

usage: python tools/exp/run_interp_read_exp.py [RUN ...]
  RUN = product | plain | ipeW[:pad_kib] | plW[:pad_kib]   (W = waves per workgroup)
Times: the kernels' own dispatch stamps, median over ROUNDS interleaved rounds.
Interpolating runs are compared with the product's interpolating output and
statistics, plain runs with the product's plain read.
"""
import ctypes
import os
import statistics
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import _lib, ops  # noqa: E402

B, L, H, D, BS = 8, 4096, 32, 128, 16
ROUNDS = int(os.environ.get("ROUNDS", "30"))
BER = float(os.environ.get("BER", "1e-3"))
DEFAULT = ["product", "plain", "ipe8:16", "ipe4:8", "ipe2:0", "ipe1:0", "pl8:16", "pl4:8", "pl2:0", "pl1:0"]


def main():
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "exp", "libipe.so"))
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_ipe.argtypes = [ci, ci, ci] + [vp] * 5 + [i64] * 6 + [vp, vp, vp, vp]
    prod = lib.kvecc_shim_read_batch
    prod.argtypes = _lib.SIGNATURES["kvecc_shim_read_batch"]
    tn = lib.kvecc_time_next_launch
    tn.argtypes = [vp, vp]
    runs = sys.argv[1:] or DEFAULT
    nlb = L // BS
    nb = B * nlb
    gen = torch.Generator().manual_seed(11)
    caches, scales = [], []
    for side in range(2):
        x = torch.randint(0, 16, (nb * H * BS * D,), generator=gen, dtype=torch.uint8).to(dev)
        cw = ops.hamming84_encode(x)
        ops.inject_into(cw, cw, BER, 8, seed=42 + side)
        caches.append(cw.view(nb, 1, H, BS * D))
        scales.append((torch.rand(nb, 1, H, BS, generator=gen) * 0.1 + 0.01).to(dev))
    table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
    out = (torch.empty(B, H, L, D, dtype=torch.float16, device=dev),
           torch.empty(B, H, L, D, dtype=torch.float16, device=dev))
    s = torch.cuda.current_stream().cuda_stream
    stats = {r: ops.new_stats(dev) for r in runs}
    ptrs = [caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
            table.data_ptr()]

    def interp_of(r):
        return r == "product" or (r.startswith("ipe") and not r.startswith("ipe302"))

    def call(r, ev=None):
        if ev is not None:
            tn(ev[0].cuda_event, ev[1].cuda_event)
        if r in ("product", "plain"):
            rc = prod(*ptrs, nlb, B, L, H, D, 1, BS, 0, 2, int(r == "product"), out[0].data_ptr(),
                      out[1].data_ptr(), ops._DT[torch.float16], stats[r].data_ptr(), s)
        else:
            name, _, pad = r.partition(":")
            waves = int(name[3:] if name.startswith("ipe") else name[2:])
            rc = lib.kvecc_exp_ipe(waves, int(interp_of(r)), int(pad or 0) * 1024, *ptrs, nlb, B, L, H, D, BS,
                                   out[0].data_ptr(), out[1].data_ptr(), stats[r].data_ptr(), s)
        assert rc == 0, r

    for r in runs:
        for _ in range(20):
            call(r)
    torch.cuda.synchronize()
    for st in stats.values():
        st.zero_()
    refs, same = {}, {}
    for r in ["product", "plain"] + runs:
        if r in same:
            continue
        if r not in stats:
            stats[r] = ops.new_stats(dev)
        stats[r].zero_()
        out[0].fill_(float("nan"))
        out[1].fill_(float("nan"))
        call(r)
        torch.cuda.synchronize()
        key = interp_of(r)
        if key not in refs:
            refs[key] = (out[0].clone(), out[1].clone(), ops.read_stats(stats[r]))
        ref = refs[key]
        same[r] = torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]) and ops.read_stats(stats[r]) == ref[2]
    del refs
    times = {r: [] for r in runs}
    block = int(os.environ.get("BLOCK", "1"))  # BLOCK > 1: bench-like blocks of launches per run
    for _ in range(ROUNDS):
        for r in runs:
            if block > 1:
                for _ in range(100):
                    call(r)
            for _ in range(block):
                ev = ops.kernel_timer(dev)
                call(r, ev)
                times[r].append(ev)
    torch.cuda.synchronize()
    nbytes = 2 * B * L * H * (D + 4 + 2 * D)
    print(f"BER {BER}, {ROUNDS} rounds, blocks of {block}")
    for r in runs:
        us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
        med = statistics.median(us)
        print(f"{r:12s} median {med:6.1f} us  min {min(us):6.1f}  {nbytes / med / 1e3:5.0f} GB/s  "
              f"frac {nbytes / med / 1e3 / 8000:5.3f}  same={same[r]}", flush=True)


if __name__ == "__main__":
    main()
