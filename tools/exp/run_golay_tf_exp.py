"""A/B of the full-grid, table-free fused Golay read (tools/exp/golay_tf_exp.hip,
libgtf.so) against the product's persistent kernel (kvecc_shim_read_batch in the
same library), interleaved in one process on bench.py's fused_golay_decode
workload: [B=8, L=4096, Hkv=32, D=128] K+V, block 16, BER 1e-2, fp16 out.

usage: python tools/exp/run_golay_tf_exp.py [RUN ...]   RUN = variant[:lds_pad_kib]
Times are the kernels' own dispatch stamps, median over ROUNDS interleaved rounds.
Outputs and statistics are compared with the product's (tf_synonly and
tf_fastonly compute wrong values on purpose).  Also checks, before timing, a
BER 5e-2 cache (many double and triple errors, some uncorrectable) for
equality with the product.
"""
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

from kvecc import _lib, ops  # noqa: E402
from run_golay_read_exp import B, BS, D, H, L, golay_caches  # noqa: E402

ROUNDS = int(os.environ.get("ROUNDS", "30"))
DEFAULT = ["gq:0", "tf_fastonly:0", "tf_synonly:0", "pk_gq:0", "pk_tf_synonly:0"]


def main():
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(os.path.join(HERE, "libgtf.so"))
    lib.kvecc_exp_gtf_name.restype = ctypes.c_char_p
    names = [lib.kvecc_exp_gtf_name(i).decode() for i in range(lib.kvecc_exp_gtf_count())]
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_gtf.argtypes = [ci, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, ci, vp, vp, vp, ci, vp]
    lib.kvecc_exp_gtf.restype = ci
    prod = lib.kvecc_shim_read_batch
    prod.argtypes = _lib.SIGNATURES["kvecc_shim_read_batch"]
    prod.restype = ci
    tn = lib.kvecc_time_next_launch
    tn.argtypes = [vp, vp]
    runs = sys.argv[1:] or DEFAULT
    nlb = L // BS
    nb = B * nlb
    gen = torch.Generator().manual_seed(7)
    table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
    scales = [(torch.rand(nb, 1, H, BS, generator=gen) * 0.1 + 0.01).to(dev) for _ in range(2)]
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = (D + 2) // 3
    out = (torch.empty(B, H, L, D, dtype=torch.float16, device=dev),
           torch.empty(B, H, L, D, dtype=torch.float16, device=dev))
    for packed in (False, True):
        sel = [r for r in runs if r.startswith("pk_") == packed]
        if not sel:
            continue
        cid = ops.SHIM_CODECS["golay_packed" if packed else "golay"]
        per = ((3 * g + 3) // 4 * 4) if packed else g
        allruns = ["product"] + sel
        stats = {r: ops.new_stats(dev) for r in allruns}

        def call(r, caches, ev=None):
            bs = caches[0].shape[-1] // per
            if ev is not None:
                tn(ev[0].cuda_event, ev[1].cuda_event)
            if r == "product":
                rc = prod(caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
                          table.data_ptr(), table.shape[1], B, L, H, D, 1, bs, 0, cid, 0,
                          out[0].data_ptr(), out[1].data_ptr(), ops._DT[torch.float16], stats[r].data_ptr(), stream)
            else:
                parts = r.split(":")
                v = names.index(parts[0])
                pad = int(parts[1]) * 1024 if len(parts) > 1 else 0
                rc = lib.kvecc_exp_gtf(v, caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(),
                                       scales[1].data_ptr(), table.data_ptr(), table.shape[1], B, L, H, D, bs,
                                       int(packed), out[0].data_ptr(), out[1].data_ptr(), stats[r].data_ptr(),
                                       pad, stream)
            assert rc == 0, (r, rc)

        def compare(caches, label):
            for s in stats.values():
                s.zero_()
            ref, same = None, {}
            for r in allruns:
                out[0].fill_(float("nan"))
                out[1].fill_(float("nan"))
                call(r, caches)
                torch.cuda.synchronize()
                if ref is None:
                    ref = (out[0].clone(), out[1].clone())
                same[r] = (torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
                           and ops.read_stats(stats[r]) == ops.read_stats(stats["product"]))
            print(f"{label}: stats {ops.read_stats(stats['product'])} same {same}", flush=True)
            return same

        heavy = golay_caches(dev, packed, gen, nb, ber=5e-2)
        compare(heavy, f"{'packed' if packed else 'int32'} BER 5e-2")
        del heavy
        caches = golay_caches(dev, packed, gen, nb)
        for r in allruns:
            for _ in range(20):
                call(r, caches)
        torch.cuda.synchronize()
        same = compare(caches, f"{'packed' if packed else 'int32'} BER 1e-2")
        times = {r: [] for r in allruns}
        for _ in range(ROUNDS):
            for r in allruns:
                ev = ops.kernel_timer(dev)
                call(r, caches, ev)
                times[r].append(ev)
        torch.cuda.synchronize()
        nbytes = 2 * B * L * H * ((3 * g if packed else 4 * g) + 4 + 2 * D)
        for r in allruns:
            us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
            med = statistics.median(us)
            print(f"{'packed' if packed else 'int32 '} {r:20s} median {med:6.1f} us  min {min(us):6.1f}  "
                  f"{nbytes / med / 1e3:5.0f} GB/s  frac {nbytes / med / 1e3 / 8000:5.3f}  same={same[r]}", flush=True)
        del caches


if __name__ == "__main__":
    main()
