"""A/B of the experimental fused Golay read variants (tools/exp/golay_read_exp.hip,
libgread.so) against the product kernel (kvecc_shim_read_batch in the same
library), interleaved in one process: [B=8, L=4096, Hkv=32, D=128] K+V, block
16, BER 1e-2, fp16 out -- bench.py's fused_golay_decode workload.

usage: python tools/exp/run_golay_read_exp.py [RUN ...]
  RUN = variant[:per_cu[:lds_pad_kib]]  (default: the list below)
Times are the kernels' own dispatch stamps, median over ROUNDS interleaved rounds
(BLOCK consecutive launches per run in turn); outputs and statistics are
compared with the product's (variants named *cfree / *nogather compute wrong
values on purpose).
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
BLOCK = int(os.environ.get("BLOCK", "1"))
LIB = os.path.join(REPO, "tools", "exp", "libgread.so")
DEFAULT = [
    "pers:2", "pers_cfree:2", "pers_nogather:2", "pers_pad8:2", "pers_fetch1st:2", "pers_glds:2",
    "full1_s0:0:0", "full1_s1:0:0", "full1_glds:0:0", "full1_glds:0:28", "full1_glds:0:60",
    "full2_glds:0:0", "full2_glds:0:28", "full4_glds:0:0", "full1_glds_b1024:0:0", "full2_glds_b1024:0:0",
    "full1_splitp_s1:0:0", "full2_splitp_s1:0:0", "full1_glds_nogather:0:0", "full1_glds_cfree:0:0",
    "pk_pers:2", "pk_full1_glds:0:0", "pk_full2_glds:0:0",
]


def golay_caches(dev, packed, gen, nb, ber=1e-2):
    g = (D + 2) // 3
    out = []
    for side in range(2):
        x = torch.randint(0, 16, (nb, 1, H, BS, D), generator=gen, dtype=torch.uint8).to(dev)
        cw = ops.golay_encode_rows(x).view(-1)
        ops.inject_into(cw, cw, ber, 24, seed=42 + side)
        cw = cw.view(nb, 1, H, BS * g)
        if packed:
            cw = torch.stack([(cw >> (8 * k)) & 0xFF for k in range(3)], -1).to(torch.uint8)
            cw = cw.view(nb, 1, H, BS, 3 * g)
            row = (3 * g + 3) // 4 * 4
            pad = torch.zeros(nb, 1, H, BS, row, dtype=torch.uint8, device=dev)
            pad[..., :3 * g] = cw
            cw = pad.view(nb, 1, H, BS * row)
        out.append(cw.contiguous())
    return out


def main():
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(LIB)
    lib.kvecc_exp_gread_name.restype = ctypes.c_char_p
    names = [lib.kvecc_exp_gread_name(i).decode() for i in range(lib.kvecc_exp_gread_count())]
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_gread.argtypes = [ci, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, ci, vp, vp, vp, ci, ci, vp]
    lib.kvecc_exp_gread.restype = ci
    lib.kvecc_exp_gread_fixed.argtypes = [ci, ci, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, ci, vp, vp, vp, vp]
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
        caches = golay_caches(dev, packed, gen, nb)
        cid = ops.SHIM_CODECS["golay_packed" if packed else "golay"]
        per = ((3 * g + 3) // 4 * 4) if packed else g
        bs = caches[0].shape[-1] // per
        allruns = ["product"] + sel
        stats = {r: ops.new_stats(dev) for r in allruns}

        def call(r, ev=None):
            if ev is not None:
                tn(ev[0].cuda_event, ev[1].cuda_event)
            if r in ("fixed", "pk_fixed"):  # the product kernel, fixed item counts (3 / 4)
                rc = lib.kvecc_exp_gread_fixed(3, 4, caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(),
                                               scales[1].data_ptr(), table.data_ptr(), table.shape[1], B, L, H, D, bs,
                                               int(packed), out[0].data_ptr(), out[1].data_ptr(),
                                               stats[r].data_ptr(), stream)
            elif r == "product":
                rc = prod(caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
                          table.data_ptr(), table.shape[1], B, L, H, D, 1, bs, 0, cid, 0,
                          out[0].data_ptr(), out[1].data_ptr(), ops._DT[torch.float16], stats[r].data_ptr(), stream)
            else:
                parts = r.split(":")
                v = names.index(parts[0])
                per_cu = int(parts[1]) if len(parts) > 1 else 2
                pad = int(parts[2]) * 1024 if len(parts) > 2 else 0
                rc = lib.kvecc_exp_gread(v, caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(),
                                         scales[1].data_ptr(), table.data_ptr(), table.shape[1], B, L, H, D, bs,
                                         int(packed), out[0].data_ptr(), out[1].data_ptr(), stats[r].data_ptr(),
                                         per_cu, pad, stream)
            assert rc == 0, (r, rc)

        for r in allruns:
            for _ in range(20):
                call(r)
        torch.cuda.synchronize()
        for s in stats.values():
            s.zero_()
        ref, same = None, {}
        for r in allruns:
            out[0].fill_(float("nan"))
            out[1].fill_(float("nan"))
            call(r)
            torch.cuda.synchronize()
            if ref is None:
                ref = (out[0].clone(), out[1].clone())
            same[r] = (torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
                       and ops.read_stats(stats[r]) == ops.read_stats(stats["product"]))
        del ref
        times = {r: [] for r in allruns}
        for _ in range(0, ROUNDS, BLOCK):
            for r in allruns:
                for _ in range(BLOCK):
                    ev = ops.kernel_timer(dev)
                    call(r, ev)
                    times[r].append(ev)
        torch.cuda.synchronize()
        nbytes = 2 * B * L * H * ((3 * g if packed else 4 * g) + 4 + 2 * D)
        for r in allruns:
            us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
            med = statistics.median(us)
            print(f"{'packed' if packed else 'int32 '} {r:24s} median {med:6.1f} us  min {min(us):6.1f}  "
                  f"{nbytes / med / 1e3:5.0f} GB/s  frac {nbytes / med / 1e3 / 8000:5.3f}  same={same[r]}", flush=True)
        del caches


if __name__ == "__main__":
    main()
