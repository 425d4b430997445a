"""A/B of the fused Hamming(8,4) read (plain and interpolating) at other work
variants (tools/exp/bytes_read_exp.hip: kvecc_exp_bytes_read_ip, runs
"name[:per_cu]"; kvecc_exp_bytes_read_ipwg, runs "ipwg[:pad_kib]" /
"ipwgf[:pad_kib]") against the product (kvecc_shim_read_batch), interleaved: [B=8, L=4096, Hkv=32, D=128] K+V,
block 16, BER 1e-3, fp16 out -- bench.py's fused_golay_decode.hamming84 workload.

usage: python tools/exp/run_bytes_read_exp.py [name[:per_cu] | ipwg[:pad_kib] | ipwgf[:pad_kib] | ladN ...]
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
DEFAULT = ["ip", "ipwgf:16", "ipwgf:0", "ipwg:16", "plain"]


def main():
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "exp", "libbread.so"))
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_bytes_read_ip.argtypes = [ci, ci] + [vp] * 5 + [i64] * 6 + [vp, vp, vp, vp]
    lib.kvecc_exp_bytes_read_ipwg.argtypes = [ci] + [vp] * 5 + [i64] * 6 + [vp, vp, vp, vp]
    lib.kvecc_exp_bytes_ladder.argtypes = [ci] + [vp] * 5 + [i64] * 6 + [vp, vp, vp, vp]
    lib.kvecc_exp_bytes_ip_name.restype = ctypes.c_char_p
    ipn = [lib.kvecc_exp_bytes_ip_name(i).decode() for i in range(lib.kvecc_exp_bytes_ip_count())]
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
    for interp in (1,):  # "plain": the product without interpolation, for reference (same=False)
        sel = ["product"] + runs
        stats = {r: ops.new_stats(dev) for r in sel}

        def call(r, ev=None):
            if ev is not None:
                tn(ev[0].cuda_event, ev[1].cuda_event)
            if r in ("product", "plain"):
                rc = prod(caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
                          table.data_ptr(), nlb, B, L, H, D, 1, BS, 0, 2, int(r == "product"), out[0].data_ptr(),
                          out[1].data_ptr(), ops._DT[torch.float16], stats[r].data_ptr(), s)
            elif r.startswith("lad"):  # ladN: bytes_ladder_kernel<N>
                rc = lib.kvecc_exp_bytes_ladder(int(r[3:]), caches[0].data_ptr(), caches[1].data_ptr(),
                                                scales[0].data_ptr(), scales[1].data_ptr(), table.data_ptr(),
                                                nlb, B, L, H, D, BS, out[0].data_ptr(), out[1].data_ptr(),
                                                stats[r].data_ptr(), s)
            elif r.startswith("ipwg"):  # ipwg[:pad_kib], ipwgf[:pad_kib] = the flag form
                pad = int(r.partition(":")[2] or 0) * 1024 + (1 if r.startswith("ipwgf") else 0)
                rc = lib.kvecc_exp_bytes_read_ipwg(pad, caches[0].data_ptr(), caches[1].data_ptr(),
                                                   scales[0].data_ptr(), scales[1].data_ptr(), table.data_ptr(),
                                                   nlb, B, L, H, D, BS, out[0].data_ptr(), out[1].data_ptr(),
                                                   stats[r].data_ptr(), s)
            else:
                name, _, pc = r.partition(":")
                rc = lib.kvecc_exp_bytes_read_ip(ipn.index(name), int(pc or 2), caches[0].data_ptr(),
                                                 caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
                                                 table.data_ptr(), nlb, B, L, H, D, BS, out[0].data_ptr(),
                                                 out[1].data_ptr(), stats[r].data_ptr(), s)
            assert rc == 0, r

        for r in sel:
            for _ in range(20):
                call(r)
        torch.cuda.synchronize()
        for st in stats.values():
            st.zero_()
        ref, same = None, {}
        for r in sel:
            out[0].fill_(float("nan"))
            out[1].fill_(float("nan"))
            call(r)
            torch.cuda.synchronize()
            if ref is None:
                ref = (out[0].clone(), out[1].clone())
            same[r] = torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]) and \
                ops.read_stats(stats[r]) == ops.read_stats(stats["product"])
        del ref
        times = {r: [] for r in sel}
        for _ in range(ROUNDS):
            for r in sel:
                ev = ops.kernel_timer(dev)
                call(r, ev)
                times[r].append(ev)
        torch.cuda.synchronize()
        nbytes = 2 * B * L * H * (D + 4 + 2 * D)
        for r in sel:
            us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
            med = statistics.median(us)
            print(f"interp {r:14s} median {med:6.1f} us  min {min(us):6.1f}  "
                  f"{nbytes / med / 1e3:5.0f} GB/s  frac {nbytes / med / 1e3 / 8000:5.3f}  same={same[r]}", flush=True)


if __name__ == "__main__":
    main()
