"""A/B of the packed Golay decode variants (tools/exp/packed_dec_exp.hip,
libpkdec.so) against the product (kvecc_golay_decode_packed in the same library),
interleaved in one process: M = 8*4096*32*43 codewords of the bench's data
(encoded triplets at BER 1e-2, 3 bytes each) -> packed nibbles + uncorrectable
bits, 4.625 B per codeword.

usage: python tools/exp/run_packed_dec_exp.py [variant[:per_cu] ...]
"""
import ctypes
import os
import statistics
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import _lib, ops  # noqa: E402

ROUNDS = int(os.environ.get("ROUNDS", "40"))
DEFAULT = ["pk:2", "pk_cfree:2", "pk_glds:2", "pk_glds:3", "pk_b256:3", "pk_b256:4", "pk_glds_b256:4",
           "pk_p50:2", "pk_p90:2", "pk_cfree_glds:2", "pk:3"]


def main():
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "exp", "libpkdec.so"))
    lib.kvecc_exp_pkdec_name.restype = ctypes.c_char_p
    names = [lib.kvecc_exp_pkdec_name(i).decode() for i in range(lib.kvecc_exp_pkdec_count())]
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.kvecc_exp_pkdec.argtypes = [ci, vp, vp, vp, i64, vp, ci, vp]
    prod = lib.kvecc_golay_decode_packed
    prod.argtypes = _lib.SIGNATURES["kvecc_golay_decode_packed"]
    tn = lib.kvecc_time_next_launch
    tn.argtypes = [vp, vp]
    runs = ["product"] + (sys.argv[1:] or DEFAULT)
    m = 8 * 4096 * 32 * 43
    trip = torch.randint(0, 16, (m, 3), dtype=torch.uint8, device=dev)
    enc = ops.golay_encode(trip)
    ops.inject_into(enc, enc, 1e-2, 24, seed=42)
    cw = torch.stack([(enc >> (8 * k)) & 0xFF for k in range(3)], 1).to(torch.uint8).reshape(-1).contiguous()
    del trip, enc
    nib = torch.empty((3 * m + 1) // 2, dtype=torch.uint8, device=dev)
    fl = torch.empty((m + 7) // 8, dtype=torch.uint8, device=dev)
    stats = {r: ops.new_stats(dev) for r in runs}
    s = torch.cuda.current_stream().cuda_stream

    def call(r, ev=None):
        if ev is not None:
            tn(ev[0].cuda_event, ev[1].cuda_event)
        if r == "product":
            rc = prod(cw.data_ptr(), nib.data_ptr(), fl.data_ptr(), m, stats[r].data_ptr(), s)
        else:
            name, _, pc = r.partition(":")
            rc = lib.kvecc_exp_pkdec(names.index(name), cw.data_ptr(), nib.data_ptr(), fl.data_ptr(), m,
                                     stats[r].data_ptr(), int(pc or 2), s)
        assert rc == 0, r

    for r in runs:
        for _ in range(20):
            call(r)
    torch.cuda.synchronize()
    for st in stats.values():
        st.zero_()
    ref, same = None, {}
    for r in runs:
        nib.fill_(0xEE)
        fl.fill_(0xEE)
        call(r)
        torch.cuda.synchronize()
        if ref is None:
            ref = (nib.clone(), fl.clone())
        same[r] = torch.equal(nib, ref[0]) and torch.equal(fl, ref[1]) and \
            ops.read_stats(stats[r]) == ops.read_stats(stats["product"])
    times = {r: [] for r in runs}
    for _ in range(ROUNDS):
        for r in runs:
            ev = ops.kernel_timer(dev)
            call(r, ev)
            times[r].append(ev)
    torch.cuda.synchronize()
    nbytes = 4.625 * m
    for r in runs:
        us = [a.elapsed_time(b) * 1e3 for a, b in times[r]]
        med = statistics.median(us)
        print(f"{r:20s} median {med:6.1f} us  min {min(us):6.1f}  {nbytes / med / 1e3:5.0f} GB/s  "
              f"frac {nbytes / med / 1e3 / 8000:5.3f}  same={same[r]}", flush=True)


if __name__ == "__main__":
    main()
