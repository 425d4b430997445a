"""Kernel micro-benchmarks (interleaved A/B in one process, cold-cache).

Each measurement flushes the 256 MiB Infinity Cache by writing a 1 GiB
buffer first, then times one launch with HIP events on the launching stream.
Reports median / min over rounds.

usage: python tools/kbench.py [--rounds 10] [--which golay,hamming,inject,copy]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def timed(fn, flush, rounds):
    ts = []
    for _ in range(rounds):
        flush()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)  # us
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--which", default="golay,hamming,inject,copy,interp,fused")
    args = ap.parse_args()
    which = set(args.which.split(","))
    from kvecc import ops
    dev = torch.device("cuda:0")
    junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)

    def flush():
        junk.fill_(1)

    res = {}
    B, L, H, D = 8, 4096, 32, 128
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 16, (B, L, H, D), generator=g, dtype=torch.uint8).to(dev)

    if "copy" in which:
        src = torch.empty(360 << 20, dtype=torch.uint8, device=dev)
        dst = torch.empty_like(src)
        med, mn = timed(lambda: dst.copy_(src), flush, args.rounds)
        res["copy_360MB"] = {"us": med, "min_us": mn, "GBps": 2 * src.numel() / med / 1e3}

    if "golay" in which:
        trip = torch.zeros(B, L, H, 129, dtype=torch.uint8, device=dev)
        trip[..., :128] = x
        trip = trip.view(-1)
        m = trip.numel() // 3
        cw = torch.empty(m, dtype=torch.int32, device=dev)
        ops.golay_encode_into(trip, cw, m)
        noisy = torch.empty_like(cw)
        ops.inject_into(cw, noisy, 1e-2, 24, seed=42)
        noisy3 = torch.empty_like(cw)
        ops.inject_into(cw, noisy3, 1e-3, 24, seed=42)
        out = torch.empty(m * 3, dtype=torch.uint8, device=dev)
        cnt = torch.empty(m, dtype=torch.uint8, device=dev)
        st = ops.new_stats(dev)
        variants = {
            "golay_encode": lambda: ops.golay_encode_into(trip, cw, m),
            "golay_decode_clean": lambda: ops.golay_decode_into(cw, out, cnt, st),
            "golay_decode_ber1e-3": lambda: ops.golay_decode_into(noisy3, out, cnt, st),
            "golay_decode_ber1e-2": lambda: ops.golay_decode_into(noisy, out, cnt, st),
            "golay_decode_ber1e-2_nocount_nostats": lambda: ops.golay_decode_into(noisy, out),
        }
        for k, fn in variants.items():
            med, mn = timed(fn, flush, args.rounds)
            byts = 7 * m if "encode" in k else 8 * m
            res[k] = {"us": med, "min_us": mn, "GBps": byts / med / 1e3}

    if "hamming" in which:
        flat = x.view(-1)
        n = flat.numel()
        cw = torch.empty_like(flat)
        ops.hamming84_encode_into(flat, cw)
        noisy = torch.empty_like(cw)
        ops.inject_into(cw, noisy, 1e-3, 8, seed=42)
        d = torch.empty_like(flat)
        t = torch.empty_like(flat)
        st = ops.new_stats(dev)
        variants = {
            "h84_encode": (lambda: ops.hamming84_encode_into(flat, cw), 2),
            "h84_decode_ber1e-3": (lambda: ops.hamming84_decode_into(noisy, d, t, st), 3),
        }
        for k, (fn, bpv) in variants.items():
            med, mn = timed(fn, flush, args.rounds)
            res[k] = {"us": med, "min_us": mn, "GBps": bpv * n / med / 1e3}

    if "inject" in which:
        flat = x.view(-1)
        n = flat.numel()
        out = torch.empty_like(flat)
        med, mn = timed(lambda: ops.inject_into(flat, out, 1e-3, 8, seed=42), flush, 3)
        res["inject_u8_nb8"] = {"us": med, "philox_per_s": n * 8 / med * 1e6}

    if "interp" in which:
        # H84 decode output of [8,4096,32,128] interpolated along L (seq_dim=1):
        # q, err in and out: 3 B/element
        q = x.clone()
        err = (torch.rand(B, L, H, D, generator=g) < 0.01).to(torch.uint8).mul_(2).to(dev)
        out = torch.empty_like(q)
        n = q.numel()
        outer, length, inner = B, L, H * D
        flag = ops.any_equal(err.view(-1), 2)
        variants = {
            "interp_vec": lambda: ops.interpolate_into(q.view(-1), err.view(-1), out.view(-1),
                                                       outer, length, inner),
            "interp_vec_gated": lambda: ops.interpolate_into(q.view(-1), err.view(-1), out.view(-1),
                                                             outer, length, inner, gate=flag),
            "any_equal": lambda: ops.any_equal(err.view(-1), 2, flag),
            "interp_auto": lambda: ops.interpolate_auto_into(q.view(-1), err.view(-1), out.view(-1),
                                                             outer, length, inner),
            "interpolate_double_errors": lambda: ops.interpolate_double_errors(q, err, seq_dim=1),
        }
        for k, fn in variants.items():
            med, mn = timed(fn, flush, args.rounds)
            byts = n if k == "any_equal" else 3 * n
            res[k] = {"us": med, "min_us": mn, "GBps": byts / med / 1e3}

    if "fused" in which:
        rows, d = B * L * H, D
        xf = torch.randn(rows, d, generator=g).to(torch.float16).to(dev)
        cw = torch.empty(rows, d, dtype=torch.uint8, device=dev)
        sc = torch.empty(rows, dtype=torch.float32, device=dev)
        ops.quantize_encode_rows_into(xf, 2, cw, sc)
        out16 = torch.empty(rows, d, dtype=torch.float16, device=dev)
        out32 = torch.empty(rows, d, dtype=torch.float32, device=dev)
        st = ops.new_stats(dev)
        variants = {
            "quantize_encode_h84_fp16": (lambda: ops.quantize_encode_rows_into(xf, 2, cw, sc),
                                         rows * (3 * d + 4)),
            "decode_dequant_h84_fp16": (lambda: ops.decode_dequant_h84_into(cw, sc, out16, True, st),
                                        rows * (3 * d + 4)),
            "decode_dequant_h84_fp32": (lambda: ops.decode_dequant_h84_into(cw, sc, out32, True, st),
                                        rows * (5 * d + 4)),
        }
        for k, (fn, byts) in variants.items():
            med, mn = timed(fn, flush, args.rounds)
            res[k] = {"us": med, "min_us": mn, "GBps": byts / med / 1e3}

    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
