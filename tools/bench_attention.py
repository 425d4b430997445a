"""Paged decode attention with inline ECC decode: HBM roofline measurement.

One decode step of [B, H, D] queries over a paged Hamming(8,4) (or Golay) KV
cache of `ctx` tokens per sequence (BASELINE's [8, 4096, 32, 128] shape by
default).  Algorithmic bytes per launch = K + V codewords + K/V scales + the
block table; reported against the 8 TB/s HBM peak.  Prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="hamming84")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=32)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=4096)
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100,
                    help="untimed calls first, repeated until --warmup-s seconds have passed")
    ap.add_argument("--warmup-s", type=float, default=0.5,
                    help="minimum warm-up time: the clocks take a few hundred ms to ramp on an idle GPU "
                         "(100 calls = 7 ms read 10-15 %% slow)")
    ap.add_argument("--passes", type=int, default=5, help="timed passes of --iters calls; the median is reported")
    ap.add_argument("--data", choices=["random", "encoded"], default="random",
                    help="cache contents: random bytes / int32 words (every codeword decodes through the full "
                         "correction path: the decode tables' worst case), or encoded random INT4 values with "
                         "bit errors at --ber (what a cache holds)")
    ap.add_argument("--ber", type=float, default=None, help="encoded data: BER (default 1e-3 H84, 1e-2 Golay)")
    args = ap.parse_args()
    from kvecc import ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    nb = (args.ctx + args.bs - 1) // args.bs
    blocks = args.batch * nb
    per = args.d if args.codec == "hamming84" else (args.d + 2) // 3
    if args.codec == "golay_packed":  # bytes per token row (KVECC_GOLAY_PACKED_ROW)
        per = (3 * per + 3) // 4 * 4
    from kvecc.memory_layout import kv_cache_pair  # K/V as SimpleBlockManager lays them out
    kc, vc = kv_cache_pair((blocks, 1, args.kv_heads, args.bs * per),
                           torch.int32 if args.codec == "golay" else torch.uint8, dev)
    if args.data == "random":
        kc.random_(0, 1 << 24 if args.codec == "golay" else 256, generator=g)
        vc.copy_(kc.roll(1, 0))
    else:
        ber = args.ber if args.ber is not None else (1e-3 if args.codec == "hamming84" else 1e-2)
        for side, dst in enumerate((kc, vc)):
            x = torch.randint(0, 16, (blocks, 1, args.kv_heads, args.bs, args.d), device=dev, generator=g,
                              dtype=torch.uint8)
            if args.codec == "hamming84":
                cw = ops.hamming84_encode(x.view(-1))
                ops.inject_into(cw, cw, ber, 8, seed=42 + side)
                dst.view(-1).copy_(cw)
            else:
                gg = (args.d + 2) // 3
                cw = ops.golay_encode_rows(x).view(-1)
                ops.inject_into(cw, cw, ber, 24, seed=42 + side)
                if args.codec == "golay":
                    dst.view(-1).copy_(cw)
                else:  # 3 bytes per codeword, rows padded to KVECC_GOLAY_PACKED_ROW
                    b3 = torch.stack([(cw >> (8 * k)) & 0xFF for k in range(3)], -1).to(torch.uint8)
                    dst.view(blocks, 1, args.kv_heads, args.bs, per)[..., :3 * gg].copy_(
                        b3.view(blocks, 1, args.kv_heads, args.bs, 3 * gg))
            del x
    ks = torch.rand(blocks, 1, args.kv_heads, args.bs, device=dev, generator=g)
    vs = torch.rand_like(ks)
    table = torch.randperm(blocks, device=dev, generator=g).to(torch.int32).view(args.batch, nb)
    lens = torch.full((args.batch,), args.ctx, dtype=torch.int32, device=dev)
    q = torch.randn(args.batch, args.heads, args.d, device=dev, generator=g).half()
    out = torch.empty_like(q)
    call = lambda: ops.paged_attention_into(q, kc, vc, table, lens, ks, vs, out, 0, args.bs,  # noqa
                                            1 / math.sqrt(args.d), args.codec, args.ctx)
    import statistics
    import time
    t0 = time.perf_counter()
    while True:
        for _ in range(args.warmup):
            call()
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= args.warmup_s:
            break
    passes = []
    for _ in range(args.passes):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            call()
        e1.record()
        torch.cuda.synchronize()
        passes.append(e0.elapsed_time(e1) / args.iters)
    ms = statistics.median(passes)
    tokens = args.batch * args.ctx
    cw_bytes = 2 * tokens * args.kv_heads * per * kc.element_size()
    bytes_ = cw_bytes + 2 * tokens * args.kv_heads * 4 + table.numel() * 4
    gbs = bytes_ / (ms * 1e-3) / 1e9
    print(json.dumps({"kernel": "paged_attention", "codec": args.codec, "batch": args.batch,
                      "heads": args.heads, "kv_heads": args.kv_heads, "head_dim": args.d,
                      "ctx": args.ctx, "ms_per_call": ms, "bytes_per_call": bytes_,
                      "pass_ms": [round(x, 5) for x in passes],
                      "achieved_gbs": gbs, "hbm_frac": gbs / 8000.0,
                      "data": args.data if args.data == "random" else f"encoded, BER {ber}",
                      "includes": "split kernel + combine kernel + workspace alloc"}))


if __name__ == "__main__":
    main()
