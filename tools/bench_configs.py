"""Every BASELINE.json config on one MI355X, in one JSON document.

  config 1  H74 encode/decode on [1,128,1,64], backend="cpu", BER 0
  config 2  H84 encode + inject(BER 1e-3, 8 bits, seed 42) + decode on
            [8,4096,32,128]; also the shim's per-row scheme (N = 128 per row)
  config 3  Golay per-head triplets of [8,4096,32,128]: encode + inject(BER
            1e-2, 24 bits, seed 42) + decode; flat packing (M_f) as well
  config 5  Monte-Carlo sweep, 4 codecs x 3 BERs x 3 seeds (kvecc.montecarlo)
plus the extended kernels (packed Golay, paged attention, shim write/read).
Config 4 (GPT-2 forward) is tools/bench_shim.py.

Kernel times are HIP events around `reps` back-to-back launches of one kernel,
after 100 untimed calls (a cold GPU reads 10-15 % high until its clocks ramp)
(inputs resident in HBM, statistics on the device); "pipeline" times one
encode -> inject -> decode chain.  Bytes/unit follow SURVEY 8(d).

usage: python tools/bench_configs.py [--reps 20] > profiles/r01/configs.json
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))

import torch  # noqa: E402

PEAK = 8000.0  # GB/s


def timed(fn, reps, warmup=100, warmup_s=0.3):
    # at least `warmup` calls and `warmup_s` seconds: after an idle set-up the
    # clocks take a few hundred ms to ramp (100 calls of a 50-us kernel read
    # 10-15 % slow; tools/bench_attention.py)
    import time
    t0 = time.perf_counter()
    n = 0
    while n < warmup or time.perf_counter() - t0 < warmup_s:
        fn()
        n += 1
        if n % 50 == 0:
            torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def entry(us, units, unit_name, bytes_per_unit=None):
    e = {"us": round(us, 3), f"{unit_name}_per_s": units / (us * 1e-6)}
    if bytes_per_unit is not None:
        gbs = bytes_per_unit * units / (us * 1e-6) / 1e9
        e.update({"bytes_per_unit": bytes_per_unit, "GBps": gbs, "hbm_frac": gbs / PEAK})
    return e


def config1():
    from kvecc import cpu_ops
    x = torch.randint(0, 16, (1, 128, 1, 64), generator=torch.Generator().manual_seed(0),
                      dtype=torch.uint8)
    t0 = time.perf_counter()
    reps = 200
    for _ in range(reps):
        cw = cpu_ops.hamming74_encode(x)
        dec, (n,) = cpu_ops.hamming74_decode(cw)
    us = (time.perf_counter() - t0) / reps * 1e6
    return {"backend": "cpu", "shape": [1, 128, 1, 64], "ber": 0.0, "bit_exact_roundtrip":
            bool(torch.equal(dec, x)) and n == 0, "encode_decode_us": us,
            "threads": cpu_ops.NUM_THREADS}


def config2(reps):
    from kvecc import ops
    dev = torch.device("cuda:0")
    x = torch.randint(0, 16, (8, 4096, 32, 128), generator=torch.Generator().manual_seed(0),
                      dtype=torch.uint8).to(dev).view(-1)
    n = x.numel()
    cw, noisy, data, et = (torch.empty_like(x) for _ in range(4))
    st = ops.new_stats(dev)
    ops.hamming84_encode_into(x, cw)
    out = {
        "encode": entry(timed(lambda: ops.hamming84_encode_into(x, cw), reps), n, "values", 2),
        "inject_ber1e-3": entry(timed(lambda: ops.inject_into(cw, noisy, 1e-3, 8, seed=42), 3), n,
                                "values"),
        "decode": entry(timed(lambda: ops.hamming84_decode_into(noisy, data, et, st), reps), n,
                        "values", 3),
        "inject_rows_shim_scheme": entry(timed(lambda: ops.inject_rows_into(
            cw, noisy, n // 128, 128, 1e-3, 8, seed_base=42), 3), n, "values"),
    }
    out["inject_ber1e-3"]["philox_per_s"] = out["inject_ber1e-3"]["values_per_s"] * 8

    def pipeline():
        ops.hamming84_encode_into(x, cw)
        ops.inject_into(cw, noisy, 1e-3, 8, seed=42)
        ops.hamming84_decode_into(noisy, data, et, st)
    out["pipeline_encode_inject_decode"] = entry(timed(pipeline, 3), n, "values")
    st.zero_()
    pipeline()
    c, d = ops.read_stats(st)
    out["decode_stats"] = {"corrected": c, "detected": d}
    out["roundtrip_ok_rate"] = float((data == x).float().mean())
    return out


def config3(reps):
    from kvecc import ops
    dev = torch.device("cuda:0")
    x = torch.randint(0, 16, (8, 4096, 32, 128), generator=torch.Generator().manual_seed(0),
                      dtype=torch.uint8).to(dev)
    res = {}
    for name, trip in (("per_head_M_h", None), ("flat_M_f", None)):
        if name == "per_head_M_h":
            t = torch.zeros(8, 4096, 32, 129, dtype=torch.uint8, device=dev)
            t[..., :128] = x
            trip = t.view(-1)
        else:
            flat = x.view(-1)
            trip = torch.cat([flat, flat.new_zeros((3 - flat.numel() % 3) % 3)])
        m = trip.numel() // 3
        cw, noisy = torch.empty(m, dtype=torch.int32, device=dev), torch.empty(m, dtype=torch.int32,
                                                                                device=dev)
        outp = torch.empty(3 * m, dtype=torch.uint8, device=dev)
        cnt = torch.empty(m, dtype=torch.uint8, device=dev)
        st = ops.new_stats(dev)
        ops.golay_encode_into(trip, cw, m)
        r = {"codewords": m,
             "encode": entry(timed(lambda: ops.golay_encode_into(trip, cw, m), reps), m, "codewords", 7),
             "inject_ber1e-2": entry(timed(lambda: ops.inject_into(cw, noisy, 1e-2, 24, seed=42), 3),
                                     m, "codewords"),
             "decode": entry(timed(lambda: ops.golay_decode_into(noisy, outp, cnt, st), reps), m,
                             "codewords", 8)}
        r["inject_ber1e-2"]["philox_per_s"] = r["inject_ber1e-2"]["codewords_per_s"] * 24
        r["encode_plus_decode"] = entry(r["encode"]["us"] + r["decode"]["us"], m, "codewords", 15)

        def pipeline():
            ops.golay_encode_into(trip, cw, m)
            ops.inject_into(cw, noisy, 1e-2, 24, seed=42)
            ops.golay_decode_into(noisy, outp, cnt, st)
        r["pipeline_encode_inject_decode"] = entry(timed(pipeline, 3), m, "codewords")
        res[name] = r
    return res


def extended(reps):
    from kvecc import ops
    dev = torch.device("cuda:0")
    out = {}
    m = 8 * 4096 * 32 * 43
    nib = torch.randint(0, 256, ((3 * m + 1) // 2,), dtype=torch.uint8, device=dev)
    cw3 = ops.golay_encode_packed(nib, m)
    nib2 = torch.empty_like(nib)
    fl = torch.empty((m + 7) // 8, dtype=torch.uint8, device=dev)
    st = ops.new_stats(dev)
    out["packed_golay_encode"] = entry(timed(lambda: ops.golay_encode_packed_into(nib, cw3, m), reps),
                                       m, "codewords", 4.5)
    out["packed_golay_decode"] = entry(timed(lambda: ops.golay_decode_packed_into(
        cw3, nib2, fl, m, st), reps), m, "codewords", 4.625)
    n = 8 * 4096 * 32 * 128
    hn = torch.randint(0, 256, (n // 2,), dtype=torch.uint8, device=dev)
    hcw = ops.hamming84_encode_packed(hn, n)
    hn2 = torch.empty_like(hn)
    ht = torch.empty(n // 4, dtype=torch.uint8, device=dev)
    out["packed_h84_encode"] = entry(timed(lambda: ops.hamming84_encode_packed_into(hn, hcw, n), reps),
                                     n, "values", 1.5)
    out["packed_h84_decode"] = entry(timed(lambda: ops.hamming84_decode_packed_into(
        hcw, hn2, ht, n, st), reps), n, "values", 1.75)
    # paged decode attention, [8 seqs x 4096 ctx, 32 heads, D=128]; MHA and
    # GQA with 8 cache heads (Llama-style 32/8: a workgroup serves 4 query heads)
    for codec, hkv in (("hamming84", 32), ("golay", 32), ("golay_packed", 32),
                       ("hamming84", 8), ("golay", 8), ("golay_packed", 8)):
        b, hq, d, ctx, bs = 8, 32, 128, 4096, 16
        per = d if codec == "hamming84" else (d + 2) // 3
        if codec == "golay_packed":  # bytes per token row (KVECC_GOLAY_PACKED_ROW)
            per = (3 * per + 3) // 4 * 4
        nb = ctx // bs
        blocks = b * nb
        from kvecc.memory_layout import kv_cache_pair  # K/V as SimpleBlockManager lays them out
        kc, vc = kv_cache_pair((blocks, 1, hkv, bs * per), torch.int32 if codec == "golay" else torch.uint8, dev)
        kc.random_(0, 1 << 24 if codec == "golay" else 256)
        vc.copy_(kc.roll(1, 0))
        ks = torch.rand(blocks, 1, hkv, bs, device=dev)
        vs = torch.rand_like(ks)
        table = torch.randperm(blocks, device=dev).to(torch.int32).view(b, nb)
        lens = torch.full((b,), ctx, dtype=torch.int32, device=dev)
        q = torch.randn(b, hq, d, device=dev).half()
        o = torch.empty_like(q)
        us = timed(lambda: ops.paged_attention_into(q, kc, vc, table, lens, ks, vs, o, 0, bs,
                                                    1 / math.sqrt(d), codec, ctx), reps)
        byts = 2 * b * ctx * hkv * (per * kc.element_size() + 4)
        e = entry(us, b * ctx, "tokens")
        e.update({"heads": hq, "kv_heads": hkv, "bytes": byts, "GBps": byts / (us * 1e-6) / 1e9,
                  "hbm_frac": byts / (us * 1e-6) / 1e9 / PEAK})
        out[f"paged_attention_{codec}" + ("" if hkv == hq else f"_gqa{hq}x{hkv}")] = e
    return out


def config5():
    from kvecc.montecarlo import HipShard, MonteCarloConfig, run_sweep
    cfg = MonteCarloConfig()
    shard = HipShard(cfg, 0, 1, "cuda:0")
    rows, sec = run_sweep(cfg, shard)
    return {"trials": len(rows), "seconds": sec, "shape": list(cfg.shape),
            "values_per_trial": 8 * 4096 * 32 * 128,
            "trial_values_per_s": len(rows) * 8 * 4096 * 32 * 128 / sec, "rows": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    doc = {"device": torch.cuda.get_device_name(0), "timing": "HIP events, back-to-back launches, "
           "inputs resident in HBM, peak 8 TB/s", "config1": config1(),
           "config2": config2(args.reps), "config3": config3(args.reps),
           "extended": extended(args.reps), "config5": config5()}
    print(json.dumps(doc, indent=1, default=float))


if __name__ == "__main__":
    main()
