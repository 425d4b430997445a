"""BASELINE config 4: Hamming(8,4)+interpolation inside patch_model_with_ecc_attention.

Random-init GPT-2 (12 layers, 12 heads, 768 hidden, n_positions 1024), fp16,
input_ids = randint(0, 50257, (1, 1024)) with seed 0, ECCShimConfig(codec,
use_interpolation, ber, inject_errors=ber>0, seed=42, block_size=16).
Reports the forward latency of the patched model (cache reset before every
forward, as the reference's per-text loop does) next to the unpatched model,
plus get_ecc_stats of one forward.  Prints one JSON line.

usage: python tools/bench_shim.py [--codec hamming84] [--interp 1] [--bers 0 1e-3 1e-2]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))

import torch  # noqa: E402


def graphed(fn, warmup=3):
    """Capture fn (one forward) in a HIP graph after warm-up on a side stream;
    returns a callable that replays it (its outputs live in the graph's pool)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g.replay


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="hamming84")
    ap.add_argument("--interp", type=int, default=1)
    ap.add_argument("--golay-storage", default="int32", choices=["int32", "packed"])
    ap.add_argument("--bers", type=float, nargs="*", default=[0.0, 1e-3, 1e-2])
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--composed", action="store_true",
                    help="per-op kernels instead of the fused cache write/read")
    ap.add_argument("--graph", action="store_true",
                    help="time HIP-graph replays of the whole forward (patched and unpatched)")
    ap.add_argument("--cpu-backend", action="store_true",
                    help="also run the same forward on the host backend (fp32, CPU)")
    args = ap.parse_args()
    from transformers import GPT2Config, GPT2LMHeadModel
    from kvecc.ecc_shim import (ECCShimConfig, get_ecc_stats, patch_model_with_ecc_attention,
                                reset_ecc_cache)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = GPT2LMHeadModel(GPT2Config(n_positions=1024)).half().to(dev).eval()
    ids = torch.randint(0, 50257, (1, args.seq), generator=torch.Generator().manual_seed(0)).to(dev)
    out = {"config": {"model": "gpt2 12L/12H/768 random-init fp16", "seq_len": args.seq,
                      "codec": args.codec, "golay_storage": args.golay_storage,
                      "use_interpolation": bool(args.interp),
                      "block_size": 16, "seed": 42, "fused": not args.composed}, "runs": []}
    with torch.no_grad():
        med, mn = timed(lambda: model(ids), args.steps, args.warmup)
        out["unpatched_ms"] = med
        if args.graph:
            out["unpatched_graph_ms"] = timed(graphed(lambda: model(ids)), args.steps, args.warmup)[0]
        nblocks = (args.seq + 15) // 16
        for ber in args.bers:
            cfg = ECCShimConfig(codec=args.codec, ber=ber, inject_errors=ber > 0, seed=42,
                                block_size=16, use_interpolation=bool(args.interp),
                                fused=not args.composed, golay_storage=args.golay_storage)
            with patch_model_with_ecc_attention(model, cfg, num_blocks=nblocks):
                def fwd():
                    reset_ecc_cache(model)
                    return model(ids)
                med, mn = timed(fwd, args.steps, args.warmup)
                graph_ms = timed(graphed(fwd), args.steps, args.warmup)[0] if args.graph else None
                reset_ecc_cache(model)
                res = model(ids, labels=ids)
                st = get_ecc_stats(model)
            out["runs"].append({"ber": ber, "forward_ms": med, "min_ms": mn, "graph_ms": graph_ms,
                                "tokens_per_s": args.seq / (med * 1e-3),
                                "loss": float(res.loss),
                                "logits_finite": bool(torch.isfinite(res.logits).all()),
                                "stats": st})
        if args.cpu_backend:
            import time
            cpu_model = GPT2LMHeadModel(GPT2Config(n_positions=1024)).eval()
            cpu_model.load_state_dict({k: t.float().cpu() for k, t in model.state_dict().items()})
            cpu_ids = ids.cpu()
            out["cpu_backend"] = []
            for ber in args.bers:
                cfg = ECCShimConfig(codec=args.codec, ber=ber, inject_errors=ber > 0, seed=42,
                                    block_size=16, use_interpolation=bool(args.interp),
                                    backend="cpu")
                with patch_model_with_ecc_attention(cpu_model, cfg, num_blocks=nblocks):
                    reset_ecc_cache(cpu_model)
                    t0 = time.perf_counter()
                    res = cpu_model(cpu_ids, labels=cpu_ids)
                    el = time.perf_counter() - t0
                    st = get_ecc_stats(cpu_model)
                gpu_run = next(r for r in out["runs"] if r["ber"] == ber)
                out["cpu_backend"].append({"ber": ber, "forward_ms": el * 1e3, "loss": float(res.loss),
                                           "dtype": "fp32", "threads": torch.get_num_threads(),
                                           "stats": st,
                                           # the error counts depend on the injected bits only
                                           # (per-row Philox seeds), not on the fp16/fp32 data
                                           "stats_equal_to_gpu": st == gpu_run["stats"]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
