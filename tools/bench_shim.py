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


def peak_added(fn):
    """Bytes one call of fn adds to the allocator's peak over what was allocated before it."""
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    fn()
    torch.cuda.synchronize()
    return torch.cuda.max_memory_allocated() - base


def compiled_run(model, ids, eager_fwd, args):
    """torch.compile(model, fullgraph=True) of the patched forward: forward time
    (median), peak memory added by one forward against eager, ECC statistics
    against eager, and the cache bytes per layer (the size a functionalized
    clone of k_cache / v_cache per write would add)."""
    import time

    from kvecc.ecc_shim import get_ecc_stats, reset_ecc_cache
    torch._dynamo.reset()
    comp = torch.compile(model, fullgraph=True, backend=args.compile)

    def cfwd():
        reset_ecc_cache(model)
        return comp(ids)

    t0 = time.perf_counter()
    cfwd()
    torch.cuda.synchronize()
    compile_s = time.perf_counter() - t0
    med, mn = timed(cfwd, args.steps, args.warmup)
    eager_med = timed(eager_fwd, args.steps, args.warmup)[0]
    mem_e = peak_added(eager_fwd)
    mem_c = peak_added(cfwd)
    reset_ecc_cache(model)
    logits = comp(ids).logits
    st = get_ecc_stats(model)
    reset_ecc_cache(model)
    ref = model(ids).logits
    st_e = get_ecc_stats(model)
    mgr = model._ecc_block_manager
    per_layer = mgr.k_cache.numel() * mgr.k_cache.element_size() // mgr.k_cache.shape[1]
    return {"backend": args.compile, "forward_ms": med, "min_ms": mn, "eager_forward_ms": eager_med,
            "compile_s": compile_s, "peak_added_bytes": {"eager": mem_e, "compiled": mem_c},
            "cache_bytes_per_layer_side": per_layer, "cache_bytes_side": mgr.k_cache.numel() * mgr.k_cache.element_size(),
            "stats_equal_to_eager": st == st_e,
            "max_abs_logit_diff": float((logits.float() - ref.float()).abs().max())}


def cpu_only(args):
    """Config 4 on the host backend alone (fp32 on the CPU): forward time and statistics."""
    import time

    from transformers import GPT2Config, GPT2LMHeadModel
    from kvecc.ecc_shim import ECCShimConfig, get_ecc_stats, patch_model_with_ecc_attention, reset_ecc_cache
    torch.manual_seed(0)
    model = GPT2LMHeadModel(GPT2Config(n_positions=1024)).eval()
    ids = torch.randint(0, 50257, (1, args.seq), generator=torch.Generator().manual_seed(0))
    out = {"config": {"model": "gpt2 12L/12H/768 random-init fp32 (host)", "seq_len": args.seq,
                      "codec": args.codec, "use_interpolation": bool(args.interp), "block_size": 16,
                      "seed": 42, "backend": "cpu", "threads": torch.get_num_threads()}, "runs": []}
    with torch.no_grad():
        t0 = time.perf_counter()
        model(ids)
        out["unpatched_ms"] = (time.perf_counter() - t0) * 1e3
        for ber in args.bers:
            cfg = ECCShimConfig(codec=args.codec, ber=ber, inject_errors=ber > 0, seed=42, block_size=16,
                                use_interpolation=bool(args.interp), backend="cpu")
            with patch_model_with_ecc_attention(model, cfg, num_blocks=(args.seq + 15) // 16):
                ts = []
                for _ in range(max(args.steps, 1)):
                    reset_ecc_cache(model)
                    t0 = time.perf_counter()
                    res = model(ids, labels=ids)
                    ts.append(time.perf_counter() - t0)
                st = get_ecc_stats(model)
            out["runs"].append({"ber": ber, "forward_ms": statistics.median(ts) * 1e3, "loss": float(res.loss),
                                "stats": st})
    print(json.dumps(out))


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
    ap.add_argument("--compile", choices=("none", "inductor", "aot_eager"), default="none",
                    help="also time torch.compile(model, fullgraph=True) of the patched forward with this "
                         "backend, and the peak memory a forward adds (eager vs compiled): a "
                         "functionalized copy of the caches would show as about one cache per write")
    ap.add_argument("--no-gpu", action="store_true", help="host backend only (with --cpu-backend)")
    args = ap.parse_args()
    from transformers import GPT2Config, GPT2LMHeadModel
    from kvecc.ecc_shim import (ECCShimConfig, get_ecc_stats, patch_model_with_ecc_attention,
                                reset_ecc_cache)
    if args.no_gpu:
        return cpu_only(args)
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
                run = {"ber": ber, "forward_ms": med, "min_ms": mn, "graph_ms": graph_ms,
                       "tokens_per_s": args.seq / (med * 1e-3), "loss": float(res.loss),
                       "logits_finite": bool(torch.isfinite(res.logits).all()), "stats": st}
                if args.compile != "none":
                    run["compiled"] = compiled_run(model, ids, fwd, args)
            out["runs"].append(run)
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
