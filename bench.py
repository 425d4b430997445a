"""Headline benchmark: Golay(24,12) INT4 encode+decode on [B=8, L=4096, H=32, D=128].

Metric (BASELINE.json): "INT4 codewords/sec encode+decode (Golay24, L=4096) +
achieved HBM GB/s", configuration 3: Golay(24,12) triplet encode+decode on
[8,4096,32,128] at BER 1e-2 on one MI355X.

One step = golay_encode of the per-head-padded triplets (ecc_shim.py packing:
D=128 -> 129 -> 43 codewords per head, M = 45,088,768 codewords) followed by
golay_decode of those codewords corrupted at BER 1e-2 (the corruption is
injected once, before timing, with the reference's Philox stream; its own
throughput is measured separately and reported under "inject").  Inputs are
resident in HBM before the timed region; statistics stay on the device.

Multi-GPU (torchrun, one process per GPU): weak scaling -- every rank owns its
own [8,4096,32,128] shard (global codeword offset rank*M, so the fault pattern
equals a single-device run over the concatenated tensor); no collective in the
data path, one RCCL all_reduce of the decode statistics after timing.

Roofline: on every --event-every'th timed step the encode and decode kernels
carry a pair of HIP events in their own dispatch (kvecc_time_next_launch ->
hipExtLaunchKernel), so the stamps are the kernels' own start and end (they
agree with rocprofv3's kernel durations); achieved = 8 B/codeword * M / mean
decode time.  Such a dispatch costs the step ~8 us, hence the sampling.
--timing markers brackets the launches with hipEventRecord instead (each record
adds ~2-4 us to the bracketed kernel's time).

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

B, L, H, D = 8, 4096, 32, 128
BER = 1e-2
SEED = 42
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
DECODE_BYTES_PER_CW = 8  # 4 B codeword in, 3 B triplet + 1 B count out
ENCODE_BYTES_PER_CW = 7  # 3 B triplet in, 4 B codeword out


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="time budget of the CPU baseline sample (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads for the CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--side-warmup", type=int, default=100,
                    help="warm-up calls before each optional section (packed, rows, fused reads); the "
                         "clocks ramp after the idle set-up of each section: the fused H(8,4) read "
                         "timed 151-154 us after 5 calls and 139-141 after 100 "
                         "(profiles/r03/fused/fused_warm.log)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-inject", action="store_true")
    ap.add_argument("--no-packed", action="store_true")
    ap.add_argument("--timing", choices=("kernel", "markers"), default="kernel",
                    help="kernel: events carried by each timed launch (hipExtLaunchKernel); "
                         "markers: hipEventRecord around the launches of sampled steps")
    ap.add_argument("--event-every", type=int, default=10,
                    help="time the kernels of every k-th timed step (a timed dispatch costs the "
                         "step ~8 us; timing every step cost 7-9%% of throughput)")
    ap.add_argument("--roofline-samples", type=int, default=30,
                    help="extra encode/decode steps after the timed region whose kernels carry "
                         "events, added to the roofline's kernel-time sample")
    ap.add_argument("--no-fused", action="store_true",
                    help="skip the fused Golay read (shim_read_batch) measurement")
    ap.add_argument("--no-rows", action="store_true",
                    help="skip the per-head rows (golay_encode_rows / decode_rows) measurement")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for N > 1 (nccl = RCCL; gloo only to rehearse several "
                         "ranks on one GPU)")
    ap.add_argument("--dist", action="store_true",
                    help="create the RCCL process group even at world size 1 (exercises the "
                         "barrier and the stats/timing all-reduces on one GPU)")
    ap.add_argument("--no-interp", action="store_true", help="skip the interpolation roofline section")
    ap.add_argument("--no-quant", action="store_true",
                    help="skip the fused quantize+encode / decode+dequantize roofline section")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the encode+inject+decode pipeline")
    ap.add_argument("--no-montecarlo", action="store_true", help="skip the config-5 sweep section")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the strong-scaling section (the headline's one tensor split over the ranks)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak (default): every rank owns a whole [8,4096,32,128] tensor; strong: the ONE "
                         "[8,4096,32,128] tensor is split along B over the ranks (at most 8)")
    ap.add_argument("--no-sections", action="store_true",
                    help="headline only: skip every optional section and the CPU baselines")
    ap.add_argument("--sections", default=None,
                    help="comma-separated sections to run, every other one skipped: " + ",".join(SECTIONS))
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--inject-pmc-json", default=os.path.join(REPO, "profiles", "inject_valu.json"),
                    help="VALU instructions per Philox (rocprofv3 SQ_INSTS_VALU pass) for the inject roofline")
    a = ap.parse_args(argv)
    if a.no_sections and a.sections is None:
        a.sections = ""
    if a.sections is not None:
        keep = {s.strip() for s in a.sections.split(",") if s.strip()}
        unknown = keep - set(SECTIONS)
        if unknown:
            ap.error(f"unknown section(s) {sorted(unknown)}; known: {','.join(SECTIONS)}")
        for s, flag in SECTIONS.items():
            setattr(a, flag, s not in keep)
    return a


# section name -> the --no-* flag that skips it
SECTIONS = {"cpu": "no_cpu_baseline", "inject": "no_inject", "packed": "no_packed", "fused": "no_fused",
            "rows": "no_rows", "interp": "no_interp", "quant": "no_quant", "pipeline": "no_pipeline",
            "montecarlo": "no_montecarlo", "strong": "no_strong"}


def cpu_baseline(budget_s, threads):
    """The C oracle (a port of the reference path) timed on the host: Golay
    encode + decode of a bounded sample of the same workload, one chunk per
    host thread (ctypes releases the GIL, so the threads run in parallel)."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    from oracle import oracle
    oracle.lib()
    g = np.random.default_rng(0)
    m = 1 << 16  # codewords per chunk
    chunks = []
    for t in range(threads):
        trip = g.integers(0, 16, size=(m, 3), dtype=np.int64).astype(np.uint8)
        cw = oracle.golay_encode(trip)
        noisy, _, _ = oracle.inject(cw[: 1 << 11], BER, 24, SEED)  # decode sees errors
        cw[: 1 << 11] = noisy
        chunks.append((trip, cw))

    def work(i):
        trip, cw = chunks[i]
        oracle.golay_encode(trip)
        oracle.golay_decode(cw)
        return m

    done = 0
    with ThreadPoolExecutor(threads) as pool:
        t0 = time.perf_counter()
        while True:
            done += sum(pool.map(work, range(threads)))
            el = time.perf_counter() - t0
            if el >= budget_s:
                break
    return {"value": done / el, "unit": "codewords/s", "cores": threads, "kind": "port",
            "host": host_info(),
            "sample": f"{done} codewords of Golay encode+decode (BER 1e-2 on a slice) in {el:.1f} s, "
                      f"oracle/kvecc_oracle.c on {threads} host threads"}


def _warm(fn, n, seconds=0.25):
    """At least n calls of fn and `seconds` of them: after a set-up phase with
    the GPU idle the clocks take a few hundred ms to ramp, and back-to-back
    full-grid kernels run 10-30 % slow for their first ~40 launches
    (profiles/r04/fused/sustained.log)."""
    t0 = time.perf_counter()
    k = 0
    while k < n or time.perf_counter() - t0 < seconds:
        fn()
        k += 1
        if k % 50 == 0:
            torch.cuda.synchronize()


def kernel_ms(dev, call, steps, warmup):
    """Mean duration of the first kvecc kernel each call() launches, from HIP
    events carried by that kernel's own dispatch (kvecc_time_next_launch), over
    `steps` launches after the time-based warm-up."""
    from kvecc import ops
    _warm(call, warmup)
    evs = [ops.kernel_timer(dev) for _ in range(steps)]
    torch.cuda.synchronize()
    for k in range(steps):
        ops.time_next_launch(*evs[k])
        call()
    torch.cuda.synchronize()
    return sum(e[0].elapsed_time(e[1]) for e in evs) / steps


def call_ms(dev, call, steps, warmup):
    """Mean time per call() from events recorded around `steps` back-to-back
    calls on the current stream: every kernel the call launches and the gaps
    between them (for calls of more than one kernel)."""
    _warm(call, warmup)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        call()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def hbm_roofline(kernel, nbytes, ms, unit_note):
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": kernel, "kernel_ms": ms, "bytes_per_launch": nbytes,
            "bytes_per_unit": unit_note, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS}


def interp_bench(dev, steps, warmup):
    """Double-error interpolation along L (interpolation_triton.py:120-265) of the
    H(8,4) decode of [8,4096,32,128] at BER 1e-3 -- the tensor the config-5
    hamming84_interp trial interpolates (each (b, h, d) column a sequence).
    3 B per element (q and err in, out); the kernel alone, and the API call
    (kvecc_interpolate_auto: the same pass records the no-double fast path)."""
    from kvecc import ops
    n = B * L * H * D
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 16, (n,), generator=g, dtype=torch.uint8).to(dev)
    cw = ops.hamming84_encode(x)
    ops.inject_into(cw, cw, 1e-3, 8, seed=SEED)
    q = torch.empty_like(x)
    et = torch.empty_like(x)
    ops.hamming84_decode_into(cw, q, et)
    del cw, x
    out = torch.empty_like(q)
    ms = kernel_ms(dev, lambda: ops.interpolate_into(q, et, out, B, L, H * D), steps, warmup)
    # the API call is two launches (the recording pass and the fix-up kernel,
    # which exits at once here): timed as a whole, around the calls
    ms_api = call_ms(dev, lambda: ops.interpolate_auto_into(q, et, out, B, L, H * D), steps, warmup)
    r = hbm_roofline("interp_tile_kernel<false>", 3 * n, ms, "3 B/element (q, err in; out)")
    r.update({"workload": "interpolate_double_errors along L of the H(8,4) decode of [8,4096,32,128], BER 1e-3",
              "doubles": int((et == 2).sum()),
              "api": dict(hbm_roofline("kvecc_interpolate_auto: interp_tile_kernel<true> + interp_fixup_kernel",
                                       3 * n, ms_api, "3 B/element"),
                          timing="events around back-to-back API calls (both launches and the gap between them)"),
              "timing": f"HIP events carried by the dispatch, mean of {steps} launches after >= {warmup} "
                        "warm-up calls and >= 0.25 s"})
    return r


def quant_bench(dev, steps, warmup):
    """Fused quantize + Hamming(8,4) encode (fused_kernels.py:18-160) of fp16 rows
    [8*4096*32, 128] (D*3+4 B/row: 2 B in and 1 B out per value, fp32 scale out),
    and the fused H(8,4) decode + dequantize (fused_kernels.py:272-437) of those
    codewords at BER 1e-3 back to fp16 (D*3+4 B/row) and fp32 (D*5+4 B/row)."""
    from kvecc import _lib, ops
    rows = B * L * H
    g = torch.Generator().manual_seed(5)
    x = torch.randn(rows, D, generator=g, dtype=torch.float32).to(dev).to(torch.float16)
    cw = torch.empty(rows, D, dtype=torch.uint8, device=dev)
    sc = torch.empty(rows, dtype=torch.float32, device=dev)
    ms_q = kernel_ms(dev, lambda: ops.quantize_encode_rows_into(x, _lib.CODEC_H84, cw, sc), steps, warmup)
    del x
    ops.inject_into(cw.view(-1), cw.view(-1), 1e-3, 8, seed=SEED)
    st = ops.new_stats(dev)
    res = {"quantize_encode": hbm_roofline("quantize_encode_tile_kernel (fp16 -> H84)", rows * (3 * D + 4), ms_q,
                                           "D*3+4 B/row (fp16 in, codeword + fp32 scale out)")}
    for name, dt, per in (("decode_dequant", torch.float16, 3 * D + 4),
                          ("decode_dequant_fp32", torch.float32, 5 * D + 4)):
        out = torch.empty(rows, D, dtype=dt, device=dev)
        ms = kernel_ms(dev, lambda: ops.decode_dequant_h84_into(cw, sc, out, True, st), steps, warmup)
        res[name] = hbm_roofline(f"decode_dequant_tile_kernel (-> {str(dt)[6:]})", rows * per, ms,
                                 f"{'D*3+4' if per == 3 * D + 4 else 'D*5+4'} B/row (codeword + scale in, "
                                 f"{str(dt)[6:]} out)")
        del out
    res.update({"workload": f"fp16 rows [{rows}, {D}] = [8,4096,32,128] K, row absmax INT4, Hamming(8,4), "
                            "BER 1e-3 between encode and decode",
                "timing": f"HIP events carried by the dispatch, mean of {steps} launches after >= {warmup} "
                          "warm-up calls and >= 0.25 s"})
    return res


def table_digest(rows):
    """sha256 of the sweep's [trials x 5] counter table as little-endian int64,
    rows in trial order: equal for every world size when the sharding is exact."""
    import hashlib
    import struct
    from kvecc.montecarlo import STAT_NAMES
    flat = [int(r[k]) for r in rows for k in STAT_NAMES]
    return hashlib.sha256(struct.pack(f"<{len(flat)}q", *flat)).hexdigest()


def gather_floats(dist, world, dev, vals, gloo):
    """Every rank's `vals` (a list of floats), rank order; [vals] without a group."""
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    if dist is None:
        return [t.tolist()]
    if gloo:
        t = t.cpu()
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def montecarlo_bench(dev, dist=None, rank=0, world=1, gloo=False):
    """BASELINE config 5: the 36-trial codec sweep (4 codecs x BER
    {1e-4,1e-3,1e-2} x seeds {42,101,997}) at [8,4096,32,128] through
    kvecc.montecarlo.run_sweep -- evaluation/sweep.py:352-626 driven as
    evaluation/experiments/monte_carlo.py:75-128 do, batch-sharded: rank r runs
    batch rows shard_bounds(8, r, N) of every trial (one fused launch per trial,
    kvecc_mc_trial, global Philox offsets), one statistics fold, and the sweep's
    ONE all_reduce(SUM) of the int64 [36 x 5] table (RCCL over xGMI).  Every
    rank runs it; a warm-up sweep first, the second timed between barriers
    (the all-reduce inside), the slowest rank's time reported."""
    from kvecc import montecarlo as mc
    cfg = mc.MonteCarloConfig()
    shard = mc.HipShard(cfg, rank, world, dev)
    mc.run_sweep(cfg, shard, dist, rank)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows, compute_s = mc.run_sweep(cfg, shard, dist, rank)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    per_rank = gather_floats(dist, world, dev, [wall, compute_s, shard.b0, shard.b1], gloo)
    sec = max(p[0] for p in per_rank)
    return {"workload": "config 5: 36 trials, 4 codecs x BER {1e-4,1e-3,1e-2} x seeds {42,101,997}, "
                        f"[8,4096,32,128] batch-sharded over {world} rank(s)",
            "world": world, "trials": len(rows), "ms": sec * 1e3,
            "ms_per_trial": sec * 1e3 / len(rows), "fused": shard.fused,
            "values_per_s": len(rows) * B * L * H * D / sec,
            "table_sha256": table_digest(rows),
            "per_rank": [{"rank": r, "batch_rows": [int(p[2]), int(p[3])], "ms": p[0] * 1e3,
                          "trials_ms": p[1] * 1e3} for r, p in enumerate(per_rank)],
            "collective": ("one all_reduce(SUM) of the int64 [36 x 5] table "
                           f"({dist.get_backend()})" if dist is not None else None),
            "scaling": "strong (the config's one [8,4096,32,128] tensor split along B)",
            "bound": "valu (Philox per bit; the trial reads the ground truth once)",
            "timing": "wall clock of the second run_sweep between barriers (device-synchronised, the "
                      "all-reduce included), max over ranks; trials_ms = the rank's trials alone"}


def strong_setup(dev, rank, world):
    """The headline's workload split along B: the ONE [8,4096,32,128] tensor
    (seed 0, identical for every world size), rank r encoding / decoding batch
    rows shard_bounds(8, r, N) with the injection told the global codeword
    count and the shard's global offset -- the fault pattern, and so the
    all-reduced statistics, of any world size equal the single-GPU run's."""
    from kvecc import montecarlo as mc
    if world > B:
        raise ValueError(f"strong scaling splits B={B} rows: at most {B} ranks, got {world}")
    b0, b1 = mc.shard_bounds(B, rank, world)
    gen = torch.Generator().manual_seed(0)
    x = torch.randint(0, 16, (B, L, H, D), generator=gen, dtype=torch.uint8)[b0:b1].to(dev)
    per_b = L * H * ((D + 2) // 3)
    return x, b0 * per_b, B * per_b


def strong_section(dev, dist, rank, world, steps, warmup, gloo):
    """Strong scaling beside the weak headline: the same encode +
    decode step over the one [8,4096,32,128] tensor split along B, wall clock
    of `steps` steps between barriers, slowest rank; statistics all-reduced."""
    from kvecc import ops
    x, off, gn = strong_setup(dev, rank, world)
    h = Headline(dev, x, off, gn)
    del x
    for _ in range(warmup):
        h.step()
    h.stats.zero_()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        h.step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    st = ops.stats_totals(h.stats)
    inj = ops.stats_totals(h.inj_stats)
    if dist is not None:
        if gloo:
            st, inj = st.cpu(), inj.cpu()
        dist.all_reduce(st, op=dist.ReduceOp.SUM)
        dist.all_reduce(inj, op=dist.ReduceOp.SUM)
    per_rank = gather_floats(dist, world, dev, [wall, h.m], gloo)
    sec = max(p[0] for p in per_rank)
    total = gn * steps
    return {"workload": f"golay24 per-head encode+decode of ONE [B=8,L=4096,H=32,D=128] tensor split along "
                        f"B over {world} rank(s)",
            "world": world, "codewords_total": gn, "value": total / sec, "unit": "codewords/s",
            "ms_per_step": sec / steps * 1e3, "steps": steps,
            "decode_stats": dict(zip(("bits_corrected", "uncorrectable"), st.tolist())),
            "inject_stats": dict(zip(("flips", "affected"), inj.tolist())),
            "per_rank": [{"rank": r, "codewords": int(p[1]), "elapsed_s": p[0]} for r, p in enumerate(per_rank)],
            "timing": f"wall clock of {steps} steps between barriers after {warmup} warm-up steps, max over ranks"}


class Headline:
    """One rank's resident encode+decode workload: nibbles x [b, L, H, D] padded
    per head (ecc_shim.py:669-679, D=128 -> 43 codewords), encoded once and
    corrupted at BER 1e-2 with the reference's Philox stream at global codeword
    offset `offset0` of `global_n` (injection runs here, before any timing);
    step() = golay_encode + golay_decode of those buffers."""

    def __init__(self, dev, x, offset0, global_n):
        from kvecc import ops
        self.ops = ops
        b = x.shape[0]
        gsz = (D + 2) // 3
        trip = torch.zeros(b, L, H, gsz * 3, dtype=torch.uint8, device=dev)
        trip[..., :D] = x
        self.trip = trip.view(-1, 3)
        self.m = m = self.trip.shape[0]
        self.cw = torch.empty(m, dtype=torch.int32, device=dev)
        ops.golay_encode_into(self.trip.view(-1), self.cw, m)
        self.noisy = torch.empty_like(self.cw)
        self.inj_stats = ops.new_stats(dev)
        self.offset0, self.global_n = offset0, global_n
        ops.inject_into(self.cw, self.noisy, BER, 24, seed=SEED, stats=self.inj_stats, global_n=global_n,
                        offset0=offset0)
        self.out_trip = torch.empty(m * 3, dtype=torch.uint8, device=dev)
        self.counts = torch.empty(m, dtype=torch.uint8, device=dev)
        self.stats = ops.new_stats(dev)
        torch.cuda.synchronize()

    def step(self, st=None):
        self.ops.golay_encode_into(self.trip.view(-1), self.cw, self.m)
        self.ops.golay_decode_into(self.noisy, self.out_trip, self.counts, self.stats if st is None else st)


def fused_decode_bench(dev, steps, warmup, packed=False):
    """The shim's fused Golay read (gather -> Golay decode -> dequantize -> fp16,
    ecc_shim.py:990-1071; kvecc_shim_read_batch's wave-tile kernel) over a paged
    cache of B=8 sequences x L=4096 tokens, Hkv=32, D=128, block_size 16, K and
    V, BER 1e-2 codewords.  Algorithmic bytes per token row and side: 43
    codewords (4 B each, 3 B packed) + 4 B scale in, 128 fp16 out."""
    from kvecc import ops
    bs, g = 16, (D + 2) // 3
    nlb = L // bs
    nb = B * nlb
    gen = torch.Generator().manual_seed(7)
    caches, scales = [], []
    for side in range(2):
        x = torch.randint(0, 16, (nb, 1, H, bs, D), generator=gen, dtype=torch.uint8).to(dev)
        cw = ops.golay_encode_rows(x).view(-1)
        ops.inject_into(cw, cw, BER, 24, seed=SEED + side)
        cw = cw.view(nb, 1, H, bs * g)
        if packed:
            cw = torch.stack([(cw >> (8 * k)) & 0xFF for k in range(3)], -1).to(torch.uint8)
            cw = cw.view(nb, 1, H, bs, 3 * g)
            row = (3 * g + 3) // 4 * 4
            pad = torch.zeros(nb, 1, H, bs, row, dtype=torch.uint8, device=dev)
            pad[..., :3 * g] = cw
            cw = pad.view(nb, 1, H, bs * row)
        caches.append(cw.contiguous())
        scales.append((torch.rand(nb, 1, H, bs, generator=gen) * 0.1 + 0.01).to(dev))
        del x
    table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
    codec = "golay_packed" if packed else "golay"
    outs = (torch.empty(B, H, L, D, dtype=torch.float16, device=dev),
            torch.empty(B, H, L, D, dtype=torch.float16, device=dev))
    st = ops.new_stats(dev)

    def call():
        ops.shim_read_batch(caches[0], caches[1], scales[0], scales[1], table, L, D, 0, codec,
                            torch.float16, stats=st, out=outs)

    _warm(call, warmup)
    evs = [ops.kernel_timer(dev) for _ in range(steps)]
    torch.cuda.synchronize()
    for k in range(steps):
        ops.time_next_launch(*evs[k])
        call()
    torch.cuda.synchronize()
    ms = sum(e[0].elapsed_time(e[1]) for e in evs) / steps
    rows = 2 * B * L * H
    bytes_per_row = (3 * g if packed else 4 * g) + 4 + 2 * D
    gbs = rows * bytes_per_row / (ms * 1e-3) / 1e9
    return {"workload": f"shim_read_batch {codec} -> fp16, [B={B},L={L},Hkv={H},D={D}] K+V, "
                        f"block_size {bs}, BER {BER}",
            "kernel": "shim_read_golay_tiles_kernel", "kernel_ms": ms,
            "codewords_per_s": rows * g / (ms * 1e-3),
            "bytes_per_launch": rows * bytes_per_row,
            "bytes_per_token_row": bytes_per_row, "hbm_gbs": gbs, "frac": gbs / HBM_PEAK_GBS,
            "write_share": 2 * D / bytes_per_row,
            "ceiling_note": "moving exactly these bytes (the same tiles through the same block table, the "
                            "row scales, 4 KiB stores per tile) with no decode at all takes 153.6-157.3 us "
                            "(0.73-0.74) in the same process as the kernel's 159.0 "
                            "(profiles/r06/golay_read_direct_probe.txt); 128-byte aligned 2816-byte units with "
                            "no scales ran 147 us (profiles/r03/fused/store_perm.log); every decode structure "
                            "tried lands at 157-162 us (profiles/r06/golay_read_byteclass.txt)",
            "timing": f"HIP events carried by the dispatch, mean of {steps} launches after >= {warmup} warm-up calls and >= 0.25 s"}


def fused_h84_bench(dev, steps, warmup):
    """The shim's fused read for its default codec, Hamming(8,4) (ecc_shim.py:990-1071):
    gather -> SECDED decode (-> double-error interpolation along the context) ->
    dequantize -> fp16 over [B=8, L=4096, Hkv=32, D=128] K+V, block 16, BER 1e-3.
    Bytes per token row and side: 128 codeword bytes + 4 B scale in, 256 B out
    (interpolation's neighbour rows come from the wave's LDS tile, except the
    two halo rows per 16-row tile)."""
    from kvecc import ops
    bs = 16
    nlb = L // bs
    nb = B * nlb
    gen = torch.Generator().manual_seed(11)
    caches, scales = [], []
    for side in range(2):
        x = torch.randint(0, 16, (nb * H * bs * D,), generator=gen, dtype=torch.uint8).to(dev)
        cw = ops.hamming84_encode(x)
        ops.inject_into(cw, cw, 1e-3, 8, seed=SEED + side)
        caches.append(cw.view(nb, 1, H, bs * D))
        scales.append((torch.rand(nb, 1, H, bs, generator=gen) * 0.1 + 0.01).to(dev))
        del x
    table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
    outs = (torch.empty(B, H, L, D, dtype=torch.float16, device=dev),
            torch.empty(B, H, L, D, dtype=torch.float16, device=dev))
    st = ops.new_stats(dev)
    res = {}
    for interp in (False, True):
        def call():
            ops.shim_read_batch(caches[0], caches[1], scales[0], scales[1], table, L, D, 0, "hamming84",
                                torch.float16, stats=st, interp=interp, out=outs)
        _warm(call, warmup)
        evs = [ops.kernel_timer(dev) for _ in range(steps)]
        torch.cuda.synchronize()
        for k in range(steps):
            ops.time_next_launch(*evs[k])
            call()
        torch.cuda.synchronize()
        ms = sum(e[0].elapsed_time(e[1]) for e in evs) / steps
        nbytes = 2 * B * L * H * (D + 4 + 2 * D)
        res["interp" if interp else "plain"] = {
            "kernel_ms": ms, "values_per_s": 2 * B * L * H * D / (ms * 1e-3),
            "bytes_per_launch": nbytes, "hbm_gbs": nbytes / (ms * 1e-3) / 1e9,
            "frac": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    res.update({"workload": "shim_read_batch hamming84 -> fp16, [B=8,L=4096,Hkv=32,D=128] K+V, block_size 16, "
                            "BER 1e-3; plain and with double-error interpolation",
                "kernel": "shim_read_bytes_tiles_kernel", "bytes_per_token_row": D + 4 + 2 * D,
                "timing": f"HIP events carried by the dispatch, mean of {steps} launches after >= {warmup} warm-up calls and >= 0.25 s"})
    return res


def rows_bench(dev, x, noisy_rows, steps, warmup):
    """Per-head Golay rows (the shim's and the config-5 sweep's layout,
    ecc_shim.py:623-682): golay_encode_rows of the [8,4096,32,128] nibbles and
    golay_decode_rows of its BER-1e-2 codewords, kernel time from events carried
    by each dispatch.  Bytes/row: 128 nibble bytes + 43 * 4 codeword bytes."""
    from kvecc import ops
    rows, d = x.numel() // D, D
    cw = torch.empty(rows, (D + 2) // 3, dtype=torch.int32, device=dev)
    nib = torch.empty(rows, D, dtype=torch.uint8, device=dev)
    st = ops.new_stats(dev)
    xr = x.view(rows, D)
    def pair():
        ops.golay_encode_rows_into(xr, cw)
        ops.golay_decode_rows_into(noisy_rows, nib, st)

    _warm(pair, warmup)
    ev = [ops.kernel_timer(dev) + ops.kernel_timer(dev) for _ in range(steps)]
    torch.cuda.synchronize()
    for k in range(steps):
        ops.time_next_launch(ev[k][0], ev[k][1])
        ops.golay_encode_rows_into(xr, cw)
        ops.time_next_launch(ev[k][2], ev[k][3])
        ops.golay_decode_rows_into(noisy_rows, nib, st)
    torch.cuda.synchronize()
    enc = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
    dec = sum(e[2].elapsed_time(e[3]) for e in ev) / steps
    nbytes = rows * (D + 4 * ((D + 2) // 3))
    return {"workload": "golay_encode_rows / golay_decode_rows, [8,4096,32,128] (43 codewords per head row)",
            "kernels": ["golay_encode_rows_full_kernel", "golay_decode_rows_reg_kernel"],
            "kernel_ms": {"encode": enc, "decode": dec}, "bytes_per_launch": nbytes,
            "hbm_gbs": {"encode": nbytes / (enc * 1e-3) / 1e9, "decode": nbytes / (dec * 1e-3) / 1e9},
            "frac": {"encode": nbytes / (enc * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "decode": nbytes / (dec * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "timing": f"HIP events carried by the dispatch, mean of {steps} launches after >= {warmup} warm-up calls and >= 0.25 s"}


def cpu_quota():
    """cgroup v2 CPU quota of this process as 'N cores' (or 'unlimited')."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return "unlimited" if q == "max" else f"{int(q) / int(p):g} cores"
    except (OSError, ValueError):
        return "unknown"


def host_info():
    """CPU model, visible cores and OMP_NUM_THREADS of the host."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")),
                         None)
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "cpu_quota": cpu_quota(),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_backend_baseline(budget_s, threads):
    """The product's host backend (kvecc.cpu_ops, backend="cpu": the kernels'
    codec algebra on std::threads) on the FULL per-GPU workload: Golay encode +
    decode of M = 45,088,768 codewords.  One warm-up pass, then the median of
    the passes that fit in ~budget_s (at least 5) on `threads` threads, and the
    median of 3 passes on 1 thread."""
    import statistics

    from kvecc import cpu_ops
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 16, (B, L, H, D), generator=g, dtype=torch.uint8)
    gsz = (D + 2) // 3
    trip = torch.zeros(B, L, H, gsz * 3, dtype=torch.uint8)
    trip[..., :D] = x
    trip = trip.view(-1, 3)
    del x
    m = trip.shape[0]
    cpu_ops.set_num_threads(threads)
    cw = cpu_ops.golay_encode(trip)
    noisy = cpu_ops.inject_bit_errors_triton(cw, BER, 24, SEED)
    # outputs allocated once, as on the GPU side (fresh tensors per pass would
    # time the kernel's page faults on first touch, not the codec)
    flat = trip.view(-1)
    out_trip = torch.empty(m * 3, dtype=torch.uint8)
    counts = torch.empty(m, dtype=torch.uint8)
    st = cpu_ops.new_stats()

    def one_pass():
        cpu_ops.golay_encode_into(flat, cw, m)
        cpu_ops.golay_decode_into(noisy, out_trip, counts, st)

    def passes(n_threads, min_reps, budget):
        cpu_ops.set_num_threads(n_threads)
        one_pass()  # warm-up
        times, t_start = [], time.perf_counter()
        while len(times) < min_reps or time.perf_counter() - t_start < budget:
            t0 = time.perf_counter()
            one_pass()
            times.append(time.perf_counter() - t0)
        return statistics.median(times), len(times)

    med, reps = passes(threads, 5, budget_s)
    med1, reps1 = passes(1, 3, 0.0)
    cpu_ops.set_num_threads(threads)
    return {"value": m / med, "unit": "codewords/s", "cores": threads, "kind": "host-backend",
            "one_thread": {"value": m / med1, "passes": reps1},
            "host": host_info(),
            "sample": f"median of {reps} passes of full [8,4096,32,128] Golay encode+decode "
                      f"({m} codewords, BER 1e-2) after a warm-up, kvecc.cpu_ops on {threads} "
                      f"host threads; one_thread: median of {reps1} passes on 1 thread"}


def main(argv=None):
    args = parse(argv)
    # --gpus N > 1 without a launcher: start the N ranks as child processes
    # (before anything here touches the GPU) and exit with their status
    from kvecc import launch
    if args.gpus is None:  # under torchrun: the launcher's world
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    rc = launch.launch_if_needed(os.path.abspath(__file__), sys.argv[1:] if argv is None else list(argv),
                                 args.gpus, args.backend)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:  # only an explicit --gpus can disagree
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.scaling == "strong" and world > B:
        print(f"bench: --scaling strong splits B={B}: at most {B} ranks, got {world}", file=sys.stderr)
        sys.exit(2)
    gloo = args.backend == "gloo"
    # one GPU per rank; --backend gloo lets several ranks share one device to
    # rehearse the multi-rank path on a 1-GPU box (RCCL refuses that)
    ngpu = torch.cuda.device_count()
    local_dev = local % ngpu if args.backend == "gloo" and ngpu else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    dist = None
    if world > 1 or args.dist:
        import torch.distributed as dist
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        launch.check_world(dist, args.gpus)

    import kvecc
    from kvecc import ops
    kvecc.require_hip()

    # ---- synthetic INT4 KV tensor, resident in HBM ---------------------------
    gsz = (D + 2) // 3                      # 43 codewords per head vector
    if args.scaling == "weak":
        # every rank owns a whole [8,4096,32,128] tensor (seed = rank), codeword
        # offset rank*M of the concatenation
        gen = torch.Generator().manual_seed(rank)
        x = torch.randint(0, 16, (B, L, H, D), generator=gen, dtype=torch.uint8).to(dev)
        m1 = B * L * H * gsz
        hl = Headline(dev, x, rank * m1, m1 * world)
    else:
        x, off, gn = strong_setup(dev, rank, world)
        hl = Headline(dev, x, off, gn)
    del x
    trip, cw, noisy, out_trip, counts = hl.trip, hl.cw, hl.noisy, hl.out_trip, hl.counts
    m, inj_stats, stats = hl.m, hl.inj_stats, hl.stats
    total_m = hl.global_n  # codewords one step processes over all ranks

    kernel_timing = args.timing == "kernel"

    def step(ev=None, st=stats):
        if ev is not None and kernel_timing:
            ops.time_next_launch(ev[0], ev[1])
        elif ev is not None:
            ev[0].record()
        ops.golay_encode_into(trip.view(-1), cw, m)
        if ev is not None and kernel_timing:
            ops.time_next_launch(ev[2], ev[3])
        elif ev is not None:
            ev[1].record()
        ops.golay_decode_into(noisy, out_trip, counts, st)
        if ev is not None and not kernel_timing:
            ev[2].record()

    for _ in range(args.warmup):
        step()
    stats.zero_()
    if kernel_timing:  # (enc start, enc end, dec start, dec end) per step, handles created
        events = [ops.kernel_timer(dev) + ops.kernel_timer(dev) for _ in range(args.steps)]
    else:
        events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
                  for _ in range(args.steps)]
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # steps every-1, 2*every-1, ... (not step 0, right behind the sync): a
    # timed dispatch also costs the step ~8 us (kernel) or ~4 us (markers)
    sampled = list(range(args.event_every - 1, args.steps, args.event_every)) or [args.steps - 1]
    for k in range(args.steps):
        step(events[k] if k in sampled else None)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()

    elapsed = t1 - t0
    timed = [events[k] for k in sampled]
    if kernel_timing and args.roofline_samples > 0:
        # more kernel-carried samples for the roofline, after the timed region
        # (the throughput above is untouched; statistics go to a scratch buffer)
        scratch = ops.new_stats(dev)
        extra = [ops.kernel_timer(dev) + ops.kernel_timer(dev) for _ in range(args.roofline_samples)]
        for ev in extra:
            step(ev, scratch)
        torch.cuda.synchronize()
        timed = timed + extra
    if kernel_timing:
        enc_ms = sum(e[0].elapsed_time(e[1]) for e in timed) / len(timed)
        dec_ms = sum(e[2].elapsed_time(e[3]) for e in timed) / len(timed)
    else:
        enc_ms = sum(e[0].elapsed_time(e[1]) for e in timed) / len(timed)
        dec_ms = sum(e[1].elapsed_time(e[2]) for e in timed) / len(timed)
    tt = torch.tensor([elapsed, enc_ms, dec_ms], dtype=torch.float64, device=dev)
    st = ops.stats_totals(stats)
    per_rank = [tt.tolist() + [m]]
    world_info = {"backend": None, "world_size": 1}
    if dist is not None:
        per_rank = gather_floats(dist, world, dev, tt.tolist() + [m], gloo)  # per-rank times, reported
        if gloo:  # gloo reduces host tensors
            tt, st = tt.cpu(), st.cpu()
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.all_reduce(st, op=dist.ReduceOp.SUM)     # the single stats all-reduce
        world_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    elapsed, enc_ms, dec_ms = tt.tolist()
    bits, unc = st.tolist()

    # ---- correctness spot check (outside timing) -----------------------------
    ref_trip, ref_stats = None, None
    if rank == 0:
        chk = ops.new_stats(dev)
        ops.golay_decode_into(cw, out_trip, counts, chk)  # clean codewords round-trip
        torch.cuda.synchronize()
        assert torch.equal(out_trip.view(-1, 3), trip), "encode->decode round trip failed"
        assert ops.read_stats(chk) == [0, 0]

    # ---- optional sections: each runs on rank 0 only, after the timed region;
    # a failure (e.g. out of memory) records {"error": ...} under its key and
    # the headline line still prints; each frees its tensors before the next
    def optional(name, fn):
        if rank != 0:
            return None
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            print(f"bench: section {name} failed: {e!r}", file=sys.stderr)
            return {"error": repr(e)[:500]}
        finally:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    # ---- collective sections: every rank runs them, together, before the
    # rank-0-only sections.  One rank: a failure is recorded like an optional
    # section's.  Several ranks: a failure raises (a rank that skipped a
    # collective would leave the others waiting), and the launcher stops them.
    def collective(name, fn):
        if dist is None:
            return optional(name, fn)
        try:
            return fn()
        finally:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    # strong scaling beside the weak headline (with --scaling strong the
    # headline itself is the strong figure)
    strong = None if args.no_strong or args.scaling == "strong" or world > B else collective(
        "strong", lambda: strong_section(dev, dist, rank, world, args.steps, args.warmup, gloo))
    # BASELINE config 5, batch-sharded over the ranks with one all-reduce
    montecarlo = None if args.no_montecarlo else collective(
        "montecarlo", lambda: montecarlo_bench(dev, dist, rank, world, gloo))

    # ---- injection throughput (VALU-bound, Philox4x32-10 per bit) ------------
    def inject_section():
        scratch = ops.new_stats(dev)
        inj_ms = kernel_ms(dev, lambda: ops.inject_into(cw, noisy, BER, 24, seed=SEED, stats=scratch,
                                                        global_n=total_m, offset0=hl.offset0), 10, 3)
        philox = m * 24  # one Philox4x32-10 per bit (fault_injection_triton.py:303-334)
        res = {"kernel": "inject_kernel<int32, 24> (with stats)", "ms": inj_ms,
               "codewords_per_s": m / (inj_ms * 1e-3), "philox_per_s": philox / (inj_ms * 1e-3),
               "flips": ops.read_stats(inj_stats)[0], "bound": "valu",
               "timing": "HIP events carried by the dispatch, mean of 10 launches after >= 3 warm-up calls"}
        # VALU roofline: wave-level VALU instructions per Philox from the committed
        # counter pass (rocprofv3 cannot run inside this process) x the live
        # Philox rate.  Peak = the VALU issue slots of 256 CUs x 4 SIMDs at the
        # 2.4 GHz spec clock, one wave64 instruction per quad-cycle per SIMD, the
        # pairs the SIMD dual-issues (SQ_ACTIVE_INST_VALU2: 5 % of this kernel's
        # instructions) sharing a slot (profiles/inject_valu.json,
        # tools/inject_summary.py).  The nominal 2-cycle rate -- every instruction
        # paired -- is reported beside it, and valu_busy_pmc is the counters' own
        # busy fraction: issue slots used / slots the launch had at its clock.
        nominal = 256 * 4 * 2.4e9 / 2
        if os.path.exists(args.inject_pmc_json):
            with open(args.inject_pmc_json) as f:
                pmc = json.load(f)
            ipp = pmc["valu_insts_per_philox"]  # lane-instructions per Philox (SQ_INSTS_VALU x 64 / Philox)
            achieved = philox / (inj_ms * 1e-3) * ipp / 64  # wave-instructions per second
            peak = pmc.get("issue_peak_wave_instr_per_s", nominal)
            res["roofline"] = {"bound": "valu", "achieved": achieved, "peak": peak,
                               "unit": "wave VALU instructions/s", "frac": achieved / peak,
                               "peak_basis": pmc.get("peak_basis"),
                               "dual_issue_frac": pmc.get("dual_issue_frac"),
                               "nominal_peak": nominal, "frac_of_nominal": achieved / nominal,
                               "valu_insts_per_philox": ipp, "valu_busy_pmc": pmc.get("valu_busy"),
                               "source": pmc.get("source")}
        return res

    inject = None if args.no_inject else optional("inject", inject_section)

    # ---- the Monte-Carlo pipeline: encode -> inject (BER 1e-2) -> decode per
    # step, what a config-5 trial does; injection (VALU-bound) dominates it
    def pipeline_section():
        scratch = ops.new_stats(dev)
        noisy2 = torch.empty_like(cw)

        def one():
            ops.golay_encode_into(trip.view(-1), cw, m)
            ops.inject_into(cw, noisy2, BER, 24, seed=SEED, global_n=total_m, offset0=hl.offset0)
            ops.golay_decode_into(noisy2, out_trip, counts, scratch)

        for _ in range(2):
            one()
        reps = 5
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            one()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        return {"workload": "golay_encode + inject_bit_errors(BER 1e-2, 24 bits, Philox per bit) + "
                            "golay_decode of the headline's codewords, back to back",
                "ms": ms, "codewords_per_s": m / (ms * 1e-3),
                "note": "the headline value excludes injection (done once, before timing); this is the "
                        "rate a Monte-Carlo trial sees"}

    pipeline = None if args.no_pipeline else optional("end_to_end_pipeline", pipeline_section)

    # ---- native packed layout (3-byte codewords, nibbles two per byte) -------
    # Same codewords, its own bytes/unit (4.5 B encode, 4.625 B decode); never
    # mixed into `value`, which is the reference layout.
    side_warmup = max(args.warmup, args.side_warmup)  # optional sections only; the step keeps W

    def packed_section():
        nib = ops.pack_nibbles(trip.view(-1))
        cw3 = ops.golay_encode_packed(nib, m)
        noisy3 = torch.stack([(noisy >> (8 * k)) & 0xFF for k in range(3)], 1).to(torch.uint8)
        noisy3 = noisy3.reshape(-1).contiguous()
        nib_out = torch.empty_like(nib)
        flags = torch.empty((m + 7) // 8, dtype=torch.uint8, device=dev)  # uncorrectable bits
        pst = ops.new_stats(dev)
        steps = max(args.steps, 10)
        # HIP events carried by each kernel's own dispatch (as the other sections);
        # event markers between the launches read 2-4 us high
        pe = [ops.kernel_timer(dev) + ops.kernel_timer(dev) for _ in range(steps)]
        def pair():
            ops.golay_encode_packed_into(nib, cw3, m)
            ops.golay_decode_packed_into(noisy3, nib_out, flags, m, pst)

        _warm(pair, side_warmup)
        torch.cuda.synchronize()
        for k in range(steps):
            ops.time_next_launch(pe[k][0], pe[k][1])
            ops.golay_encode_packed_into(nib, cw3, m)
            ops.time_next_launch(pe[k][2], pe[k][3])
            ops.golay_decode_packed_into(noisy3, nib_out, flags, m, pst)
        torch.cuda.synchronize()
        p_enc = sum(e[0].elapsed_time(e[1]) for e in pe) / steps
        p_dec = sum(e[2].elapsed_time(e[3]) for e in pe) / steps
        return {"layout": "3-byte codewords, INT4 nibbles two per byte (native, not the reference's)",
                "timing": f"HIP events carried by the dispatches, mean of {steps} launches each after "
                          f">= {side_warmup} warm-up pairs and >= 0.25 s",
                "codewords_per_s": m / ((p_enc + p_dec) * 1e-3),
                "kernel_ms": {"encode": p_enc, "decode": p_dec},
                "bytes_per_codeword": {"encode": 4.5, "decode": 4.625},
                "hbm_gbs": {"encode": 4.5 * m / (p_enc * 1e-3) / 1e9,
                            "decode": 4.625 * m / (p_dec * 1e-3) / 1e9}}

    packed = None if args.no_packed else optional("packed", packed_section)

    def rows_section():
        xr = torch.randint(0, 16, (B, L, H, D), generator=torch.Generator().manual_seed(rank),
                           dtype=torch.uint8).to(dev)
        noisy_rows = noisy.view(B * L * H, gsz)  # the same BER-1e-2 codewords, one row per head
        return rows_bench(dev, xr, noisy_rows, max(args.steps, 10), side_warmup)

    rows = None if args.no_rows else optional("golay_rows", rows_section)
    interp = None if args.no_interp else optional(
        "interp", lambda: interp_bench(dev, max(args.steps, 10), side_warmup))
    quant = None if args.no_quant else optional(
        "fused_quant", lambda: quant_bench(dev, max(args.steps, 10), side_warmup))

    fused = None
    if not args.no_fused:
        fused = optional("fused_golay_decode", lambda: fused_decode_bench(dev, max(args.steps, 10), side_warmup))
        if fused is not None:
            fused["packed"] = optional("fused_golay_decode.packed",
                                       lambda: fused_decode_bench(dev, max(args.steps, 10), side_warmup,
                                                                  packed=True))
            fused["hamming84"] = optional("fused_golay_decode.hamming84",
                                          lambda: fused_h84_bench(dev, max(args.steps, 10), side_warmup))

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    total_cw = total_m * args.steps  # every rank's codewords over the slowest rank's time
    value = total_cw / elapsed
    if args.scaling == "strong":  # shards differ in size: rank 0's own kernels and codewords
        enc_ms, dec_ms = per_rank[0][1], per_rank[0][2]
    dec_gbs = DECODE_BYTES_PER_CW * m / (dec_ms * 1e-3) / 1e9
    enc_gbs = ENCODE_BYTES_PER_CW * m / (enc_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            traffic = json.load(f).get("golay_decode_bytes_per_launch")
    cpu = host = None
    if world == 1 and not args.no_cpu_baseline:
        def cpu_section():
            c = cpu_baseline(args.cpu_seconds, args.cpu_threads)
            all_cores = os.cpu_count() or 1
            c["all_cores"] = cpu_baseline(min(args.cpu_seconds, 6.0), all_cores)
            c["all_cores"]["note"] = (f"{all_cores} threads = os.cpu_count(); the process's CPU "
                                      f"quota is {cpu_quota()} (cgroup cpu.max), so threads beyond "
                                      f"it time-share")
            return c

        cpu = optional("cpu_baseline", cpu_section)
        host = optional("cpu_backend", lambda: cpu_backend_baseline(min(args.cpu_seconds, 5.0),
                                                                     args.cpu_threads))
    line = {
        "metric": "INT4 codewords/sec encode+decode (Golay24, L=4096) + achieved HBM GB/s",
        "value": value,
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u8/int32 (bitwise)",
        "data": ("synthetic: torch.randint(0,16) INT4 nibbles, seed=rank; BER 1e-2 Philox corruption"
                 if args.scaling == "weak" else
                 "synthetic: ONE torch.randint(0,16) [8,4096,32,128] tensor (seed 0) split along B; "
                 "BER 1e-2 Philox corruption"),
        "config": {"workload": ("golay24 per-head encode+decode, [B=8,L=4096,H=32,D=128] per GPU"
                                if args.scaling == "weak" else
                                "golay24 per-head encode+decode, ONE [B=8,L=4096,H=32,D=128] split along B"),
                   "codewords_per_gpu": m, "codewords_per_step": total_m, "ber": BER, "seed": SEED,
                   "parallelism": f"dp{world}",
                   "global_batch": B * world if args.scaling == "weak" else B, "seq_len": L,
                   "process_group": world_info,
                   "launcher": ("self (bench.py spawned its ranks)" if os.environ.get(launch.ENV_LAUNCHED) == "1"
                                else "external (torchrun)" if world > 1 else "single process"),
                   "per_rank": [{"rank": r, "elapsed_s": v[0], "encode_ms": v[1], "decode_ms": v[2],
                                 "codewords": int(v[3]), "codewords_per_s": v[3] * args.steps / v[0]}
                                for r, v in enumerate(per_rank)]},
        "hbm_gbs": {"decode": dec_gbs, "encode": enc_gbs,
                    "round_trip": (DECODE_BYTES_PER_CW + ENCODE_BYTES_PER_CW) * m
                    / ((enc_ms + dec_ms) * 1e-3) / 1e9},
        "kernel_ms": {"encode": enc_ms, "decode": dec_ms},
        "roofline": {"bound": "hbm", "achieved": dec_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": dec_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "golay_decode_kernel", "bytes_per_launch": DECODE_BYTES_PER_CW * m,
                     "timing": (f"HIP events carried by the kernel dispatches (hipExtLaunchKernel) "
                                f"of every {args.event_every}th timed step and of "
                                f"{args.roofline_samples} steps after the timed region "
                                f"({len(timed)} samples)" if kernel_timing else
                                f"hipEventRecord markers on every {args.event_every}th timed step")},
        "decode_stats": {"bits_corrected": bits, "uncorrectable": unc, "steps": args.steps},
        "inject": inject,
        "end_to_end_pipeline_cw_per_s": pipeline["codewords_per_s"] if pipeline and "codewords_per_s" in pipeline
        else None,
        "end_to_end_pipeline": pipeline,
        "fused_golay_decode": fused,
        "golay_rows": rows,
        "interp": interp,
        "fused_quant": quant,
        "strong_scaling": strong,
        "montecarlo": montecarlo,
        "packed": packed,
        "cpu_baseline": cpu,
        "cpu_backend": host,
    }
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
