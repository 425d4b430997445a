"""Batch-sharded Monte-Carlo fault-injection sweep (BASELINE config 5).

Counterpart of the reference's sweep drivers (evaluation/sweep.py:352-626,
evaluation/experiments/monte_carlo.py:75-395 and the flat-injection Monte
Carlo of evaluation/experiments/quantization_ecc_comparison.py:72-247), cut
down to the codec path: for every (codec, BER, seed) trial, a synthetic INT4
KV tensor [B, L, H, D] is encoded, corrupted with the reference's Philox bit
flips, decoded (and interpolated for "hamming84_interp"), and five counters
are kept: [flips, elements affected, corrected, detected/uncorrectable,
residual nibble mismatches vs the ground truth].

MI355X layout: one process per GPU; rank r owns batch rows [b0, b1).  The
fault pattern of a shard is the one the unsharded run would draw, because the
flat injection is told the global element count and the shard's global
offset; the ground truth itself is drawn from the same Philox stream
(BER 0.5 over 4 bits of a zero tensor = uniform nibbles), so it is identical
for any shard decomposition and reproducible by the test oracle.  Counters
stay on the device for the whole sweep; the only collective is ONE
all_reduce(SUM) of the [trials, 5] int64 table at the end (RCCL over xGMI on
MI355X, gloo in the CPU tests).  Finished trials are appended to a JSONL file,
so an interrupted sweep resumes where it stopped.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from dataclasses import dataclass, field

import torch

STAT_NAMES = ("flips", "affected", "corrected", "detected", "mismatches")
CODECS = ("hamming74", "hamming84", "hamming84_interp", "golay")
N_BITS = {"hamming74": 7, "hamming84": 8, "hamming84_interp": 8, "golay": 24}


@dataclass
class MonteCarloConfig:
    shape: tuple = (8, 4096, 32, 128)  # [B, L, H, D]
    codecs: tuple = CODECS
    bers: tuple = (1e-4, 1e-3, 1e-2)
    seeds: tuple = (42, 101, 997)
    data_seed: int = 0
    output: str | None = None  # JSONL of finished trials (resume)
    meta: dict = field(default_factory=dict)

    def trials(self):
        return [(c, float(b), int(s)) for c in self.codecs for b in self.bers for s in self.seeds]


def trial_key(codec, ber, seed):
    return f"{codec}|{ber:.6g}|{seed}"


def injected_elements(codec, shape):
    """Elements the trial's flat injection draws over (its global N): INT4
    values for the Hamming codecs, per-head-padded codewords for Golay."""
    b, l, h, d = shape
    return b * l * h * ((d + 2) // 3 if codec == "golay" else d)


def stream_key(codec, seed, shape):
    """The 32-bit Philox key base of a trial's flips.  Element `off`, bit `b`
    draws under int32(seed*N*n_bits + off*n_bits + b) (fault_injection_triton.py
    :247-294), so two seeds whose seed*N*n_bits agree mod 2^32
    draw the SAME flips: with N = 2^27 and 8 bits, seeds 101 and 997 collide
    ((997-101)*2^30 = 224*2^32)."""
    return (seed * injected_elements(codec, shape) * N_BITS[codec]) & 0xFFFFFFFF


def seed_aliases(cfg: MonteCarloConfig):
    """{trial key: key of the first trial it duplicates}: same codec and BER, and
    a seed whose Philox key base collides (stream_key).  Such trials reproduce
    the reference's bits exactly and are NOT independent samples."""
    first, alias = {}, {}
    for codec, ber, seed in cfg.trials():
        k = (codec, ber, stream_key(codec, seed, cfg.shape), cfg.data_seed)
        key = trial_key(codec, ber, seed)
        if k in first:
            alias[key] = first[k]
        else:
            first[k] = key
    return alias


def shard_bounds(batch, rank, world):
    """Contiguous split of the batch axis; the first batch % world ranks get one more row."""
    base, extra = divmod(batch, world)
    b0 = rank * base + min(rank, extra)
    return b0, b0 + base + (1 if rank < extra else 0)


class _TrialBuffers:
    """One trial's device buffers (HipShard keeps two, for the stream pipeline)."""

    def __init__(self, ops, shape, g, dev):
        sb, l, h, d = shape
        self.cw8 = torch.empty(shape, dtype=torch.uint8, device=dev)
        self.cw32 = torch.empty((sb, l, h, g), dtype=torch.int32, device=dev)
        self.dec = torch.empty(shape, dtype=torch.uint8, device=dev)
        self.et = torch.empty(shape, dtype=torch.uint8, device=dev)
        self.itp = torch.empty(shape, dtype=torch.uint8, device=dev)
        self.st_inj = ops.new_stats(dev)
        self.st_dec = ops.new_stats(dev)
        self.st_cmp = ops.new_stats(dev)  # residual mismatches (kvecc_count_ne_u8)
        self.ready = torch.cuda.Event()   # encode + inject done
        self.free = torch.cuda.Event()    # decode + count done: the buffers may be rewritten
        self.free.record()


class HipShard:
    """One rank's shard of the sweep on an MI355X (kvecc HIP kernels).

    fused=True (default): a trial is ONE launch, kvecc_mc_trial, which encodes,
    flips, decodes (and interpolates) in registers and keeps only the five
    counters -- the trial is VALU-bound on its Philox draws and touches HBM
    only to read the ground truth.  Every trial gets its own statistics buffer;
    finish() folds them all into the sweep's table in one launch
    (kvecc_stats_fold).

    fused=False: the kernel-by-kernel pipeline (encode, inject, decode,
    interpolate, count as separate launches), pipelined over two HIP streams:
    trial k's encode + injection runs on one stream while trial k-1's decode,
    interpolation and residual count run on the other, in two alternating
    buffer sets ordered by events.  Kept as the check of the fused trial
    (same counters) and for A/B timing.  finish() drains the pipeline."""

    def __init__(self, cfg: MonteCarloConfig, rank: int, world: int, device, fused: bool = True):
        from . import ops
        self.ops = ops
        self.cfg = cfg
        self.fused = fused
        self.dev = torch.device(device)
        b, l, h, d = cfg.shape
        self.b0, self.b1 = shard_bounds(b, rank, world)
        self.sb = self.b1 - self.b0
        per_b = l * h * d
        self.n_total = b * per_b
        self.off = self.b0 * per_b
        self.g = (d + 2) // 3
        self.m_total = b * l * h * self.g
        self.m_off = self.b0 * l * h * self.g
        shape = (self.sb, l, h, d)
        # ground truth: uniform nibbles from the Philox stream, shard-consistent
        self.x = torch.zeros(shape, dtype=torch.uint8, device=self.dev)
        if self.sb:
            ops.inject_into(self.x.view(-1), self.x.view(-1), 0.5, 4, cfg.data_seed,
                            global_n=self.n_total, offset0=self.off)
        self.k = 0
        self.pending = None
        self._stat_chunks, self._queued = [], []  # fused: statistics buffers, (buffer, row) per trial
        # the fused interpolating trial reads 4-value column chunks: at a
        # geometry with heads*head_dim % 4 != 0 that one codec runs the
        # kernel-by-kernel pipeline, every other codec stays fused
        self._interp_unfused = fused and (h * d) % 4 != 0
        self.bufs = None
        if fused and not self._interp_unfused:
            return
        with torch.cuda.device(self.dev):
            self.bufs = [_TrialBuffers(ops, shape, self.g, self.dev) for _ in range(2)]
            self.s_inj = torch.cuda.Stream(self.dev)
            self.s_dec = torch.cuda.Stream(self.dev)

    _CHUNK = 64  # statistics buffers allocated at once (fused)

    def _stats_buffer(self):
        i = len(self._queued)
        if i // self._CHUNK >= len(self._stat_chunks):
            self._stat_chunks.append(torch.zeros(self._CHUNK, self.ops.STATS_SLOTS * self.ops.STATS_STRIDE,
                                                 dtype=torch.int64, device=self.dev))
        return self._stat_chunks[i // self._CHUNK][i % self._CHUNK]

    def run_trial(self, codec, ber, seed, row):
        """Queue one trial; its 5 counters land in `row` (device int64[5]) once
        the shard has run it (finish(), or the next trial for fused=False)."""
        ops = self.ops
        if self.sb == 0:
            return row
        if self.uses_fused(codec):
            st = self._stats_buffer()
            golay = codec == "golay"
            ops.mc_trial_into(self.x, codec, ber, seed, self.m_total if golay else self.n_total,
                              self.m_off if golay else self.off, st)
            self._queued.append(row)
            return row
        caller = torch.cuda.current_stream(self.dev)
        buf = self.bufs[self.k % 2]
        self.k += 1
        x = self.x.view(-1)
        with torch.cuda.stream(self.s_inj):
            self.s_inj.wait_stream(caller)
            self.s_inj.wait_event(buf.free)
            buf.st_inj.zero_()
            if codec == "golay":
                ops.golay_encode_rows_into(self.x, buf.cw32)
                flat = buf.cw32.view(-1)
                ops.inject_into(flat, flat, ber, 24, seed, stats=buf.st_inj, global_n=self.m_total,
                                offset0=self.m_off)
            else:
                enc = ops.hamming74_encode_into if codec == "hamming74" else ops.hamming84_encode_into
                c = buf.cw8.view(-1)
                enc(x, c)
                ops.inject_into(c, c, ber, N_BITS[codec], seed, stats=buf.st_inj,
                                global_n=self.n_total, offset0=self.off)
            buf.ready.record(self.s_inj)
        self._drain()
        self.pending = (codec, buf, row, caller)
        return row

    def _drain(self):
        """Decode, interpolate and count the pending trial on the decode stream."""
        if self.pending is None:
            return
        ops = self.ops
        codec, buf, row, caller = self.pending
        self.pending = None
        x = self.x.view(-1)
        with torch.cuda.stream(self.s_dec):
            self.s_dec.wait_stream(caller)  # the caller's row buffer exists
            self.s_dec.wait_event(buf.ready)
            buf.st_dec.zero_()
            buf.st_cmp.zero_()
            if codec == "golay":
                ops.golay_decode_rows_into(buf.cw32, buf.dec, buf.st_dec)
                out = buf.dec
            elif codec == "hamming74":
                ops.hamming74_decode_into(buf.cw8.view(-1), buf.dec.view(-1), None, buf.st_dec)
                out = buf.dec
            else:
                ops.hamming84_decode_into(buf.cw8.view(-1), buf.dec.view(-1), buf.et.view(-1), buf.st_dec)
                out = buf.dec
                if codec == "hamming84_interp":
                    _, l, h, d = self.cfg.shape
                    # temporal neighbours along L, each (b, h, d) column a sequence
                    ops.interpolate_into(buf.dec.view(-1), buf.et.view(-1), buf.itp.view(-1),
                                         self.sb, l, h * d)
                    out = buf.itp
            ops.count_ne_into(out.view(-1), x, buf.st_cmp)  # one pass, no bool tensor
            row[0:2] += ops.stats_totals(buf.st_inj, 2)
            row[2:4] += ops.stats_totals(buf.st_dec, 2)
            row[4:5] += ops.stats_totals(buf.st_cmp, 1)
            buf.free.record(self.s_dec)

    def uses_fused(self, codec):
        """True when `codec`'s trials run as one kvecc_mc_trial launch."""
        return self.fused and not (codec == "hamming84_interp" and self._interp_unfused)

    def finish(self):
        """Fold the fused trials' statistics into their rows and drain the
        pipeline; the caller's stream then holds every queued trial's counters."""
        if self.fused:
            self._fold()
        if self.bufs is None:
            return
        self._drain()
        caller = torch.cuda.current_stream(self.dev)
        caller.wait_stream(self.s_inj)
        caller.wait_stream(self.s_dec)

    def _fold(self):
        rows, self._queued = self._queued, []
        for c, chunk in enumerate(self._stat_chunks):
            part = rows[c * self._CHUNK:(c + 1) * self._CHUNK]
            if not part:
                break
            r0 = part[0]
            step = r0.element_size() * len(STAT_NAMES)
            if all(r.data_ptr() == r0.data_ptr() + k * step and r.is_contiguous() for k, r in enumerate(part)):
                # consecutive rows of one table (run_sweep's): one launch for the chunk
                dst = torch.as_strided(r0, (len(part), len(STAT_NAMES)), (len(STAT_NAMES), 1))
                self.ops.stats_fold_into(chunk, len(part), len(STAT_NAMES), dst)
            else:
                for k, r in enumerate(part):
                    self.ops.stats_fold_into(chunk[k], 1, len(STAT_NAMES), r.view(1, -1))


class HostShard:
    """The same shard on the host backend (kvecc.cpu_ops, C++ threads): the
    sweep's CPU counterpart (BASELINE config 1's backend="cpu") and the check of
    HipShard at the config's own shape.  Every step is the HIP shard's with the
    host twin of its kernel, in the same order; counters land in a host int64
    row.  Hamming(8,4) trials with and without interpolation share their
    (seed, BER) injection, which is cached for the next trial."""

    def __init__(self, cfg: MonteCarloConfig, rank: int, world: int, threads: int | None = None):
        from . import cpu_ops
        self.ops = cpu_ops
        self.cfg = cfg
        self.dev = torch.device("cpu")
        self.threads = threads
        b, l, h, d = cfg.shape
        self.b0, self.b1 = shard_bounds(b, rank, world)
        self.sb = self.b1 - self.b0
        per_b = l * h * d
        self.n_total, self.off = b * per_b, self.b0 * per_b
        self.g = (d + 2) // 3
        self.m_total, self.m_off = b * l * h * self.g, self.b0 * l * h * self.g
        shape = (self.sb, l, h, d)
        self.x = torch.zeros(shape, dtype=torch.uint8)
        if self.sb:
            cpu_ops.inject_into(self.x.view(-1), self.x.view(-1), 0.5, 4, cfg.data_seed,
                                global_n=self.n_total, offset0=self.off, threads=threads)
        self.cw8 = torch.empty(shape, dtype=torch.uint8)
        self.cw32 = torch.empty((self.sb, l, h, self.g), dtype=torch.int32)
        self.dec = torch.empty(shape, dtype=torch.uint8)
        self.et = torch.empty(shape, dtype=torch.uint8)
        self.itp = torch.empty(shape, dtype=torch.uint8)
        self._h84 = None  # (ber, seed, injection stats) of the codewords in cw8

    def run_trial(self, codec, ber, seed, row):
        ops = self.ops
        if self.sb == 0:
            return row
        x = self.x.view(-1)
        st_inj, st_dec, st_cmp = ops.new_stats(), ops.new_stats(), ops.new_stats()
        if codec == "golay":
            ops.golay_encode_rows_into(self.x, self.cw32)
            flat = self.cw32.view(-1)
            ops.inject_into(flat, flat, ber, 24, seed, stats=st_inj, global_n=self.m_total,
                            offset0=self.m_off, threads=self.threads)
            self._h84 = None
            ops.golay_decode_rows_into(self.cw32, self.dec, st_dec)
            out = self.dec
        else:
            c = self.cw8.view(-1)
            h84 = codec in ("hamming84", "hamming84_interp")
            if h84 and self._h84 is not None and self._h84[:2] == (ber, seed):
                st_inj.copy_(self._h84[2])
            else:
                (ops.hamming74_encode_into if codec == "hamming74" else ops.hamming84_encode_into)(x, c)
                ops.inject_into(c, c, ber, N_BITS[codec], seed, stats=st_inj, global_n=self.n_total,
                                offset0=self.off, threads=self.threads)
                self._h84 = (ber, seed, st_inj.clone()) if h84 else None
            if codec == "hamming74":
                ops.hamming74_decode_into(c, self.dec.view(-1), None, st_dec)
                out = self.dec
            else:
                ops.hamming84_decode_into(c, self.dec.view(-1), self.et.view(-1), st_dec)
                out = self.dec
                if codec == "hamming84_interp":
                    _, l, h, d = self.cfg.shape
                    ops.interpolate_into(self.dec.view(-1), self.et.view(-1), self.itp.view(-1), self.sb, l, h * d)
                    out = self.itp
        ops.count_ne_into(out.view(-1), x, st_cmp)
        row[0:2] += ops.stats_totals(st_inj, 2).to(row.device)
        row[2:4] += ops.stats_totals(st_dec, 2).to(row.device)
        row[4:5] += ops.stats_totals(st_cmp, 1).to(row.device)
        return row


def _load_done(path):
    done = {}
    if path and os.path.exists(path):
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line:
                    r = json.loads(line)
                    done[r["key"]] = r
    return done


def run_sweep(cfg: MonteCarloConfig, shard, dist=None, rank=0):
    """Run every unfinished trial on `shard`, reduce once, return the result rows.

    `shard` provides run_trial(codec, ber, seed, row) and a `.dev` device.
    """
    done = _load_done(cfg.output) if rank == 0 else {}
    if dist is not None:
        obj = [sorted(done)]
        dist.broadcast_object_list(obj, src=0)
        done_keys = set(obj[0])
    else:
        done_keys = set(done)
    todo = [t for t in cfg.trials() if trial_key(*t) not in done_keys]
    table = torch.zeros((max(len(todo), 1), len(STAT_NAMES)), dtype=torch.int64, device=shard.dev)
    t0 = time.perf_counter()
    for i, (codec, ber, seed) in enumerate(todo):
        shard.run_trial(codec, ber, seed, table[i])
    if hasattr(shard, "finish"):  # pipelined shards
        shard.finish()
    if shard.dev.type == "cuda":
        torch.cuda.synchronize(shard.dev)
    elapsed = time.perf_counter() - t0
    if dist is not None:  # the sweep's single collective
        if table.is_cuda and dist.get_backend() == "gloo":
            host = table.cpu()  # gloo reduces host tensors; RCCL reduces in HBM
            dist.all_reduce(host, op=dist.ReduceOp.SUM)
            table.copy_(host)
        else:
            dist.all_reduce(table, op=dist.ReduceOp.SUM)
    rows = []
    vals = table.cpu().tolist()
    aliases = seed_aliases(cfg)
    b, l, h, d = cfg.shape
    for i, (codec, ber, seed) in enumerate(todo):
        r = {"key": trial_key(codec, ber, seed), "codec": codec, "ber": ber, "seed": seed,
             "shape": list(cfg.shape), "values": b * l * h * d,
             **{k: int(v) for k, v in zip(STAT_NAMES, vals[i])}}
        if r["key"] in aliases:
            r["alias_of"] = aliases[r["key"]]
        rows.append(r)
    if rank == 0 and cfg.output and rows:
        with open(cfg.output, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    all_rows = [done[k] for k in sorted(done)] + rows
    return all_rows, elapsed


def main(argv=None):
    ap = argparse.ArgumentParser(description="Sharded Monte-Carlo ECC sweep (torchrun-able)")
    ap.add_argument("--shape", type=int, nargs=4, default=[8, 4096, 32, 128])
    ap.add_argument("--codecs", nargs="*", default=list(CODECS))
    ap.add_argument("--bers", type=float, nargs="*", default=[1e-4, 1e-3, 1e-2])
    ap.add_argument("--seeds", type=int, nargs="*", default=[42, 101, 997])
    ap.add_argument("--output", default=None)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without torchrun the sweep starts them itself")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend (nccl = RCCL; gloo lets ranks share one GPU)")
    args = ap.parse_args(argv)
    from . import launch
    gpus = args.gpus if args.gpus is not None else int(os.environ.get("WORLD_SIZE", "1"))
    # the ranks run this module's entry point (not sys.argv[0], which under
    # `python -m kvecc.montecarlo` is this file, unimportable as a script, and
    # under another program calling main(argv) is that program)
    rc = launch.launch_if_needed(["-m", "kvecc.montecarlo"], list(sys.argv[1:] if argv is None else argv),
                                 gpus, args.backend)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        print(f"sweep: --gpus {gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    ngpu = torch.cuda.device_count()
    local_dev = local % ngpu if args.backend == "gloo" and ngpu else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        launch.check_world(dist, gpus)
    cfg = MonteCarloConfig(shape=tuple(args.shape), codecs=tuple(args.codecs),
                           bers=tuple(args.bers), seeds=tuple(args.seeds), output=args.output)
    shard = HipShard(cfg, rank, world, dev)
    rows, elapsed = run_sweep(cfg, shard, dist, rank)
    if rank == 0:
        for r in rows:
            print(json.dumps(r))
        print(json.dumps({"trials": len(rows), "seconds": elapsed, "world": world,
                          "backend": dist.get_backend() if dist is not None else None}))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
