"""Batched fused shim read (kvecc_shim_read_batch): gather -> decode -> dequantize
for every sequence of a paged cache (ecc_shim.py:990-1071, the consumer of
golay_decode the headline's "fused Golay decode" names).

CPU tier: the host twin against a numpy restatement over the oracle's decoders
(bit-exact values and statistics).  GPU tier: the HIP path -- the wave-tile
Golay kernel for d % 8 == 0, the per-sequence kernels otherwise -- against the
host twin, bit for bit, over codecs, output dtypes, head dims, block sizes,
partial blocks, missing blocks, and the full [B=8, L=4096, Hkv=32, D=128] size.
"""

import numpy as np
import pytest
import torch

BER = 2e-2


def _pack_golay(cache, g):
    """int32 Golay cache [..., bs * g] -> packed rows of KVECC_GOLAY_PACKED_ROW(g) bytes."""
    row = (3 * g + 3) // 4 * 4
    w = cache.reshape(*cache.shape[:-1], -1, g).numpy().astype(np.uint32)
    out = np.zeros(w.shape[:-1] + (row,), np.uint8)
    for byte in range(3):
        out[..., byte:3 * g:3] = (w >> (8 * byte)) & 0xFF
    return torch.from_numpy(out.reshape(*cache.shape[:-1], -1))


def make_cache(codec, batch, ctx, hkv, d, bs, layers=2, seed=0, spare=3, ber=BER):
    """Random paged caches (cpu backend, oracle-pinned codecs) with BER-level errors.
    Returns caches, scales, block table [batch, max_blocks] (a random
    permutation of physical blocks) and the codeword count per row."""
    from kvecc import cpu_ops
    g = torch.Generator().manual_seed(seed)
    nlb = (ctx + bs - 1) // bs
    nb = batch * nlb + spare
    golay = codec in ("golay", "golay_packed")
    per = (d + 2) // 3 if golay else d
    vals = torch.randint(0, 16, (2, nb, layers, hkv, bs, d), generator=g, dtype=torch.uint8)
    caches = []
    for side in range(2):
        x = vals[side]
        if golay:
            cw = cpu_ops.golay_encode_rows(x).reshape(nb, layers, hkv, bs * per)
            cw = cpu_ops.inject_bit_errors_triton(cw, ber, 24, seed=seed + side)
            caches.append(_pack_golay(cw, per) if codec == "golay_packed" else cw)
        else:
            enc = {"hamming84": cpu_ops.hamming84_encode, "hamming74": cpu_ops.hamming74_encode,
                   "int4": lambda t: t}[codec](x).reshape(nb, layers, hkv, bs * d)
            if codec != "int4":
                enc = cpu_ops.inject_bit_errors_triton(enc, ber, 8 if codec == "hamming84" else 7,
                                                       seed=seed + side)
            caches.append(enc)
    ks = torch.rand(nb, layers, hkv, bs, generator=g) * 0.5 + 0.01
    vs = torch.rand(nb, layers, hkv, bs, generator=g) * 0.5 + 0.01
    max_blocks = nlb + 1
    table = torch.full((batch, max_blocks), -1, dtype=torch.int32)
    table[:, :nlb] = torch.randperm(nb, generator=g)[: batch * nlb].to(torch.int32).view(batch, nlb)
    return caches[0], caches[1], ks, vs, table


def oracle_read(oracle, cache, scales, table, ctx, d, layer, codec, out_dtype, interp=False):
    """numpy restatement of the read for one side: [B, hkv, ctx, d] and (stat0, stat1).

    interp (H84): the composed read of ecc_shim.py:1038-1059 per sequence --
    decode the whole context, then oracle.interpolate_double_errors along ctx
    (interpolation_triton.py:120-159, neighbours clamped to [0, ctx - 1]); a
    missing (-1) block's rows read as zero codewords (decode(0) = 0, no error)
    and output +0."""
    nb, layers, hkv, row = cache.shape
    golay = codec in ("golay", "golay_packed")
    g = (d + 2) // 3
    per = ((3 * g + 3) // 4 * 4) if codec == "golay_packed" else (g if golay else d)
    bs = row // per
    c = cache.numpy().reshape(nb, layers, hkv, bs, per)
    sc = scales.numpy()
    batch = table.shape[0]
    out = np.zeros((batch, hkv, ctx, d), np.float32)
    st = [0, 0]
    for b in range(batch):
        pos = np.arange(ctx)
        blk = table[b, pos // bs].numpy().astype(np.int64)
        slot = pos % bs
        ok = blk >= 0
        rows = c[blk[ok], layer, :, slot[ok]]  # [n, hkv, per]
        s = sc[blk[ok], layer, :, slot[ok]]  # [n, hkv]
        if golay:
            if codec == "golay_packed":
                b3 = rows[..., :3 * g].astype(np.uint32).reshape(*rows.shape[:-1], g, 3)
                w = (b3[..., 0] | b3[..., 1] << 8 | b3[..., 2] << 16).astype(np.int32)
            else:
                w = rows.astype(np.int32)
            trip, _, (bits, unc) = oracle.golay_decode(w.reshape(-1))
            q = trip.reshape(*w.shape[:-1], 3 * g)[..., :d]
            st[0] += bits
            st[1] += unc
        elif codec == "hamming84" and interp:
            full = np.zeros((ctx, hkv, d), np.uint8)
            full[pos[ok]] = rows  # missing rows: codeword 0
            q, et, (c1, c2) = oracle.hamming84_decode(full.reshape(-1))
            q = oracle.interpolate_double_errors(q.reshape(ctx, hkv, d), et.reshape(ctx, hkv, d), seq_dim=0)
            q = q[pos[ok]]
            st[0] += c1
            st[1] += c2
        elif codec == "hamming84":
            q, _, (c1, c2) = oracle.hamming84_decode(rows.reshape(-1))
            q = q.reshape(rows.shape)
            st[0] += c1
            st[1] += c2
        elif codec == "hamming74":
            q, _, (c1,) = oracle.hamming74_decode(rows.reshape(-1))
            q = q.reshape(rows.shape)
            st[0] += c1
        else:
            q = rows
        val = (q.astype(np.float32) - np.float32(8.0)) * s[..., None].astype(np.float32)
        out[b][:, pos[ok]] = val.transpose(1, 0, 2)
    t = torch.from_numpy(out)
    return t.to(out_dtype), st


CPU_CASES = [("golay", 2, 37, 3, 128, 16), ("golay_packed", 2, 37, 3, 128, 16),
             ("golay", 3, 20, 2, 64, 7), ("golay", 1, 9, 2, 100, 4), ("hamming84", 2, 33, 2, 64, 16),
             ("hamming74", 2, 17, 2, 32, 8), ("int4", 1, 12, 3, 16, 4)]


@pytest.mark.parametrize("codec,batch,ctx,hkv,d,bs", CPU_CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_cpu_batch_read_vs_oracle(oracle, codec, batch, ctx, hkv, d, bs, dtype):
    from kvecc import cpu_ops
    kc, vc, ks, vs, table = make_cache(codec, batch, ctx, hkv, d, bs, seed=ctx)
    st = cpu_ops.new_stats()
    k, v = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, 1, codec, dtype, stats=st)
    ek, sk = oracle_read(oracle, kc, ks, table, ctx, d, 1, codec, dtype)
    ev, sv = oracle_read(oracle, vc, vs, table, ctx, d, 1, codec, dtype)
    assert torch.equal(k, ek) and torch.equal(v, ev)
    assert cpu_ops.read_stats(st) == [sk[0] + sv[0], sk[1] + sv[1]]


def _plant_doubles(cache, table, d, bs, layer, rows):
    """Make every codeword of the listed (sequence, position) rows a double
    error (two flipped data bits: SECDED DOUBLE_DETECTED) in-place."""
    c = cache.view(cache.shape[0], cache.shape[1], cache.shape[2], bs, d)
    for b, pos in rows:
        blk = int(table[b, pos // bs])
        if blk >= 0:
            c[blk, layer, :, pos % bs, :] ^= 0x03


# H(8,4) + interpolation against the oracle: doubles planted in the first and
# last rows of 16-row tiles, at the context's ends and next to missing blocks.
INTERP_CPU_CASES = [(2, 70, 2, 64, 16), (1, 40, 3, 32, 16), (2, 33, 2, 128, 8), (1, 1, 1, 16, 16),
                    (2, 45, 2, 48, 7)]


@pytest.mark.parametrize("batch,ctx,hkv,d,bs", INTERP_CPU_CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_cpu_batch_read_interp_vs_oracle(oracle, batch, ctx, hkv, d, bs, dtype):
    from kvecc import cpu_ops
    kc, vc, ks, vs, table = make_cache("hamming84", batch, ctx, hkv, d, bs, seed=ctx + 5, ber=3e-3)
    rows = set()
    for b in range(batch):
        for pos in (0, ctx - 1, 15, 16, 31, 32, bs - 1, bs, 2 * bs - 1):
            if 0 <= pos < ctx:
                rows.add((b, pos))
    for kv in (kc, vc):
        _plant_doubles(kv, table, d, bs, 1, sorted(rows))
    nlb = (ctx + bs - 1) // bs
    if nlb > 2:  # a missing inner block: its neighbours interpolate against zeros
        table[batch - 1, 1] = -1
    st = cpu_ops.new_stats()
    k, v = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, 1, "hamming84", dtype, interp=True, stats=st)
    ek, sk = oracle_read(oracle, kc, ks, table, ctx, d, 1, "hamming84", dtype, interp=True)
    ev, sv = oracle_read(oracle, vc, vs, table, ctx, d, 1, "hamming84", dtype, interp=True)
    assert sk[1] > 0  # doubles were decoded
    assert torch.equal(k, ek) and torch.equal(v, ev)
    assert cpu_ops.read_stats(st) == [sk[0] + sv[0], sk[1] + sv[1]]


def test_cpu_missing_byte_block_reads_zero():
    """Byte codecs: a -1 block reads as +0 rows; as an interpolation neighbour
    its codewords read as 0 (decode(0) = 0)."""
    from kvecc import cpu_ops
    kc, vc, ks, vs, table = make_cache("hamming84", 1, 40, 2, 64, 16, seed=4)
    table[0, 1] = -1
    k, _ = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, 40, 64, 1, "hamming84", torch.float32, interp=True)
    assert torch.equal(k[0, :, 16:32], torch.zeros(2, 16, 64))
    assert bool(torch.isfinite(k).all())


def test_cpu_missing_golay_block_reads_zero(oracle):
    from kvecc import cpu_ops
    kc, vc, ks, vs, table = make_cache("golay", 2, 40, 2, 64, 16, seed=4)
    table[1, 1] = -1
    k, v = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, 40, 64, 1, "golay", torch.float32)
    assert torch.equal(k[1, :, 16:32], torch.zeros(2, 16, 64))
    ek, _ = oracle_read(oracle, kc, ks, table, 40, 64, 1, "golay", torch.float32)
    assert torch.equal(k, ek)


GPU_CASES = CPU_CASES + [("golay", 4, 257, 4, 128, 16), ("golay_packed", 3, 100, 8, 64, 32),
                         ("golay", 2, 50, 2, 256, 8), ("golay", 1, 3, 1, 8, 16),
                         ("golay_packed", 2, 64, 2, 512, 2), ("golay", 2, 31, 2, 96, 5),
                         # byte codecs: wave tiles for d % 16 == 0, per-sequence kernels otherwise
                         ("hamming84", 4, 257, 4, 128, 16), ("hamming74", 2, 100, 3, 64, 32),
                         ("int4", 2, 50, 2, 256, 8), ("hamming84", 1, 3, 1, 16, 16),
                         ("hamming84", 2, 64, 2, 512, 2), ("hamming84", 2, 31, 2, 48, 5),
                         ("hamming84", 2, 20, 2, 36, 4), ("hamming74", 1, 70, 2, 128, 128)]


@pytest.mark.gpu
@pytest.mark.parametrize("codec,batch,ctx,hkv,d,bs", GPU_CASES)
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_hip_batch_read_vs_cpu(gpu, codec, batch, ctx, hkv, d, bs, dtype):
    from kvecc import cpu_ops, ops
    kc, vc, ks, vs, table = make_cache(codec, batch, ctx, hkv, d, bs, seed=ctx + d)
    st = cpu_ops.new_stats()
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, 1, codec, dtype, stats=st)
    gst = ops.new_stats(gpu)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), ctx, d, 1, codec, dtype, stats=gst)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


INTERP_CASES = [(3, 70, 2, 64, 16), (2, 33, 2, 128, 16), (1, 1, 1, 16, 16), (2, 100, 3, 512, 4),
                (2, 45, 2, 32, 7), (1, 17, 2, 128, 64), (2, 40, 2, 36, 8),
                # blocks that split into unequal tiles (the last chunk shorter): d 256 -> 7-row
                # tiles of 16-row blocks (7, 7, 2); d 128 with 24-row blocks (16, 8)
                (2, 100, 2, 256, 16), (2, 90, 2, 128, 24)]


@pytest.mark.gpu
@pytest.mark.parametrize("batch,ctx,hkv,d,bs", INTERP_CASES)
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_hip_batch_read_interp_vs_cpu(gpu, batch, ctx, hkv, d, bs, dtype):
    """H(8,4) with double-error interpolation: neighbours across block and tile
    boundaries, context ends clamped, partial blocks, statistics."""
    from kvecc import cpu_ops, ops
    kc, vc, ks, vs, table = make_cache("hamming84", batch, ctx, hkv, d, bs, seed=9 + ctx)
    st, gst = cpu_ops.new_stats(), ops.new_stats(gpu)
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, 1, "hamming84", dtype,
                                     interp=True, stats=st)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), ctx, d, 1, "hamming84",
                               dtype, interp=True, stats=gst)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


# many tiles (shim_read_h84_interp_kernel: one tile per wave; a double in a
# tile's first or last row reads the neighbour row from memory, an interior one
# interpolates inside the tile): several tiles per block (bs 64 > 16 rows per
# tile), partial last blocks, missing blocks (first, inner, last; a neighbour
# row in a missing block reads as zero codewords).  At low BER most tiles hold
# no double error (no interpolation arithmetic, no neighbour rows) and a few
# need a neighbour row; at 2e-2 nearly every tile edge does.
MANY_TILE_CASES = [(4, 2001, 4, 32, 6, 2e-2), (3, 5000, 8, 128, 64, 2e-2), (2, 4099, 16, 64, 16, 1e-3),
                   (3, 5000, 8, 128, 64, 1e-3), (4, 2001, 4, 32, 6, 3e-4), (2, 4099, 16, 128, 16, 0.0),
                   (2, 3001, 4, 256, 16, 2e-2), (3, 2500, 4, 128, 24, 2e-2)]


@pytest.mark.gpu
@pytest.mark.parametrize("batch,ctx,hkv,d,bs,ber", MANY_TILE_CASES)
def test_hip_batch_read_interp_many_tiles(gpu, batch, ctx, hkv, d, bs, ber):
    from kvecc import cpu_ops, ops
    kc, vc, ks, vs, table = make_cache("hamming84", batch, ctx, hkv, d, bs, layers=1, seed=ctx, ber=ber)
    table[0, 3] = -1
    table[batch - 1, (ctx - 1) // bs] = -1  # the last block of a sequence
    table[1, 0] = -1  # the first
    st, gst = cpu_ops.new_stats(), ops.new_stats(gpu)
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, 0, "hamming84", torch.float16,
                                     interp=True, stats=st)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), ctx, d, 0, "hamming84", torch.float16,
                               interp=True, stats=gst)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


# random geometries (seeded): every head size the wave-tile kernels take
# (d % 16 == 0, interpolation up to d = 512), block sizes that split into
# equal and unequal tiles, partial last blocks, 1-3 layers, BER high enough
# that most tiles hold doubles -- the byte reads, plain and interpolating,
# against the host twin
def _random_geometries(n, seed=2024):
    import random
    r = random.Random(seed)
    out = []
    for _ in range(n):
        d = 16 * r.randint(1, 32)
        bs = r.choice([1, 3, 4, 7, 8, 16, 24, 32, 40, 64])
        ctx = r.randint(1, 12 * bs + 5)
        out.append((r.randint(1, 3), ctx, r.randint(1, 3), d, bs, r.randint(1, 3), r.choice([True, False])))
    return out


# KVECC_SWEEP_SCALE / KVECC_SWEEP_SEED: an extended run (tests/test_geometry_sweep.py)
_SCALE = int(__import__("os").environ.get("KVECC_SWEEP_SCALE", "1"))
_SEED = int(__import__("os").environ.get("KVECC_SWEEP_SEED", "0"))


@pytest.mark.gpu
@pytest.mark.parametrize("batch,ctx,hkv,d,bs,layers,interp", _random_geometries(16 * _SCALE, 2024 + _SEED))
def test_hip_byte_read_random_geometry(gpu, batch, ctx, hkv, d, bs, layers, interp):
    from kvecc import cpu_ops, ops
    kc, vc, ks, vs, table = make_cache("hamming84", batch, ctx, hkv, d, bs, layers=layers, seed=ctx + d,
                                       ber=3e-2)
    layer = layers - 1
    st, gst = cpu_ops.new_stats(), ops.new_stats(gpu)
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, layer, "hamming84", torch.float16,
                                     interp=interp, stats=st)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), ctx, d, layer, "hamming84", torch.float16,
                               interp=interp, stats=gst)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


def _random_golay_geometries(n, seed=4048):
    import random
    r = random.Random(seed)
    out = []
    for _ in range(n):
        d = 8 * r.randint(1, 48)
        bs = r.choice([1, 3, 4, 7, 8, 16, 24, 32, 40, 64])
        ctx = r.randint(1, 12 * bs + 5)
        out.append((r.choice(["golay", "golay_packed"]), r.randint(1, 3), ctx, r.randint(1, 3), d, bs,
                    r.randint(1, 3)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("codec,batch,ctx,hkv,d,bs,layers", _random_golay_geometries(12 * _SCALE, 4048 + _SEED))
def test_hip_golay_read_random_geometry(gpu, codec, batch, ctx, hkv, d, bs, layers):
    """The Golay wave-tile read (d % 8 == 0) on random geometries against the host twin."""
    from kvecc import cpu_ops, ops
    kc, vc, ks, vs, table = make_cache(codec, batch, ctx, hkv, d, bs, layers=layers, seed=ctx + d)
    layer = layers - 1
    st, gst = cpu_ops.new_stats(), ops.new_stats(gpu)
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, layer, codec, torch.float16, stats=st)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), ctx, d, layer, codec, torch.float16,
                               stats=gst)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


@pytest.mark.gpu
@pytest.mark.parametrize("codec,interp,d", [("hamming84", False, 64), ("hamming84", True, 64),
                                            ("hamming74", False, 64), ("int4", False, 64),
                                            # per-sequence kernels: d % 16 != 0, or interp with d > 512
                                            ("hamming84", False, 36), ("hamming84", True, 48),
                                            ("hamming74", False, 36), ("int4", False, 48),
                                            ("hamming84", True, 528)])
def test_hip_missing_byte_block_reads_zero(gpu, codec, interp, d):
    """A -1 block (never produced by the shim) reads as +0 rows, and as zero
    codewords where it is an interpolation neighbour -- the same on both backends
    and in both the wave-tile and the per-sequence kernels."""
    from kvecc import cpu_ops, ops
    kc, vc, ks, vs, table = make_cache(codec, 2, 40, 2, d, 16, seed=4)
    table[1, 1] = -1
    table[0, 0] = -1
    st, gst = cpu_ops.new_stats(), ops.new_stats(gpu)
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, 40, d, 1, codec, torch.float16, stats=st,
                                     interp=interp)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), 40, d, 1, codec, torch.float16,
                               stats=gst, interp=interp)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert torch.equal(k[1, :, 16:32].cpu(), torch.zeros(2, 16, d, dtype=torch.float16))
    assert torch.equal(k[0, :, 0:16].cpu(), torch.zeros(2, 16, d, dtype=torch.float16))
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["golay", "golay_packed"])
def test_hip_missing_golay_block_reads_zero(gpu, codec):
    from kvecc import cpu_ops, ops
    kc, vc, ks, vs, table = make_cache(codec, 2, 40, 2, 64, 16, seed=4)
    table[1, 1] = -1
    table[0, 0] = -1
    st, gst = cpu_ops.new_stats(), ops.new_stats(gpu)
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, 40, 64, 1, codec, torch.float16, stats=st)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), 40, 64, 1, codec, torch.float16,
                               stats=gst)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert torch.equal(k[1, :, 16:32].cpu(), torch.zeros(2, 16, 64, dtype=torch.float16))
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["golay", "golay_packed", "hamming84", "hamming84+interp"])
def test_hip_batch_read_full_size(gpu, codec):
    """[B=8, L=4096, Hkv=32, D=128] (the bench's fused-decode workload), fp16,
    bit-exact against the host twin, statistics included."""
    from kvecc import cpu_ops, ops
    batch, ctx, hkv, d, bs = 8, 4096, 32, 128, 16
    interp = codec.endswith("+interp")
    codec = codec.split("+")[0]
    kc, vc, ks, vs, table = make_cache(codec, batch, ctx, hkv, d, bs, layers=1, seed=1, spare=0)
    st = cpu_ops.new_stats()
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, 0, codec, torch.float16, stats=st,
                                     interp=interp)
    gst = ops.new_stats(gpu)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), ctx, d, 0, codec, torch.float16,
                               stats=gst, interp=interp)
    assert torch.equal(k.cpu(), ek)
    assert torch.equal(v.cpu(), ev)
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["golay", "golay_packed"])
def test_hip_golay_read_unaligned_out(gpu, codec):
    """Outputs that start off a 16-byte boundary leave the wave-tile kernel
    (16-byte buffer stores) for the per-sequence kernel: same values."""
    from kvecc import cpu_ops, ops
    batch, ctx, hkv, d, bs = 2, 40, 2, 64, 16
    kc, vc, ks, vs, table = make_cache(codec, batch, ctx, hkv, d, bs, seed=12)
    st, gst = cpu_ops.new_stats(), ops.new_stats(gpu)
    ek, ev = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, ctx, d, 1, codec, torch.float16, stats=st)
    n = batch * hkv * ctx * d
    bufs = [torch.empty(n + 1, dtype=torch.float16, device=gpu) for _ in range(2)]
    out = tuple(b[1:].view(batch, hkv, ctx, d) for b in bufs)
    t = lambda x: x.to(gpu)  # noqa: E731
    k, v = ops.shim_read_batch(t(kc), t(vc), t(ks), t(vs), t(table), ctx, d, 1, codec, torch.float16,
                               stats=gst, out=out)
    assert torch.equal(k.cpu(), ek) and torch.equal(v.cpu(), ev)
    assert ops.read_stats(gst) == cpu_ops.read_stats(st)
