"""Seeded random-geometry parity sweeps for the kernels whose launch geometry
depends on the shape: paged decode attention (attention_ecc.py:264-427,
620-780, 783-909), the per-head Golay rows and the packed decodes.

The round-4 interpolating read went in green and was wrong for block / tile
splits no hand-picked case covered; a 28-shape random sweep
(tests/test_shim_read_batch.py) caught it.  These sweeps do the same for the
other geometry-dependent kernels:

  * attention: codec (Hamming(8,4), int32 and packed Golay), block_size in
    {1, 4, 8, 16, 24, 32}, head_dim in {20, 32, 64, 100, 128}, GQA groups 1-16,
    1-3 layers, context lengths that end mid-block, -1 holes in the block
    table, fp32 / fp16 / bf16 queries; HIP against the fp32 torch restatement
    (tests/test_attention.py::_torch_reference) and against the host twin;
  * rows and packed decodes: row counts, head dims, buffer offsets (unaligned
    pointers take the kernels' other paths) and tails, HIP against the host
    twin bit for bit (outputs and statistics).

A failing case prints its parameters; keep it as a regression case below.
"""

import math
import os
import random

import pytest
import torch

from tests.test_attention import _cache, _pack_golay, _torch_reference

# KVECC_SWEEP_SCALE=k multiplies every sweep's case count and KVECC_SWEEP_SEED=s
# shifts its seeds (an extended run; the defaults are the suite's)
SCALE = int(os.environ.get("KVECC_SWEEP_SCALE", "1"))
SEED = int(os.environ.get("KVECC_SWEEP_SEED", "0"))
N_ATTN = 40 * SCALE
N_ROWS = 24 * SCALE
N_PACKED = 24 * SCALE


def _attn_cases():
    rng = random.Random(20251018 + SEED)
    cases = []
    for i in range(N_ATTN):
        codec = rng.choice(["hamming84", "golay", "golay_packed"])
        bs = rng.choice([1, 4, 8, 16, 24, 32])
        d = rng.choice([20, 32, 64, 100, 128])
        kvh = rng.choice([1, 2, 4, 8])
        groups = rng.choice([1, 2, 3, 4, 8, 16])
        batch = rng.randint(1, 3)
        ctx = rng.randint(1, 24) * bs + rng.randint(1, max(1, bs - 1)) if bs > 1 else rng.randint(2, 300)
        layers = rng.randint(1, 3)
        layer = rng.randrange(layers)
        holes = rng.random() < 0.5
        dtype = rng.choice(["float32", "float16", "bfloat16"])
        ber = rng.choice([0.0, 1e-3, 1e-2])
        cases.append((i, codec, bs, d, kvh, groups, batch, ctx, layers, layer, holes, dtype, ber))
    # regression cases found by earlier sweeps go here
    return cases


ATTN_CASES = _attn_cases()


def _attn_inputs(codec, bs, d, kvh, groups, batch, ctx, layers, layer, holes, ber, seed):
    base = "hamming84" if codec == "hamming84" else "golay"
    heads = kvh * groups
    kc, vc, table, lens, ks, vs = _cache("cpu", base, batch, heads, kvh, d, ctx, ber, seed=seed,
                                         layers=layers, layer=layer, bs=bs)
    if holes:
        g = torch.Generator().manual_seed(seed + 1)
        nblk = (ctx + bs - 1) // bs
        for b in range(batch):
            if nblk > 1:
                table[b, int(torch.randint(0, nblk, (1,), generator=g))] = -1
    return base, heads, kc, vc, table, lens, ks, vs


@pytest.mark.parametrize("case", ATTN_CASES, ids=[f"a{c[0]}" for c in ATTN_CASES])
def test_attention_sweep_cpu_twin_vs_torch(case):
    """The host twin over the same geometry (the GPU test compares against it too)."""
    from kvecc import cpu_ops
    i, codec, bs, d, kvh, groups, batch, ctx, layers, layer, holes, dtype, ber = case
    if i % 4:  # a quarter of the sweep on the CPU tier (the torch reference is slow)
        pytest.skip("CPU tier runs every fourth case")
    base, heads, kc, vc, table, lens, ks, vs = _attn_inputs(codec, bs, d, kvh, groups, batch, ctx, layers,
                                                           layer, holes, ber, seed=100 + i)
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(i))
    ref = _torch_reference(q, kc, vc, table, lens, ks, vs, layer, bs, base)
    if codec == "golay_packed":
        kc, vc = _pack_golay(kc, d), _pack_golay(vc, d)
    out = torch.empty(batch, heads, d)
    cpu_ops.paged_attention_into(q, kc, vc, table, lens, ks, vs, out, layer, bs, 1 / math.sqrt(d), codec)
    _close(out, ref, torch.float32, case)


def _close(got, ref, dtype, case):
    got = got.float()
    valid = ~torch.isnan(ref)
    tol = {torch.float32: (2e-5, 2e-4), torch.float16: (1e-3, 1e-3), torch.bfloat16: (1e-2, 1e-2)}[dtype]
    assert torch.allclose(got[valid], ref[valid], atol=tol[0], rtol=tol[1]), \
        (case, float((got - ref).abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ATTN_CASES, ids=[f"a{c[0]}" for c in ATTN_CASES])
def test_attention_sweep_hip(gpu, case):
    from kvecc import cpu_ops, ops
    i, codec, bs, d, kvh, groups, batch, ctx, layers, layer, holes, dtype, ber = case
    dt = getattr(torch, dtype)
    base, heads, kc, vc, table, lens, ks, vs = _attn_inputs(codec, bs, d, kvh, groups, batch, ctx, layers,
                                                           layer, holes, ber, seed=100 + i)
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(i)).to(dt)
    ref = _torch_reference(q.float(), kc, vc, table, lens, ks, vs, layer, bs, base)
    if codec == "golay_packed":
        kc, vc = _pack_golay(kc, d), _pack_golay(vc, d)
    twin = torch.empty(batch, heads, d)
    cpu_ops.paged_attention_into(q.float(), kc, vc, table, lens, ks, vs, twin, layer, bs, 1 / math.sqrt(d),
                                 codec)
    g = lambda t: t.to(gpu)  # noqa: E731
    out = torch.empty(batch, heads, d, dtype=dt, device=gpu)
    ops.paged_attention_into(g(q), g(kc), g(vc), g(table), g(lens), g(ks), g(vs), out, layer, bs,
                             1 / math.sqrt(d), codec)
    got = out.cpu()
    _close(got, ref, dt, case)
    _close(got, twin, dt, case)
    # a context with no valid token gives the reference's constant (H84 -8, Golay 0)
    for b in range(batch):
        nblk = (int(lens[b]) + bs - 1) // bs
        if nblk and bool((table[b, :nblk] < 0).all()):
            assert torch.equal(got[b].float(), torch.full((heads, d), -8.0 if base == "hamming84" else 0.0))


# ---- per-head Golay rows ----------------------------------------------------------

def _rows_cases():
    rng = random.Random(77 + SEED)
    return [(i, rng.choice([1, 2, 3, 5, 20, 64, 100, 128, 129, 256]), rng.choice([1, 7, 63, 64, 65, 1000, 4097]),
             rng.choice([0, 1, 3, 17]), rng.choice([0.0, 1e-2, 5e-2])) for i in range(N_ROWS)]


ROWS_CASES = _rows_cases()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ROWS_CASES, ids=[f"r{c[0]}" for c in ROWS_CASES])
def test_golay_rows_sweep_hip_vs_host(gpu, case):
    """golay_encode_rows / golay_decode_rows at random (rows, head_dim), the
    codewords placed `off` int32 words into a larger buffer (unaligned rows)."""
    from kvecc import cpu_ops, ops
    i, d, rows, off, ber = case
    g = (d + 2) // 3
    x = torch.randint(0, 16, (rows, d), generator=torch.Generator().manual_seed(i), dtype=torch.uint8)
    cw = cpu_ops.golay_encode_rows(x)
    assert torch.equal(ops.golay_encode_rows(x.to(gpu)).cpu(), cw), case
    if ber > 0:
        cw = cpu_ops.inject_bit_errors_triton(cw, ber, 24, seed=i)
    big = torch.zeros(off + rows * g + 5, dtype=torch.int32)
    big[off:off + rows * g] = cw.view(-1)
    view = big[off:off + rows * g].view(rows, g)
    st_h = cpu_ops.new_stats()
    want = cpu_ops.golay_decode_rows(view.contiguous(), d, stats=st_h)
    bg = big.to(gpu)
    out = torch.full((rows, d), 0xEE, dtype=torch.uint8, device=gpu)
    st = ops.new_stats(gpu)
    ops.golay_decode_rows_into(bg[off:off + rows * g].view(rows, g), out, st)
    assert torch.equal(out.cpu(), want), case
    assert ops.read_stats(st) == cpu_ops.read_stats(st_h), case


# ---- packed decodes ------------------------------------------------------------------

def _packed_cases():
    rng = random.Random(99 + SEED)
    return [(i, rng.choice(["golay", "hamming84"]), rng.choice([1, 2, 3, 5, 31, 32, 33, 1000, 4095, 65537]),
             rng.choice([0, 1, 2, 3, 5, 16]), rng.choice([0.0, 1e-2, 5e-2])) for i in range(N_PACKED)]


PACKED_CASES = _packed_cases()


@pytest.mark.gpu
@pytest.mark.parametrize("case", PACKED_CASES, ids=[f"p{c[0]}" for c in PACKED_CASES])
def test_packed_decode_sweep_hip_vs_host(gpu, case):
    """Packed Golay / Hamming(8,4) decodes at random lengths, the codeword bytes
    `off` bytes into a larger buffer and the outputs likewise offset."""
    from kvecc import cpu_ops, ops
    i, codec, m, off, ber = case
    gen = torch.Generator().manual_seed(1000 + i)
    if codec == "golay":
        nib = torch.randint(0, 256, ((3 * m + 1) // 2,), generator=gen, dtype=torch.uint8)
        if (3 * m) % 2:
            nib[-1] &= 0x0F
        cw = cpu_ops.golay_encode_packed(nib, m)
        assert torch.equal(ops.golay_encode_packed(nib.to(gpu), m).cpu(), cw), case
        if ber > 0:
            cw = cpu_ops.inject_bit_errors_triton(cw, ber, 8, seed=i)
        n_cw, n_out, n_flag = 3 * m, (3 * m + 1) // 2, (m + 7) // 8
    else:
        nib = torch.randint(0, 256, ((m + 1) // 2,), generator=gen, dtype=torch.uint8)
        if m % 2:
            nib[-1] &= 0x0F
        cw = cpu_ops.hamming84_encode_packed(nib, m)
        assert torch.equal(ops.hamming84_encode_packed(nib.to(gpu), m).cpu(), cw), case
        if ber > 0:
            cw = cpu_ops.inject_bit_errors_triton(cw, ber, 8, seed=i)
        n_cw, n_out, n_flag = m, (m + 1) // 2, (m + 3) // 4
    big = torch.zeros(off + n_cw + 7, dtype=torch.uint8)
    big[off:off + n_cw] = cw
    if codec == "golay":
        want_nib, want_flag, want_st = cpu_ops.golay_decode_packed(big[off:off + n_cw].clone(), m,
                                                                   return_uncorrectable=True)
    else:
        want_nib, want_flag, want_st = cpu_ops.hamming84_decode_packed(big[off:off + n_cw].clone(),
                                                                       return_error_types=True)
    bg = big.to(gpu)
    out_big = torch.full((off + n_out + 3,), 0xEE, dtype=torch.uint8, device=gpu)
    flag_big = torch.full((off + n_flag + 3,), 0xEE, dtype=torch.uint8, device=gpu)
    st = ops.new_stats(gpu)
    src, dst, fl = bg[off:off + n_cw], out_big[off:off + n_out], flag_big[off:off + n_flag]
    if codec == "golay":
        ops.golay_decode_packed_into(src, dst, fl, m, st)
    else:
        ops.hamming84_decode_packed_into(src, dst, fl, m, st)
    assert torch.equal(dst.cpu(), want_nib), case
    assert torch.equal(fl.cpu(), want_flag), case
    assert tuple(ops.read_stats(st)) == tuple(want_st), case
    # nothing written outside the outputs
    assert bool((out_big[:off] == 0xEE).all()) and bool((out_big[off + n_out:] == 0xEE).all()), case
    assert bool((flag_big[:off] == 0xEE).all()) and bool((flag_big[off + n_flag:] == 0xEE).all()), case


# ---- interpolation (workgroup tiles of 64 column chunks x 32 positions) -------------

def _interp_cases():
    rng = random.Random(4242 + SEED)
    cases = []
    for i in range(24 * SCALE):
        inner = rng.choice([16, 48, 160, 1008, 1024, 1040, 4096, 24, 7])
        length = rng.choice([1, 2, 3, 4, 5, 31, 32, 33, 63, 64, 65, 100, 257])
        outer = rng.choice([1, 2, 3, 5])
        cases.append((i, outer, length, inner, rng.choice([0.0, 0.02, 0.3])))
    return cases


INTERP_CASES = _interp_cases()


@pytest.mark.gpu
@pytest.mark.parametrize("case", INTERP_CASES, ids=[f"i{c[0]}" for c in INTERP_CASES])
def test_interp_tile_sweep_hip_vs_oracle(gpu, oracle, case):
    """interpolate_double_errors along the middle axis of [outer, len, inner] at
    ragged lengths (tiles that end mid-wave, waves that end mid-tile), column
    counts that leave a partial 64-chunk group, and the scalar path (inner % 16
    != 0); both the gated kernel and the recording pass (the API)."""
    import numpy as np

    import kvecc
    from kvecc import ops
    i, outer, length, inner, pdbl = case
    rng = np.random.default_rng(i)
    q = rng.integers(0, 16, size=(outer, length, inner), dtype=np.int64).astype(np.uint8)
    e = rng.choice(np.array([0, 1, 2, 3], np.uint8), size=q.shape,
                   p=[1 - pdbl - 0.1, 0.05, pdbl, 0.05])
    want = oracle.interpolate_double_errors(q, e, seq_dim=1)
    got = kvecc.interpolate_double_errors(torch.from_numpy(q).to(gpu), torch.from_numpy(e).to(gpu), seq_dim=1)
    assert np.array_equal(got.cpu().numpy(), want), case
    # the plain kernel (every element through the formula) against the oracle's kernel semantics
    out = torch.empty(q.size, dtype=torch.uint8, device=gpu)
    ops.interpolate_into(torch.from_numpy(q).to(gpu).view(-1), torch.from_numpy(e).to(gpu).view(-1), out,
                         outer, length, inner)
    assert np.array_equal(out.cpu().numpy().reshape(q.shape),
                          oracle.interpolate_kernel(q, e, outer, length, inner).reshape(q.shape)), case
