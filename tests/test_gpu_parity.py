"""HIP kernels vs the oracle and the reference's golden vectors (MI355X only).

Bit-exact for every integer output (codewords, data, error types, counts,
statistics); fp32/fp16 dequantization is compared exactly as well, since the
arithmetic is the same IEEE sequence (torch's own .to(fp16) rounding).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _np(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------------------
# Hamming
# ---------------------------------------------------------------------------

def test_hamming_all_bytes_golden(gpu, golden):
    import kvecc
    g = golden("hamming")
    x = _t(g["inputs"], gpu)
    assert np.array_equal(_np(kvecc.hamming74_encode(x)), g["enc74"])
    assert np.array_equal(_np(kvecc.hamming84_encode(x)), g["enc84"])
    d, f, st = kvecc.hamming74_decode(x, return_error_detected=True)
    assert np.array_equal(_np(d), g["dec74_data"]) and np.array_equal(_np(f), g["dec74_flag"])
    assert st == tuple(g["dec74_stats"].tolist())
    d, t, st = kvecc.hamming84_decode(x, return_error_types=True)
    assert np.array_equal(_np(d), g["dec84_data"]) and np.array_equal(_np(t), g["dec84_type"])
    assert st == tuple(g["dec84_stats"].tolist())


@pytest.mark.parametrize("n", [1, 15, 16, 17, 4095, 4096 * 4 + 33, 3_000_001])
@pytest.mark.parametrize("offset", [0, 3])
def test_hamming_random_vs_oracle(gpu, oracle, n, offset):
    """Vector path, unaligned (byte-offset) views and ragged tails."""
    import kvecc
    rng = np.random.default_rng(n + offset)
    buf = rng.integers(0, 256, size=n + offset, dtype=np.int64).astype(np.uint8)
    x = _t(buf, gpu)[offset:]
    ref = buf[offset:]
    assert np.array_equal(_np(kvecc.hamming84_encode(x)), oracle.hamming84_encode(ref))
    assert np.array_equal(_np(kvecc.hamming74_encode(x)), oracle.hamming74_encode(ref))
    d, t, st = kvecc.hamming84_decode(x, return_error_types=True)
    od, ot, ost = oracle.hamming84_decode(ref)
    assert np.array_equal(_np(d), od) and np.array_equal(_np(t), ot) and st == ost
    d, f, st = kvecc.hamming74_decode(x, return_error_detected=True)
    od, of, ost = oracle.hamming74_decode(ref)
    assert np.array_equal(_np(d), od) and np.array_equal(_np(f), of) and st == ost


def test_hamming84_full_config_roundtrip(gpu):
    """BASELINE config 2 shape: encode -> decode is the identity, no errors."""
    import kvecc
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 16, (8, 4096, 32, 128), generator=g, dtype=torch.uint8).to(gpu)
    cw = kvecc.hamming84_encode(x)
    d, (c, det) = kvecc.hamming84_decode(cw)
    assert torch.equal(d, x) and c == 0 and det == 0
    # flip bit k of every codeword: singles everywhere, all corrected
    for k in (0, 5, 7):
        d, t, (c, det) = kvecc.hamming84_decode(cw ^ (1 << k), return_error_types=True)
        assert torch.equal(d, x)
        assert c == x.numel() if k < 7 else c == 0
        if k == 7:
            assert int((t == 3).sum()) == x.numel()


# ---------------------------------------------------------------------------
# Golay
# ---------------------------------------------------------------------------

def test_golay_golden(gpu, golden):
    import kvecc
    g = golden("golay")
    out = kvecc.golay_encode(_t(g["enc_in"], gpu))
    assert np.array_equal(_np(out), g["enc_out"])
    trip, cnt, st = kvecc.golay_decode(_t(g["dec_in"], gpu), return_error_counts=True)
    assert np.array_equal(_np(trip), g["dec_trip"])
    assert np.array_equal(_np(cnt), g["dec_count"])
    assert st == tuple(g["dec_stats"].tolist())


@pytest.mark.parametrize("m", [1, 5, 4095, 4096, 4097, 4096 * 7 + 1001, 1_000_003])
@pytest.mark.parametrize("offset", [0, 1])
def test_golay_random_vs_oracle(gpu, oracle, m, offset):
    import kvecc
    rng = np.random.default_rng(m * 7 + offset)
    trip = rng.integers(0, 256, size=(m + offset, 3), dtype=np.int64).astype(np.uint8)
    t = _t(trip, gpu)[offset:]
    cw = kvecc.golay_encode(t)
    ocw = oracle.golay_encode(trip[offset:])
    assert np.array_equal(_np(cw), ocw)
    # random 0..5 bit errors plus a few garbage words
    noisy = ocw.astype(np.int64)
    nerr = rng.integers(0, 6, size=m)
    for k in range(6):
        sel = nerr > k
        noisy[sel] ^= 1 << rng.integers(0, 24, size=int(sel.sum()))
    noisy[::97] = rng.integers(-(2**31), 2**31, size=noisy[::97].size)
    noisy = noisy.astype(np.int32)
    buf = np.concatenate([np.zeros(offset, np.int32), noisy])
    x = _t(buf, gpu)[offset:]
    d, c, st = kvecc.golay_decode(x, return_error_counts=True)
    od, oc, ost = oracle.golay_decode(noisy)
    assert np.array_equal(_np(d), od)
    assert np.array_equal(_np(c), oc)
    assert st == ost


@pytest.mark.parametrize("m", [4096 * 3 + 1, 8192 * 2 + 4095, 44_739_243 // 64])
@pytest.mark.parametrize("with_counts", [False, True])
@pytest.mark.parametrize("with_stats", [False, True])
def test_golay_tile_kernels_take_the_tail(gpu, oracle, m, with_counts, with_stats):
    """The tile kernels decode / encode the last m % tile codewords themselves
    (golay.hip), in every counts / statistics instance; lengths past whole
    decode (4096) and encode (8192) tiles, and 1/64 of config 3's flat M_f."""
    from kvecc import ops
    rng = np.random.default_rng(m + 2 * with_counts + with_stats)
    trip = rng.integers(0, 16, size=(m, 3), dtype=np.int64).astype(np.uint8)
    cw = torch.empty(m, dtype=torch.int32, device=gpu)
    ops.golay_encode_into(_t(trip, gpu).view(-1), cw, m)
    ocw = oracle.golay_encode(trip)
    assert np.array_equal(_np(cw), ocw)
    noisy = ocw.astype(np.int64) ^ (rng.random(m) < 0.3) * (1 << rng.integers(0, 24, size=m))
    noisy[::13] ^= 0x3 << 20  # a second (and third) error on some words
    noisy[::101] = rng.integers(0, 1 << 24, size=noisy[::101].size)
    noisy = noisy.astype(np.int32)
    out = torch.full((m * 3,), 0xEE, dtype=torch.uint8, device=gpu)
    counts = torch.full((m,), 0xEE, dtype=torch.uint8, device=gpu) if with_counts else None
    stats = ops.new_stats(gpu) if with_stats else None
    ops.golay_decode_into(_t(noisy, gpu), out, counts, stats)
    od, oc, ost = oracle.golay_decode(noisy)
    assert np.array_equal(_np(out).reshape(-1, 3), od)
    if with_counts:
        assert np.array_equal(_np(counts), oc)
    if with_stats:
        assert tuple(ops.read_stats(stats)) == tuple(ost)


def test_golay_full_config_roundtrip(gpu, oracle):
    """BASELINE config 3 shape with per-head packing: rows of 128 -> 43 codewords."""
    import kvecc
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 16, (8, 4096, 32, 128), generator=g, dtype=torch.uint8).to(gpu)
    cw = kvecc.ops.golay_encode_rows(x)
    assert cw.shape == (8, 4096, 32, 43)
    # sample rows against the oracle's padded triplet encode
    xs = x.view(-1, 128)[:: 997].cpu().numpy()
    pad = np.zeros((xs.shape[0], 129), np.uint8)
    pad[:, :128] = xs
    ref = oracle.golay_encode(pad.reshape(-1, 3)).reshape(-1, 43)
    assert np.array_equal(_np(cw.view(-1, 43)[:: 997]), ref)
    stats = kvecc.ops.new_stats(gpu)
    back = kvecc.ops.golay_decode_rows(cw, 128, stats)
    assert torch.equal(back, x) and kvecc.ops.read_stats(stats) == [0, 0]
    # flat triplet API on the padded layout gives the same codewords
    padded = torch.zeros(8, 4096, 32, 129, dtype=torch.uint8, device=gpu)
    padded[..., :128] = x
    cw2 = kvecc.golay_encode(padded.view(-1, 3))
    assert torch.equal(cw2, cw.view(-1))
    trip, (bits, unc) = kvecc.golay_decode(cw2)
    assert torch.equal(trip.view(8, 4096, 32, 129), padded) and bits == 0 and unc == 0


# ---------------------------------------------------------------------------
# Fault injection
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("tag", ["inject", "inject_vec"])
def test_inject_golden(gpu, golden, manifest, tag):
    import kvecc
    g = golden(tag)
    fn = (kvecc.inject_bit_errors_triton if tag == "inject"
          else kvecc.inject_bit_errors_triton_vectorized)
    for i, c in enumerate(manifest[tag]["params"]["cases"]):
        x = _t(g[f"c{i}_in"], gpu)
        out, st = fn(x, c["ber"], c["n_bits"], seed=c["seed"], return_stats=True)
        assert np.array_equal(_np(out), g[f"c{i}_out"]), (tag, c)
        assert st == tuple(g[f"c{i}_stats"].tolist()), (tag, c)


def test_inject_ber_zero_aliases_input(gpu):
    import kvecc
    x = torch.arange(100, dtype=torch.uint8, device=gpu)
    assert kvecc.inject_bit_errors_triton(x, 0.0, 8) is x
    with pytest.raises(ValueError):
        kvecc.inject_bit_errors_triton(x.float(), 0.1, 8)


@pytest.mark.parametrize("dtype,nb", [("u8", 8), ("u8", 7), ("u8", 4), ("i32", 24), ("u8", 5),
                                      ("i32", 11)])
def test_inject_random_vs_oracle(gpu, oracle, dtype, nb):
    import kvecc
    rng = np.random.default_rng(nb)
    n = 200_003
    if dtype == "u8":
        x = rng.integers(0, 256, size=n, dtype=np.int64).astype(np.uint8)
    else:
        x = rng.integers(-(2**31), 2**31, size=n, dtype=np.int64).astype(np.int32)
    for seed, ber in ((42, 1e-2), (2**30 + 5, 0.3), (0, 1e-3)):
        out, st = kvecc.inject_bit_errors_triton(_t(x, gpu), ber, nb, seed=seed, return_stats=True)
        o, _, ost = oracle.inject(x, ber, nb, seed)
        assert np.array_equal(_np(out), o) and st == ost, (seed, ber)


def test_inject_sharded_equals_flat(gpu):
    """Monte-Carlo sharding: (global_n, offset0) shards reproduce the flat run."""
    from kvecc import ops
    n = 1_000_000
    x = torch.randint(0, 2**24, (n,), dtype=torch.int32, device=gpu)
    full = torch.empty_like(x)
    st_full = ops.new_stats(gpu)
    ops.inject_into(x, full, 1e-2, 24, seed=42, stats=st_full)
    parts = torch.empty_like(x)
    st = ops.new_stats(gpu)
    bounds = [0, 123_457, 500_000, 999_999, n]
    for a, b in zip(bounds[:-1], bounds[1:]):
        ops.inject_into(x[a:b], parts[a:b], 1e-2, 24, seed=42, stats=st, global_n=n, offset0=a)
    assert torch.equal(full, parts) and ops.read_stats(st) == ops.read_stats(st_full)


def test_inject_full_config_sampled(gpu, oracle):
    """BASELINE config 2/3 sizes: sampled elements vs the oracle + BER fidelity."""
    import kvecc
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 16, (8, 4096, 32, 128), generator=g, dtype=torch.uint8).to(gpu)
    cw = kvecc.hamming84_encode(x)
    out, (flips, aff) = kvecc.inject_bit_errors_triton(cw, 1e-3, 8, seed=42, return_stats=True)
    n = cw.numel()
    assert abs(flips / (n * 8) - 1e-3) < 1e-5
    idx = np.random.default_rng(1).integers(0, n, size=3000)
    src = _np(cw.view(-1)[torch.from_numpy(idx).to(gpu)])
    got = _np(out.view(-1)[torch.from_numpy(idx).to(gpu)])
    for i, s, o in zip(idx, src, got):
        ref, _, _ = oracle.inject(np.array([s], np.uint8), 1e-3, 8, 42, global_n=n, offset0=int(i))
        assert ref[0] == o, i
    # Golay per-head layout, 24 bits per codeword at BER 1e-2
    cwg = kvecc.ops.golay_encode_rows(x).view(-1)
    outg, (fg, ag) = kvecc.inject_bit_errors_triton(cwg, 1e-2, 24, seed=42, return_stats=True)
    m = cwg.numel()
    assert abs(fg / (m * 24) - 1e-2) < 1e-4
    idx = np.random.default_rng(2).integers(0, m, size=2000)
    src = _np(cwg[torch.from_numpy(idx).to(gpu)])
    got = _np(outg[torch.from_numpy(idx).to(gpu)])
    for i, s, o in zip(idx, src, got):
        ref, _, _ = oracle.inject(np.array([s], np.int32), 1e-2, 24, 42, global_n=m, offset0=int(i))
        assert ref[0] == o, i


@pytest.mark.parametrize("dtype,row_len,nb", [("u8", 128, 8), ("u8", 64, 7), ("i32", 43, 24),
                                              ("u8", 64, 4)])
def test_inject_rows_vs_oracle(gpu, oracle, dtype, row_len, nb):
    """Shim per-row scheme: row r is its own call with seed_base + r, N = row_len."""
    from kvecc import ops
    rng = np.random.default_rng(row_len)
    rows = 300
    if dtype == "u8":
        x = rng.integers(0, 256, size=rows * row_len, dtype=np.int64).astype(np.uint8)
    else:
        x = rng.integers(0, 2**24, size=rows * row_len, dtype=np.int64).astype(np.int32)
    xt = _t(x, gpu)
    out = torch.empty_like(xt)
    st = ops.new_stats(gpu)
    ops.inject_rows_into(xt, out, rows, row_len, 0.05, nb, seed_base=1000, stats=st)
    ref = np.concatenate([oracle.inject(x[r * row_len:(r + 1) * row_len], 0.05, nb, 1000 + r)[0]
                          for r in range(rows)])
    assert np.array_equal(_np(out), ref)
    # in place
    ops.inject_rows_into(xt, xt, rows, row_len, 0.05, nb, seed_base=1000)
    assert np.array_equal(_np(xt), ref)


# ---------------------------------------------------------------------------
# Interpolation
# ---------------------------------------------------------------------------

def test_interp_golden(gpu, golden, manifest):
    import kvecc
    g = golden("interp")
    for i, c in enumerate(manifest["interp"]["params"]["cases"]):
        q = _t(g[f"c{i}_q"], gpu)
        e = _t(g[f"c{i}_err"], gpu)
        out = kvecc.interpolate_double_errors(q, e, seq_dim=c["seq_dim"])
        assert np.array_equal(_np(out), g[f"c{i}_out"]), c


@pytest.mark.parametrize("shape,seq_dim", [((1024, 12, 64), 0), ((37, 5, 48), 0),
                                           ((100, 7, 3), 0), ((4, 1000), -1), ((5000,), -1),
                                           ((3, 64, 16, 32), 1), ((2, 3, 4, 5), 2), ((1, 16, 16), 0)])
def test_interp_random_vs_oracle(gpu, oracle, shape, seq_dim):
    import kvecc
    rng = np.random.default_rng(len(shape))
    q = rng.integers(0, 16, size=shape, dtype=np.int64).astype(np.uint8)
    e = rng.choice(np.array([0, 1, 2, 3], np.uint8), size=shape, p=[0.6, 0.1, 0.25, 0.05])
    out = kvecc.interpolate_double_errors(_t(q, gpu), _t(e, gpu), seq_dim=seq_dim)
    assert np.array_equal(_np(out), oracle.interpolate_double_errors(q, e, seq_dim=seq_dim))


def test_interp_fast_path_keeps_values(gpu):
    import kvecc
    q = torch.tensor([200, 17, 3, 99], dtype=torch.uint8, device=gpu)
    e = torch.tensor([0, 1, 3, 0], dtype=torch.uint8, device=gpu)
    assert torch.equal(kvecc.interpolate_double_errors(q, e), q)
    e[1] = 2
    assert kvecc.interpolate_double_errors(q, e).tolist() == [15, 15, 3, 15]


def test_interp_vector_gate_pass(gpu):
    """No double errors: the vector path's device gate copies q unchanged (no clamp)."""
    import kvecc
    g = torch.Generator().manual_seed(4)
    q = torch.randint(0, 256, (16, 64, 48), generator=g, dtype=torch.uint8)
    e = torch.randint(0, 2, (16, 64, 48), generator=g, dtype=torch.uint8) * 3  # 0 or 3
    out = kvecc.interpolate_double_errors(q.to(gpu), e.to(gpu), seq_dim=1)
    assert torch.equal(out.cpu(), q)


@pytest.mark.parametrize("shape,seq_dim", [((64, 32, 128), 0), ((8, 40, 48), 1), ((999,), -1),
                                           ((5, 33, 7), 1)])
@pytest.mark.parametrize("case", ["none", "none_over15", "one_double_far", "double_and_over15"])
def test_interp_auto_flags_and_fixup(gpu, oracle, shape, seq_dim, case):
    """kvecc_interpolate_auto: one pass + the trailing copy give the reference's
    result in every branch (vector and scalar layouts); flags = (any double, any q > 15)."""
    from kvecc import ops
    rng = np.random.default_rng(sum(shape))
    q = rng.integers(0, 16, size=shape, dtype=np.int64).astype(np.uint8)
    e = rng.choice(np.array([0, 1, 3], np.uint8), size=shape)
    flat_q, flat_e = q.reshape(-1), e.reshape(-1)
    if case in ("none_over15", "double_and_over15"):
        flat_q[rng.integers(0, flat_q.size, 5)] = 200
    if case in ("one_double_far", "double_and_over15"):
        flat_e[flat_e.size - 1] = 2
    qd, ed = _t(q, gpu), _t(e, gpu)
    outer, length, inner = ops._seq_layout(shape, seq_dim)
    out = torch.empty(q.size, dtype=torch.uint8, device=gpu)
    flags, epoch = ops.interpolate_auto_into(qd.view(-1), ed.view(-1), out, outer, length, inner)
    want_flags = [int((e == 2).any()), int((q > 15).any())]
    assert (flags == epoch).int().tolist() == want_flags
    assert np.array_equal(_np(out).reshape(shape), oracle.interpolate_double_errors(q, e, seq_dim=seq_dim))
    if not want_flags[0]:
        assert np.array_equal(_np(out).reshape(shape), q)


def test_interp_auto_epochs_do_not_leak(gpu):
    """Consecutive calls share the flag words: a double seen by one call must not
    gate the next (each call stamps a fresh epoch instead of zeroing)."""
    import kvecc
    q = torch.full((64, 48), 200, dtype=torch.uint8, device=gpu)
    e_dbl = torch.zeros_like(q)
    e_dbl[5, 7] = 2
    e_none = torch.zeros_like(q)
    for _ in range(3):
        assert int(kvecc.interpolate_double_errors(q, e_dbl, seq_dim=0).max()) == 15
        assert torch.equal(kvecc.interpolate_double_errors(q, e_none, seq_dim=0), q)


@pytest.mark.parametrize("n,offset", [(1, 0), (17, 3), ((1 << 20) + 5, 0), ((1 << 22) + 77, 1)])
def test_any_equal(gpu, n, offset):
    from kvecc import ops
    g = torch.Generator().manual_seed(n)
    base = torch.randint(0, 2, (n + offset,), generator=g, dtype=torch.uint8)  # values 0/1
    x = base.to(gpu)[offset:]
    assert int(ops.any_equal(x, 2)) == 0
    for pos in (0, n // 2, n - 1):
        y = x.clone()
        y[pos] = 2
        assert int(ops.any_equal(y, 2)) == 1, pos


# ---------------------------------------------------------------------------
# Fused quantize/encode, decode/dequantize
# ---------------------------------------------------------------------------

def test_fused_golden(gpu, golden, manifest):
    import kvecc
    g = golden("fused")
    for i, c in enumerate(manifest["fused"]["params"]["cases"]):
        x = _t(g[f"c{i}_x"], gpu)
        # fixtures from the reference on CPU tensors: the IEEE scale rule
        cw, s = kvecc.fused_quantize_encode_hamming84(x, scale_rule="div7")
        assert np.array_equal(_np(cw), g[f"c{i}_cw84"]) and np.array_equal(_np(s), g[f"c{i}_s84"])
        cw, s = kvecc.fused_quantize_encode_hamming74(x, scale_rule="div7")
        assert np.array_equal(_np(cw), g[f"c{i}_cw74"])
        out, nc = kvecc.fused_decode_dequantize_hamming84(_t(g[f"c{i}_cw_noisy"], gpu),
                                                          _t(g[f"c{i}_s84"], gpu))
        assert np.array_equal(_np(out), g[f"c{i}_dq"]) and nc == int(g[f"c{i}_ncorr"][0])


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(4096, 128), (333, 64), (17, 100), (5, 7), (2, 3, 256)])
def test_quantize_vs_torch_path(gpu, oracle, dtype, shape):
    """Exactly the shim's torch rounding (ecc_shim.py:572-580) for every dtype,
    under both scale rules; the default is the reference's own expression
    `abs_max / 7.0` (paged_cache_ecc.py:330) evaluated by torch on the GPU."""
    import kvecc
    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.randn(*shape, generator=g) * 3).to(dtype)
    x.view(-1, shape[-1])[0] = 0
    xd = x.to(gpu)
    for rule, code in (("div7", 0), ("mul_inv7", 1)):
        q, s = kvecc.ops.quantize_rows(xd, scale_rule=rule)
        oq, os_ = oracle.quantize_rows(x.float().numpy(), rule=code)
        assert np.array_equal(_np(q), oq) and np.array_equal(_np(s), os_), rule
    q, s = kvecc.ops.quantize_rows(xd)
    ref = xd.float().abs().amax(-1) / 7.0
    ref = torch.where(ref == 0, torch.ones_like(ref), ref)
    ref_q = (torch.round(xd.float() / ref.unsqueeze(-1)).clamp(-8, 7) + 8).to(torch.uint8)
    assert torch.equal(s, ref) and torch.equal(q, ref_q) and np.array_equal(_np(q), oq)
    cw, s84 = kvecc.fused_quantize_encode_hamming84(xd)
    assert np.array_equal(_np(cw), oracle.hamming84_encode(oq))
    # decode + dequant to the input dtype (== torch .to(dtype) of the fp32 result)
    out, nc = kvecc.fused_decode_dequantize_hamming84(cw, s84, output_dtype=dtype)
    ref, _ = oracle.decode_dequant_h84(oracle.hamming84_encode(oq), os_)
    assert torch.equal(out.cpu(), torch.from_numpy(ref).to(dtype)) and nc == 0


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(4096, 128), (100, 64), (9, 48), (3, 20)])
def test_decode_dequant_noisy_vs_cpu_backend(gpu, dtype, shape):
    """Noisy codewords (singles corrected, doubles zeroed) equal the host backend."""
    import kvecc
    from kvecc import cpu_ops
    g = torch.Generator().manual_seed(shape[0])
    x = torch.randn(*shape, generator=g) * 2
    cw, s = cpu_ops.fused_quantize_encode_hamming84(x)
    noisy = cpu_ops.inject_bit_errors_triton(cw, 0.03, 8, seed=5)
    ref, nc_ref = cpu_ops.fused_decode_dequantize_hamming84(noisy, s, output_dtype=dtype)
    out, nc = kvecc.fused_decode_dequantize_hamming84(noisy.to(gpu), s.to(gpu), output_dtype=dtype)
    assert nc == nc_ref and nc > 0
    assert torch.equal(out.cpu(), ref)


# ---------------------------------------------------------------------------
# Full BASELINE sizes: HIP backend vs the host backend (chain of trust: the
# host backend is pinned to the golden vectors in tests/test_cpu_backend.py)
# ---------------------------------------------------------------------------

def test_config2_full_size_vs_cpu_backend(gpu):
    """Config 2: H84 encode + inject(BER 1e-3) + decode on [8,4096,32,128]."""
    import kvecc
    from kvecc import cpu_ops
    g = torch.Generator().manual_seed(2)
    x = torch.randint(0, 16, (8, 4096, 32, 128), dtype=torch.uint8, generator=g)
    cw_h = cpu_ops.hamming84_encode(x)
    noisy_h, st_h = cpu_ops.inject_bit_errors_triton(cw_h, 1e-3, 8, seed=7, return_stats=True)
    dec_h, et_h, dst_h = cpu_ops.hamming84_decode(noisy_h, return_error_types=True)
    cw = kvecc.hamming84_encode(x.to(gpu))
    assert torch.equal(cw.cpu(), cw_h)
    noisy, st = kvecc.inject_bit_errors_triton(cw, 1e-3, 8, seed=7, return_stats=True)
    assert st == st_h and torch.equal(noisy.cpu(), noisy_h)
    dec, et, dst = kvecc.hamming84_decode(noisy, return_error_types=True)
    assert dst == dst_h
    assert torch.equal(dec.cpu(), dec_h) and torch.equal(et.cpu(), et_h)


def test_config3_full_size_vs_cpu_backend(gpu):
    """Config 3: Golay triplets of [8,4096,32,128] (per-head padding, 43 cw/head),
    inject(BER 1e-2, 24 bits) + decode."""
    import kvecc
    from kvecc import cpu_ops, ops
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 16, (8, 4096, 32, 128), dtype=torch.uint8, generator=g)
    cw_h = cpu_ops.golay_encode_rows(x).reshape(-1)
    noisy_h, st_h = cpu_ops.inject_bit_errors_triton(cw_h, 1e-2, 24, seed=11, return_stats=True)
    trip_h, cnt_h, dst_h = cpu_ops.golay_decode(noisy_h, return_error_counts=True)
    cw = ops.golay_encode_rows(x.to(gpu)).reshape(-1)
    assert torch.equal(cw.cpu(), cw_h)
    noisy, st = kvecc.inject_bit_errors_triton(cw, 1e-2, 24, seed=11, return_stats=True)
    assert st == st_h and torch.equal(noisy.cpu(), noisy_h)
    trip, cnt, dst = kvecc.golay_decode(noisy, return_error_counts=True)
    assert dst == dst_h
    assert torch.equal(trip.cpu(), trip_h) and torch.equal(cnt.cpu(), cnt_h)


@pytest.mark.parametrize("m", [1, 7, 8, 9, 8192 * 2, 8192 * 2 + 5, 45_088_768])
@pytest.mark.parametrize("offset", [0, 1])
def test_golay_packed_vs_cpu_backend(gpu, m, offset):
    """Packed Golay storage: HIP == host backend (which tests pin to the reference
    layout), including the tail path, unaligned buffers and the full config-3 M."""
    if offset and m > 100_000:
        pytest.skip("unaligned full size adds nothing over the small cases")
    from kvecc import cpu_ops, ops
    g = torch.Generator().manual_seed(m + offset)
    nib = torch.randint(0, 256, ((3 * m + 1) // 2 + offset,), generator=g, dtype=torch.uint8)
    nib_h = nib[offset:].contiguous() if offset == 0 else nib[offset:]
    cw3_ref = cpu_ops.golay_encode_packed(nib_h, m)
    nib_d = nib.to(gpu)[offset:]
    cw3 = ops.golay_encode_packed(nib_d, m)
    assert torch.equal(cw3.cpu(), cw3_ref)
    noisy = cpu_ops.inject_bit_errors_triton(cw3_ref, 0.03, 8, seed=9)  # byte-level corruption
    out_ref, fl_ref, st_ref = cpu_ops.golay_decode_packed(noisy, m, return_uncorrectable=True)
    buf = torch.zeros(3 * m + offset, dtype=torch.uint8)
    buf[offset:] = noisy
    out, fl, st = ops.golay_decode_packed(buf.to(gpu)[offset:], m, return_uncorrectable=True)
    assert st == st_ref and st_ref[0] > 0
    assert torch.equal(out.cpu(), out_ref) and torch.equal(fl.cpu(), fl_ref)


@pytest.mark.parametrize("foff", [0, 1, 4, 16])
def test_golay_packed_decode_flag_buffer_offsets(gpu, foff):
    """Caller flag buffers at any byte offset (a KVECC_PACKED_DEC_FLAGS16 build
    stages 16-byte aligned ones through LDS) equal the host backend, and the
    bytes around the flags stay untouched."""
    from kvecc import cpu_ops, ops
    m = 8192 * 6 + 13  # whole wave tiles plus a tail
    g = torch.Generator().manual_seed(77 + foff)
    nib = torch.randint(0, 256, ((3 * m + 1) // 2,), generator=g, dtype=torch.uint8)
    noisy = cpu_ops.inject_bit_errors_triton(cpu_ops.golay_encode_packed(nib, m), 0.05, 8, seed=3)
    out_ref, fl_ref, st_ref = cpu_ops.golay_decode_packed(noisy, m, return_uncorrectable=True)
    nf = (m + 7) // 8
    fbuf = torch.full((nf + foff + 32,), 0xA5, dtype=torch.uint8, device=gpu)
    nib_out = torch.empty((3 * m + 1) // 2, dtype=torch.uint8, device=gpu)
    st = ops.new_stats(gpu)
    ops.golay_decode_packed_into(noisy.to(gpu), nib_out, fbuf[foff:foff + nf], m, st)
    f = fbuf.cpu()
    assert fl_ref.sum() > 0 and torch.equal(f[foff:foff + nf], fl_ref)
    assert bool((f[:foff] == 0xA5).all()) and bool((f[foff + nf:] == 0xA5).all())
    assert torch.equal(nib_out.cpu(), out_ref) and tuple(ops.read_stats(st)) == tuple(st_ref)
    with pytest.raises(ValueError):  # a flag buffer one byte short is refused, not overrun
        ops.golay_decode_packed_into(noisy.to(gpu), nib_out, fbuf[:nf - 1], m, st)


@pytest.mark.parametrize("n", [1, 15, 16, 17, 16 * 1000 + 9, 134_217_728])
@pytest.mark.parametrize("offset", [0, 1])
def test_hamming84_packed_vs_cpu_backend(gpu, n, offset):
    if offset and n > 100_000:
        pytest.skip("unaligned full size adds nothing over the small cases")
    from kvecc import cpu_ops, ops
    g = torch.Generator().manual_seed(n + offset)
    nib = torch.randint(0, 256, ((n + 1) // 2 + offset,), generator=g, dtype=torch.uint8)
    cw_ref = cpu_ops.hamming84_encode_packed(nib[offset:], n)
    cw = ops.hamming84_encode_packed(nib.to(gpu)[offset:], n)
    assert torch.equal(cw.cpu(), cw_ref)
    noisy = cpu_ops.inject_bit_errors_triton(cw_ref, 0.02, 8, seed=6)
    pn_ref, pt_ref, st_ref = cpu_ops.hamming84_decode_packed(noisy, return_error_types=True)
    buf = torch.zeros(n + offset, dtype=torch.uint8)
    buf[offset:] = noisy
    pn, pt, st = ops.hamming84_decode_packed(buf.to(gpu)[offset:], return_error_types=True)
    assert st == st_ref
    assert torch.equal(pn.cpu(), pn_ref) and torch.equal(pt.cpu(), pt_ref)


def test_time_next_launch_stamps_one_kernel(gpu):
    """kvecc_time_next_launch: the next launch carries the events (its own start
    and end), the hook then disarms, and results are unchanged."""
    from kvecc import ops
    x = torch.randint(0, 16, (1 << 24,), dtype=torch.uint8, device=gpu)
    ref = ops.hamming84_encode(x)
    out = torch.empty_like(x)
    start, stop = ops.kernel_timer(gpu)
    ops.time_next_launch(start, stop)
    ops.hamming84_encode_into(x, out)
    torch.cuda.synchronize()
    t1 = start.elapsed_time(stop)
    assert torch.equal(out, ref) and 0.0 < t1 < 50.0
    ops.hamming84_encode_into(x, out)  # disarmed: the events keep their stamps
    torch.cuda.synchronize()
    assert start.elapsed_time(stop) == t1


@pytest.mark.parametrize("d", [1, 2, 5, 46, 47, 48, 64, 96, 100, 127, 128, 129, 255, 256, 300, 511, 512, 513])
@pytest.mark.parametrize("rows,offset", [(1, 0), (63, 0), (64, 0), (65, 1), (1000, 0), (1000, 3)])
def test_golay_rows_vs_cpu_backend(gpu, d, rows, offset):
    """Per-head packing (ecc_shim.py:623-682): the wave-tiled LDS kernels (46 <= d <= 512:
    full and partial wave tiles, aligned and unaligned buffers) and the
    per-codeword kernels (short rows, d = 511 and 513) against the host twin, encode and a
    noisy decode."""
    from kvecc import cpu_ops, ops
    g = torch.Generator().manual_seed(d * 1009 + rows)
    base = torch.randint(0, 16, (rows * d + offset,), generator=g, dtype=torch.uint8)
    x = base[offset:].view(rows, d)
    cw = ops.golay_encode_rows(base.to(gpu)[offset:].view(rows, d))
    ref = cpu_ops.golay_encode_rows(x)
    assert torch.equal(cw.cpu(), ref)
    noisy = ref.clone().view(-1)
    flips = torch.randint(0, 1 << 24, noisy.shape, generator=g, dtype=torch.int32)
    mask = torch.rand(noisy.shape, generator=g) < 0.3
    flips &= torch.randint(0, 1 << 24, noisy.shape, generator=g, dtype=torch.int32)  # ~6 bits each
    noisy[mask] ^= flips[mask]
    noisy = noisy.view(rows, -1)
    cbuf = torch.zeros(noisy.numel() + offset, dtype=torch.int32)
    cbuf[offset:] = noisy.view(-1)
    st, cst = ops.new_stats(gpu), cpu_ops.new_stats()
    out = ops.golay_decode_rows(cbuf.to(gpu)[offset:].view(rows, -1), d, st)
    want = cpu_ops.golay_decode_rows(noisy, d, cst)
    assert torch.equal(out.cpu(), want)
    assert ops.read_stats(st) == cpu_ops.read_stats(cst)


def test_interp_auto_in_a_hip_graph(gpu):
    """A captured interpolate_double_errors replays correctly with inputs that
    alternate between 'has doubles' and 'no doubles, q > 15' (the flag words
    are re-zeroed inside the graph, not epoch-stamped)."""
    import kvecc
    q = torch.full((64, 48), 200, dtype=torch.uint8, device=gpu)
    e = torch.zeros_like(q)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        kvecc.interpolate_double_errors(q, e, seq_dim=0)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = kvecc.interpolate_double_errors(q, e, seq_dim=0)
    for has_double in (True, False, True, False):
        e.zero_()
        if has_double:
            e[5, 7] = 2
        graph.replay()
        torch.cuda.synchronize()
        if has_double:
            assert int(out.max()) == 15
        else:
            assert torch.equal(out, q)


@pytest.mark.parametrize("n,offset", [(1, 0), (15, 0), (16, 0), (1 << 20, 0), ((1 << 20) + 37, 3),
                                      (134217728 + 5, 0)])
def test_count_ne_vs_torch(gpu, n, offset):
    """kvecc_count_ne_u8 (the sweep's residual count) equals (a != b).sum():
    vector and tail paths, unaligned buffers, a [8,4096,32,128]-sized input."""
    from kvecc import ops
    g = torch.Generator(device=gpu).manual_seed(n)
    a = torch.randint(0, 256, (n + offset,), dtype=torch.uint8, device=gpu, generator=g)[offset:]
    b = a.clone()
    flips = torch.randint(0, n, (max(1, n // 100),), device=gpu, generator=g)
    b[flips] ^= 0x40
    st = ops.new_stats(gpu)
    ops.count_ne_into(a, b, st)
    assert ops.read_stats(st, 1)[0] == int((a != b).sum())


# ---------------------------------------------------------------------------
# Full BASELINE sizes anchored to the C oracle itself (not only to the host
# backend, which shares codec_math.h with the kernels): the oracle is pinned to
# the reference-generated golden vectors (tests/test_oracle.py).  The oracle is
# single-threaded; the flat tensor is cut into shards that carry the full
# tensor's global_n / offset0, run on 16 host threads (ctypes drops the GIL).
# ---------------------------------------------------------------------------

def _oracle_sharded(fn, arrays, n, parts=64, threads=16):
    """fn(lo, hi) -> tuple of numpy outputs for elements [lo, hi); concatenated."""
    from concurrent.futures import ThreadPoolExecutor
    bounds = [(n * k // parts, n * (k + 1) // parts) for k in range(parts)]
    with ThreadPoolExecutor(threads) as pool:
        res = list(pool.map(lambda b: fn(*b), bounds))
    return res


def test_config2_full_size_vs_oracle(gpu, oracle):
    """Config 2 at [8,4096,32,128]: H(8,4) encode -> inject(BER 1e-3, 8 bits, the
    flat tensor's Philox stream) -> decode, HIP against the C oracle bit for bit."""
    import numpy as np

    import kvecc
    g = torch.Generator().manual_seed(21)
    x = torch.randint(0, 16, (8, 4096, 32, 128), dtype=torch.uint8, generator=g)
    n = x.numel()
    xn = x.numpy().reshape(-1)
    cw = kvecc.hamming84_encode(x.to(gpu))
    noisy, st = kvecc.inject_bit_errors_triton(cw, 1e-3, 8, seed=42, return_stats=True)
    dec, et, dst = kvecc.hamming84_decode(noisy, return_error_types=True)

    def shard(lo, hi):
        c = oracle.hamming84_encode(xn[lo:hi])
        nz, _, s = oracle.inject(c, 1e-3, 8, 42, global_n=n, offset0=lo)
        d, e, ds = oracle.hamming84_decode(nz)
        return c, nz, s, d, e, ds

    res = _oracle_sharded(shard, None, n)
    cat = lambda k: np.concatenate([r[k] for r in res])  # noqa: E731
    assert np.array_equal(cw.cpu().numpy().reshape(-1), cat(0))
    assert np.array_equal(noisy.cpu().numpy().reshape(-1), cat(1))
    assert st == tuple(sum(r[2][k] for r in res) for k in range(2))
    assert np.array_equal(dec.cpu().numpy().reshape(-1), cat(3))
    assert np.array_equal(et.cpu().numpy().reshape(-1), cat(4))
    assert dst == tuple(sum(r[5][k] for r in res) for k in range(2)) and dst[0] > 0 and dst[1] > 0


def test_config3_full_size_vs_oracle(gpu, oracle):
    """Config 3 at [8,4096,32,128]: per-head padded Golay triplets (43 codewords
    per head, M_h = 45,088,768) -> inject(BER 1e-2, 24 bits) -> decode, HIP
    (the headline's kernels) against the C oracle bit for bit."""
    import numpy as np

    from kvecc import ops
    g = torch.Generator().manual_seed(31)
    x = torch.randint(0, 16, (8, 4096, 32, 128), dtype=torch.uint8, generator=g)
    trip = torch.zeros(8, 4096, 32, 129, dtype=torch.uint8)
    trip[..., :128] = x
    trip = trip.view(-1, 3)
    m = trip.shape[0]
    tn = trip.numpy()
    d_trip = trip.to(gpu)
    cw = torch.empty(m, dtype=torch.int32, device=gpu)
    ops.golay_encode_into(d_trip.view(-1), cw, m)
    noisy = torch.empty_like(cw)
    ist = ops.new_stats(gpu)
    ops.inject_into(cw, noisy, 1e-2, 24, seed=42, stats=ist)
    out = torch.empty(m * 3, dtype=torch.uint8, device=gpu)
    cnt = torch.empty(m, dtype=torch.uint8, device=gpu)
    dst = ops.new_stats(gpu)
    ops.golay_decode_into(noisy, out, cnt, dst)

    def shard(lo, hi):
        c = oracle.golay_encode(tn[lo:hi])
        nz, _, s = oracle.inject(c, 1e-2, 24, 42, global_n=m, offset0=lo)
        t, k, ds = oracle.golay_decode(nz)
        return c, nz, s, t, k, ds

    res = _oracle_sharded(shard, None, m)
    cat = lambda k: np.concatenate([r[k] for r in res])  # noqa: E731
    assert np.array_equal(cw.cpu().numpy(), cat(0))
    assert np.array_equal(noisy.cpu().numpy(), cat(1))
    assert ops.read_stats(ist) == [sum(r[2][k] for r in res) for k in range(2)]
    assert np.array_equal(out.cpu().numpy().reshape(-1, 3), cat(3))
    assert np.array_equal(cnt.cpu().numpy(), cat(4))
    exp = [sum(r[5][k] for r in res) for k in range(2)]
    assert ops.read_stats(dst) == exp and exp[0] > 0 and exp[1] > 0
