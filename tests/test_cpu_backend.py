"""The host ("cpu") codec backend (BASELINE config 1) against the golden
vectors and the oracle.  CPU-only: needs libkvecc.so, not a GPU.

The backend runs the kvecc_cpu_* entry points, i.e. the same codec algebra
(csrc/codec_math.h) the gfx950 kernels are compiled from, so these tests also
pin that shared algebra without a GPU.
"""

import numpy as np
import pytest
import torch


@pytest.fixture(scope="module")
def cpu():
    from kvecc.backends import get_codec_backend
    return get_codec_backend("cpu")


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def test_registry_resolves_cpu(cpu):
    from kvecc import backends
    assert cpu.__name__ == "kvecc.cpu_ops"
    assert "cpu" in backends.available_backends()
    assert all(hasattr(cpu, f) for f in backends.FUNCTIONS)


def test_rejects_device_tensors(cpu):
    x = torch.zeros(4, dtype=torch.uint8, device="meta")
    with pytest.raises(AssertionError):
        cpu.hamming84_encode(x)


def test_config1_hamming74_plumbing(cpu):
    """BASELINE config 1: Hamming(7,4) encode/decode, [1,128,1,64], BER=0."""
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 16, (1, 128, 1, 64), dtype=torch.uint8, generator=g)
    cw = cpu.hamming74_encode(x)
    assert cw.shape == x.shape and cw.dtype == torch.uint8
    noisy = cpu.inject_bit_errors_triton(cw, 0.0, 7, seed=0)
    assert noisy is cw
    dec, flag, (n,) = cpu.hamming74_decode(noisy, return_error_detected=True)
    assert torch.equal(dec, x) and n == 0 and int(flag.sum()) == 0


def test_hamming_all_bytes(cpu, golden):
    g = golden("hamming")
    x = T(g["inputs"])
    assert np.array_equal(cpu.hamming74_encode(x).numpy(), g["enc74"])
    assert np.array_equal(cpu.hamming84_encode(x).numpy(), g["enc84"])
    d, f, st = cpu.hamming74_decode(x, return_error_detected=True)
    assert np.array_equal(d.numpy(), g["dec74_data"]) and np.array_equal(f.numpy(), g["dec74_flag"])
    assert st == tuple(g["dec74_stats"].tolist())
    d, t, st = cpu.hamming84_decode(x, return_error_types=True)
    assert np.array_equal(d.numpy(), g["dec84_data"]) and np.array_equal(t.numpy(), g["dec84_type"])
    assert st == tuple(g["dec84_stats"].tolist())


@pytest.mark.parametrize("threads", [1, 3, 0])
def test_hamming_random_vs_oracle(cpu, oracle, threads):
    """Ragged sizes (word tails, thread-chunk edges) against the oracle."""
    saved = cpu.NUM_THREADS
    cpu.set_num_threads(threads)
    try:
        rng = np.random.default_rng(11)
        for n in (1, 3, 5, 67, 1 << 17, (1 << 18) + 3):
            x = rng.integers(0, 256, n, dtype=np.uint8)
            for enc, dec in (("hamming74_encode", "hamming74_decode"),
                             ("hamming84_encode", "hamming84_decode")):
                assert np.array_equal(getattr(cpu, enc)(T(x)).numpy(), getattr(oracle, enc)(x))
                ref = getattr(oracle, dec)(x)
                got = getattr(cpu, dec)(T(x), True)
                assert np.array_equal(got[0].numpy(), ref[0])
                assert np.array_equal(got[1].numpy(), ref[1])
                assert tuple(got[2]) == tuple(ref[2])
    finally:
        cpu.set_num_threads(saved)


def test_golay_golden(cpu, golden):
    g = golden("golay")
    assert np.array_equal(cpu.golay_encode(T(g["enc_in"])).numpy(), g["enc_out"])
    trip, cnt, st = cpu.golay_decode(T(g["dec_in"]), return_error_counts=True)
    assert np.array_equal(trip.numpy(), g["dec_trip"])
    assert np.array_equal(cnt.numpy(), g["dec_count"])
    assert st == tuple(g["dec_stats"].tolist())


def test_golay_rows_roundtrip(cpu):
    g = torch.Generator().manual_seed(5)
    for d in (128, 64, 7, 1):
        x = torch.randint(0, 16, (3, 5, d), dtype=torch.uint8, generator=g)
        cw = cpu.golay_encode_rows(x)
        assert cw.shape == (3, 5, (d + 2) // 3)
        st = torch.zeros(2, dtype=torch.int64)
        assert torch.equal(cpu.golay_decode_rows(cw, d, st), x)
        assert st.tolist() == [0, 0]


@pytest.mark.parametrize("tag", ["inject"])
def test_inject_golden(cpu, golden, manifest, tag):
    g = golden(tag)
    for i, c in enumerate(manifest[tag]["params"]["cases"]):
        x = T(g[f"c{i}_in"])
        out, st = cpu.inject_bit_errors_triton(x, c["ber"], c["n_bits"], c["seed"],
                                               return_stats=True)
        if c["ber"] > 0:
            assert np.array_equal(out.numpy(), g[f"c{i}_out"]), c
            assert st == tuple(g[f"c{i}_stats"].tolist()), c


def test_inject_shards_match_flat(cpu):
    rng = np.random.default_rng(3)
    x = T(rng.integers(0, 2**24, size=30000).astype(np.int32))
    full = cpu.inject_bit_errors_triton(x, 0.05, 24, seed=42)
    parts = []
    for a, b in ((0, 10000), (10000, 25000), (25000, 30000)):
        out = torch.empty(b - a, dtype=torch.int32)
        cpu.inject_into(x[a:b].contiguous(), out, 0.05, 24, 42, global_n=30000, offset0=a)
        parts.append(out)
    assert torch.equal(torch.cat(parts), full)
    with pytest.raises(Exception):
        cpu.inject_into(x[:10], torch.empty(10, dtype=torch.int32), 0.05, 24, 42, global_n=5)


def test_interp_golden(cpu, golden, manifest):
    g = golden("interp")
    for i, c in enumerate(manifest["interp"]["params"]["cases"]):
        out = cpu.interpolate_double_errors(T(g[f"c{i}_q"]), T(g[f"c{i}_err"]), seq_dim=c["seq_dim"])
        assert np.array_equal(out.numpy(), g[f"c{i}_out"]), c


def test_interp_random_vs_oracle(cpu, oracle):
    rng = np.random.default_rng(9)
    for shape, sd in (((33, 70), -1), ((17, 4, 48), 0), ((5, 9, 3, 16), 1), ((4000,), 0)):
        q = rng.integers(0, 16, shape, dtype=np.uint8)
        e = rng.choice(np.array([0, 1, 2], np.uint8), shape, p=[0.8, 0.1, 0.1])
        ref = oracle.interpolate_double_errors(q, e, seq_dim=sd)
        assert np.array_equal(cpu.interpolate_double_errors(T(q), T(e), seq_dim=sd).numpy(), ref)


def test_fused_golden(cpu, golden, manifest):
    g = golden("fused")
    for i, c in enumerate(manifest["fused"]["params"]["cases"]):
        x = T(g[f"c{i}_x"])
        q, s = cpu.quantize_rows(x)
        assert np.array_equal(q.numpy(), g[f"c{i}_torch_q"]), c
        assert np.array_equal(s.numpy(), g[f"c{i}_torch_scale"]), c
        cw, s84 = cpu.fused_quantize_encode_hamming84(x)
        assert np.array_equal(cw.numpy(), g[f"c{i}_cw84"])
        cw, _ = cpu.fused_quantize_encode_hamming74(x)
        assert np.array_equal(cw.numpy(), g[f"c{i}_cw74"])
        dq, nc = cpu.fused_decode_dequantize_hamming84(T(g[f"c{i}_cw_noisy"]), T(g[f"c{i}_s84"]))
        assert np.array_equal(dq.numpy(), g[f"c{i}_dq"]), c
        assert nc == int(g[f"c{i}_ncorr"][0])


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fused_low_precision(cpu, dtype):
    """fp16/bf16 inputs quantize like their exact fp32 upcast; outputs round once."""
    g = torch.Generator().manual_seed(2)
    x = (torch.randn(50, 128, generator=g) * 3).to(dtype)
    cw, s = cpu.fused_quantize_encode_hamming84(x)
    cw32, s32 = cpu.fused_quantize_encode_hamming84(x.float())
    assert torch.equal(cw, cw32) and torch.equal(s, s32)
    dq, _ = cpu.fused_decode_dequantize_hamming84(cw, s, output_dtype=dtype)
    dq32, _ = cpu.fused_decode_dequantize_hamming84(cw, s, output_dtype=torch.float32)
    assert dq.dtype == dtype and torch.equal(dq, dq32.to(dtype))


def test_inject_vectorized_golden(cpu, golden, manifest):
    g = golden("inject_vec")
    for i, c in enumerate(manifest["inject_vec"]["params"]["cases"]):
        x = T(g[f"c{i}_in"])
        out, st = cpu.inject_bit_errors_triton_vectorized(x, c["ber"], c["n_bits"], c["seed"],
                                                          return_stats=True)
        if c["ber"] > 0:
            assert np.array_equal(out.numpy(), g[f"c{i}_out"]), c
            assert st == tuple(g[f"c{i}_stats"].tolist()), c


@pytest.mark.parametrize("dtype,row_len,nb", [("u8", 128, 8), ("u8", 64, 7), ("i32", 43, 24),
                                              ("u8", 64, 4)])
def test_inject_rows_vs_oracle(cpu, oracle, dtype, row_len, nb):
    """Shim per-row scheme: row r is its own call with seed_base + r, N = row_len."""
    rng = np.random.default_rng(row_len)
    rows = 200
    if dtype == "u8":
        x = rng.integers(0, 256, size=rows * row_len, dtype=np.int64).astype(np.uint8)
    else:
        x = rng.integers(0, 2**24, size=rows * row_len, dtype=np.int64).astype(np.int32)
    xt = T(x)
    out = torch.empty_like(xt)
    st = cpu.new_stats()
    cpu.inject_rows_into(xt, out, rows, row_len, 0.05, nb, seed_base=1000, stats=st)
    refs = [oracle.inject(x[r * row_len:(r + 1) * row_len], 0.05, nb, 1000 + r) for r in range(rows)]
    assert np.array_equal(out.numpy(), np.concatenate([r[0] for r in refs]))
    assert cpu.read_stats(st) == [sum(r[2][0] for r in refs), sum(r[2][1] for r in refs)]
    cpu.inject_rows_into(xt, xt, rows, row_len, 0.05, nb, seed_base=1000)  # in place
    assert np.array_equal(xt.numpy(), out.numpy())


def test_golay_rows_vs_flat(cpu):
    """Row packing equals explicit zero padding + flat encode; decode stats add up."""
    g = torch.Generator().manual_seed(8)
    for d in (128, 100, 64, 5):
        x = torch.randint(0, 16, (7, 3, d), dtype=torch.uint8, generator=g)
        gs = (d + 2) // 3
        pad = torch.zeros(7, 3, 3 * gs, dtype=torch.uint8)
        pad[..., :d] = x
        cw = cpu.golay_encode_rows(x)
        assert torch.equal(cw.reshape(-1), cpu.golay_encode(pad.view(-1, 3)))
        noisy = cpu.inject_bit_errors_triton(cw, 0.05, 24, seed=1)
        st = cpu.new_stats()
        dec = cpu.golay_decode_rows(noisy, d, stats=st)
        trip, (bits, unc) = cpu.golay_decode(noisy.reshape(-1))
        assert torch.equal(dec, trip.view(7, 3, 3 * gs)[..., :d])
        assert cpu.read_stats(st) == [bits, unc]


def _packed_reference(trip_u8):
    """Packed layout restated from the reference-layout codec: int32 codewords ->
    3 little-endian bytes; triplets -> nibble stream two per byte."""
    from kvecc import cpu_ops
    cw = cpu_ops.golay_encode(trip_u8.view(-1, 3)).to(torch.int64)
    cw3 = torch.stack([(cw >> (8 * k)) & 0xFF for k in range(3)], 1).to(torch.uint8).reshape(-1)
    return cpu_ops.pack_nibbles(trip_u8.reshape(-1)), cw3


@pytest.mark.parametrize("m", [1, 2, 7, 8, 9, 100, 8192 * 2 + 5])
def test_golay_packed_vs_reference_layout(cpu, m):
    """Packed encode/decode carry exactly the reference layout's bits."""
    g = torch.Generator().manual_seed(m)
    trip = torch.randint(0, 16, (m, 3), generator=g, dtype=torch.uint8)
    nib, cw3 = _packed_reference(trip)
    assert torch.equal(cpu.golay_encode_packed(nib, m), cw3)
    # corrupt through the reference-layout path, decode both ways
    cw = cpu.golay_encode(trip)
    noisy = cpu.inject_bit_errors_triton(cw, 0.08, 24, seed=3)
    trip_ref, cnt_ref, (bits, unc) = cpu.golay_decode(noisy, return_error_counts=True)
    n64 = noisy.to(torch.int64)
    noisy3 = torch.stack([(n64 >> (8 * k)) & 0xFF for k in range(3)], 1).to(torch.uint8).reshape(-1)
    out, flags, st = cpu.golay_decode_packed(noisy3, m, return_uncorrectable=True)
    assert st == (bits, unc)
    assert torch.equal(cpu.unpack_nibbles(out, 3 * m), trip_ref.reshape(-1))
    if (3 * m) % 2:
        assert int(out[-1]) >> 4 == 0  # padding nibble is zero
    bitmask = torch.tensor([(int(flags[k // 8]) >> (k % 8)) & 1 for k in range(m)], dtype=torch.uint8)
    assert torch.equal(bitmask, (cnt_ref == 4).to(torch.uint8))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 15, 16, 17, 100, 4096 * 16 + 7])
def test_hamming84_packed_vs_reference_layout(cpu, n):
    g = torch.Generator().manual_seed(n)
    vals = torch.randint(0, 16, (n,), generator=g, dtype=torch.uint8)
    nib = cpu.pack_nibbles(vals)
    cw = cpu.hamming84_encode_packed(nib, n)
    assert torch.equal(cw, cpu.hamming84_encode(vals))
    noisy = cpu.inject_bit_errors_triton(cw, 0.05, 8, seed=4)
    data, et, st = cpu.hamming84_decode(noisy, return_error_types=True)
    pn, pt, pst = cpu.hamming84_decode_packed(noisy, return_error_types=True)
    assert pst == st
    assert torch.equal(pn, cpu.pack_nibbles(data)) and torch.equal(pt, cpu.pack_error_types(et))
    assert torch.equal(cpu.unpack_nibbles(pn, n), data)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_scale_rules(cpu, oracle, dtype):
    """Both row-scale rules against the oracle: "div7" (the reference on CPU
    tensors, the default here) and "mul_inv7" (abs_max * RN(1/7), the
    reference's `abs_max / 7.0` on a GPU); the rules disagree on many rows."""
    g = torch.Generator().manual_seed(4)
    x = (torch.randn(500, 64, generator=g) * 3).to(dtype)
    x[0] = 0
    inv7 = torch.tensor([1.0]) / torch.tensor([7.0])
    amax = x.float().abs().amax(-1)
    scales = {}
    for rule, code in (("div7", 0), ("mul_inv7", 1)):
        q, s = cpu.quantize_rows(x, scale_rule=rule)
        oq, os_ = oracle.quantize_rows(x.float().numpy(), rule=code)
        assert np.array_equal(q.numpy(), oq) and np.array_equal(s.numpy(), os_), rule
        cw, s84 = cpu.fused_quantize_encode_hamming84(x, scale_rule=rule)
        assert torch.equal(s84, s) and np.array_equal(cw.numpy(), oracle.hamming84_encode(oq))
        scales[rule] = s
    assert torch.equal(scales["mul_inv7"][1:], amax[1:] * inv7) and scales["mul_inv7"][0] == 1
    assert torch.equal(cpu.quantize_rows(x)[1], scales["div7"])
    assert int((scales["div7"] != scales["mul_inv7"]).sum()) > 50
    with pytest.raises(ValueError):
        cpu.quantize_rows(x, scale_rule="div8")


def test_golay_rows_into(cpu):
    """The _into twins write the allocating calls' bits into caller buffers and
    reject mismatched buffers."""
    g = torch.Generator().manual_seed(11)
    x = torch.randint(0, 16, (4, 6, 128), dtype=torch.uint8, generator=g)
    cw = torch.empty(4, 6, 43, dtype=torch.int32)
    cpu.golay_encode_rows_into(x, cw)
    assert torch.equal(cw, cpu.golay_encode_rows(x))
    noisy = cpu.inject_bit_errors_triton(cw, 0.05, 24, seed=3)
    out, st, st2 = torch.empty_like(x), cpu.new_stats(), cpu.new_stats()
    cpu.golay_decode_rows_into(noisy, out, st)
    assert torch.equal(out, cpu.golay_decode_rows(noisy, 128, st2))
    assert cpu.read_stats(st) == cpu.read_stats(st2)
    with pytest.raises(ValueError):
        cpu.golay_encode_rows_into(x, torch.empty(4, 6, 42, dtype=torch.int32))
    with pytest.raises(ValueError):
        cpu.golay_decode_rows_into(noisy, torch.empty(4, 6, 130, dtype=torch.uint8))


def test_count_ne_into(cpu):
    """kvecc_cpu_count_ne_u8: mismatching byte count added to stats[0]."""
    g = torch.Generator().manual_seed(12)
    for n in (0, 1, 15, 16, 17, 100003):
        a = torch.randint(0, 16, (n,), dtype=torch.uint8, generator=g)
        b = a.clone()
        if n:
            idx = torch.randint(0, n, (max(1, n // 7),), generator=g)
            b[idx] ^= 0x5
        st = cpu.new_stats()
        cpu.count_ne_into(a, b, st)
        cpu.count_ne_into(a, a, st)
        assert cpu.read_stats(st, 1)[0] == int((a != b).sum())
    with pytest.raises(ValueError):
        cpu.count_ne_into(a, b[:-1], cpu.new_stats())
