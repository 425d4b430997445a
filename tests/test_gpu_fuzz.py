"""Seeded random sizes and buffer offsets for the flat codec ops, the injection
shards, the interpolation, the fused quantize / dequantize and the packed
layouts: every HIP kernel path (vector bodies, unaligned heads, scalar tails)
against the host twin (kvecc.cpu_ops) bit for bit, outputs and statistics.

The fixed-shape parity tests (test_gpu_parity.py) pin both backends to the
oracle and the reference's golden vectors; this sweep covers the size and
alignment space between them.  KVECC_SWEEP_SCALE / KVECC_SWEEP_SEED extend it
(tests/test_geometry_sweep.py).
"""

import os
import random
import zlib

import pytest
import torch

pytestmark = pytest.mark.gpu

SCALE = int(os.environ.get("KVECC_SWEEP_SCALE", "1"))
SEED = int(os.environ.get("KVECC_SWEEP_SEED", "0"))
N = 12 * SCALE


def _cases(tag, make):
    rng = random.Random(zlib.crc32(tag.encode()) + 7919 * SEED)
    return [make(rng, i) for i in range(N)]


def _size(rng):
    # tails of every residue, small and large
    return rng.choice([1, 2, 3, 5, 7, 15, 16, 17, 63, 64, 65, 255, 1000, 4097]) + rng.choice([0, 0, 1024, 65536,
                                                                                              300000])


def _view(t, off, dev):
    """t (1-D) on `dev` starting `off` elements into a larger buffer."""
    base = torch.zeros(t.numel() + off + 16, dtype=t.dtype, device=dev)
    base[off:off + t.numel()] = t.to(dev)
    return base[off:off + t.numel()]


HAMMING = _cases("hamming", lambda r, i: (i, r.choice([7, 8]), _size(r), r.choice([0, 1, 2, 3, 5, 16]),
                                          r.choice([0.0, 1e-2, 0.1])))


@pytest.mark.parametrize("case", HAMMING, ids=[f"h{c[0]}" for c in HAMMING])
def test_fuzz_hamming(gpu, case):
    from kvecc import cpu_ops, ops
    i, bits, n, off, ber = case
    g = torch.Generator().manual_seed(1000 + i)
    x = torch.randint(0, 16, (n,), generator=g, dtype=torch.uint8)
    enc = cpu_ops.hamming84_encode if bits == 8 else cpu_ops.hamming74_encode
    cw = enc(x)
    if ber:
        cw = cpu_ops.inject_bit_errors_triton(cw, ber, bits, seed=i)
    genc = torch.empty(n, dtype=torch.uint8, device=gpu)
    (ops.hamming84_encode_into if bits == 8 else ops.hamming74_encode_into)(_view(x, off, gpu), genc)
    assert torch.equal(genc.cpu(), enc(x)), case
    data, flag = torch.empty(n, dtype=torch.uint8), torch.empty(n, dtype=torch.uint8)
    st = cpu_ops.new_stats()
    gd, gf = torch.empty(n, dtype=torch.uint8, device=gpu), torch.empty(n, dtype=torch.uint8, device=gpu)
    gst = ops.new_stats(gpu)
    if bits == 8:
        cpu_ops.hamming84_decode_into(cw, data, flag, st)
        ops.hamming84_decode_into(_view(cw, off, gpu), gd, gf, gst)
    else:
        cpu_ops.hamming74_decode_into(cw, data, flag, st)
        ops.hamming74_decode_into(_view(cw, off, gpu), gd, gf, gst)
    assert torch.equal(gd.cpu(), data) and torch.equal(gf.cpu(), flag), case
    assert ops.read_stats(gst) == cpu_ops.read_stats(st), case


GOLAY = _cases("golay", lambda r, i: (i, _size(r), r.choice([0, 1, 3, 4, 12]), r.choice([0.0, 1e-2, 5e-2])))


@pytest.mark.parametrize("case", GOLAY, ids=[f"g{c[0]}" for c in GOLAY])
def test_fuzz_golay_flat(gpu, case):
    from kvecc import cpu_ops, ops
    i, m, off, ber = case
    g = torch.Generator().manual_seed(2000 + i)
    trip = torch.randint(0, 16, (3 * m,), generator=g, dtype=torch.uint8)
    cw = torch.empty(m, dtype=torch.int32)
    cpu_ops.golay_encode_into(trip, cw, m)
    gcw = torch.empty(m, dtype=torch.int32, device=gpu)
    ops.golay_encode_into(_view(trip, off, gpu), gcw, m)
    assert torch.equal(gcw.cpu(), cw), case
    if ber:
        cw = cpu_ops.inject_bit_errors_triton(cw, ber, 24, seed=i)
    t, c, st = torch.empty(3 * m, dtype=torch.uint8), torch.empty(m, dtype=torch.uint8), cpu_ops.new_stats()
    cpu_ops.golay_decode_into(cw, t, c, st)
    gt = torch.empty(3 * m, dtype=torch.uint8, device=gpu)
    gc = torch.empty(m, dtype=torch.uint8, device=gpu)
    gst = ops.new_stats(gpu)
    ops.golay_decode_into(_view(cw, off, gpu), gt, gc, gst)
    assert torch.equal(gt.cpu(), t) and torch.equal(gc.cpu(), c), case
    assert ops.read_stats(gst) == cpu_ops.read_stats(st), case


INJECT = _cases("inject", lambda r, i: (i, r.choice(["u8", "i32"]), _size(r), r.randint(1, 8), r.randint(1, 24),
                                        r.choice([1e-4, 1e-2, 0.3, 1.0]), r.randint(0, 2 ** 31 - 1),
                                        r.choice([0, 1, 3, 1000003]), r.choice([0, 1, 5])))


@pytest.mark.parametrize("case", INJECT, ids=[f"i{c[0]}" for c in INJECT])
def test_fuzz_inject(gpu, case):
    """A shard [offset0, offset0 + n) of a global_n tensor, with counts and statistics."""
    from kvecc import cpu_ops, ops
    i, kind, n, nb8, nb32, ber, seed, extra, off = case
    g = torch.Generator().manual_seed(3000 + i)
    if kind == "u8":
        x, nb = torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8), nb8
    else:
        x, nb = torch.randint(0, 2 ** 24, (n,), generator=g, dtype=torch.int32), nb32
    gn, o0 = n + extra, extra // 2
    out, cnt, st = torch.empty_like(x), torch.empty(n, dtype=torch.uint8), cpu_ops.new_stats()
    cpu_ops.inject_into(x, out, ber, nb, seed=seed, counts=cnt, stats=st, global_n=gn, offset0=o0)
    gout = torch.empty(n, dtype=x.dtype, device=gpu)
    gcnt = torch.empty(n, dtype=torch.uint8, device=gpu)
    gst = ops.new_stats(gpu)
    ops.inject_into(_view(x, off, gpu), gout, ber, nb, seed=seed, counts=gcnt, stats=gst, global_n=gn, offset0=o0)
    assert torch.equal(gout.cpu(), out) and torch.equal(gcnt.cpu(), cnt), case
    assert ops.read_stats(gst) == cpu_ops.read_stats(st), case


INTERP = _cases("interp", lambda r, i: (i, r.choice([1, 2, 3, 7]), r.choice([1, 2, 3, 4, 31, 32, 33, 100, 513]),
                                        r.choice([1, 3, 15, 16, 17, 48, 1000, 1024, 1040]),
                                        r.choice([0.0, 0.05, 0.5]), r.choice([0, 1, 16])))


@pytest.mark.parametrize("case", INTERP, ids=[f"p{c[0]}" for c in INTERP])
def test_fuzz_interpolate(gpu, case):
    from kvecc import cpu_ops, ops
    i, outer, length, inner, pdbl, off = case
    g = torch.Generator().manual_seed(4000 + i)
    n = outer * length * inner
    q = torch.randint(0, 16, (n,), generator=g, dtype=torch.uint8)
    err = torch.where(torch.rand(n, generator=g) < pdbl, 2, torch.randint(0, 2, (n,), generator=g)).to(torch.uint8)
    out = torch.empty_like(q)
    cpu_ops.interpolate_into(q, err, out, outer, length, inner)
    gout = torch.empty(n, dtype=torch.uint8, device=gpu)
    ops.interpolate_into(_view(q, off, gpu), _view(err, off, gpu), gout, outer, length, inner)
    assert torch.equal(gout.cpu(), out), case


QUANT = _cases("quant", lambda r, i: (i, r.randint(1, 700), r.choice([4, 8, 12, 20, 64, 100, 128, 256, 512, 520]),
                                      r.choice(["float32", "float16", "bfloat16"]), r.choice([0, 1, 2]),
                                      r.choice(["div7", "mul_inv7"])))


@pytest.mark.parametrize("case", QUANT, ids=[f"q{c[0]}" for c in QUANT])
def test_fuzz_quantize_encode_and_dequantize(gpu, case):
    from kvecc import cpu_ops, ops
    i, rows, d, dtype, codec, rule = case
    dt = getattr(torch, dtype)
    g = torch.Generator().manual_seed(5000 + i)
    x = (torch.randn(rows, d, generator=g) * torch.rand(rows, 1, generator=g) * 10).to(dt)
    x[0, :] = 0  # an all-zero row (scale 1)
    cw, sc = torch.empty(rows, d, dtype=torch.uint8), torch.empty(rows)
    cpu_ops.quantize_encode_rows_into(x, codec, cw, sc, scale_rule=rule)
    gcw = torch.empty(rows, d, dtype=torch.uint8, device=gpu)
    gsc = torch.empty(rows, device=gpu)
    ops.quantize_encode_rows_into(x.to(gpu), codec, gcw, gsc, scale_rule=rule)
    assert torch.equal(gcw.cpu(), cw) and torch.equal(gsc.cpu(), sc), case
    if codec != 2:
        return
    noisy = cpu_ops.inject_bit_errors_triton(cw, 2e-2, 8, seed=i)
    for odt in (torch.float32, torch.float16, torch.bfloat16):
        for zero_doubles in (True, False):
            out, st = torch.empty(rows, d, dtype=odt), cpu_ops.new_stats()
            cpu_ops.decode_dequant_h84_into(noisy, sc, out, zero_doubles, st)
            gout, gst = torch.empty(rows, d, dtype=odt, device=gpu), ops.new_stats(gpu)
            ops.decode_dequant_h84_into(noisy.to(gpu), sc.to(gpu), gout, zero_doubles, gst)
            assert torch.equal(gout.cpu(), out), (case, odt, zero_doubles)
            assert ops.read_stats(gst) == cpu_ops.read_stats(st), (case, odt, zero_doubles)


PACKED = _cases("packed", lambda r, i: (i, r.choice(["golay", "hamming84"]), _size(r), r.choice([0.0, 1e-2, 5e-2])))


@pytest.mark.parametrize("case", PACKED, ids=[f"k{c[0]}" for c in PACKED])
def test_fuzz_packed(gpu, case):
    from kvecc import cpu_ops, ops
    i, codec, m, ber = case
    g = torch.Generator().manual_seed(6000 + i)
    if codec == "golay":
        nib = torch.randint(0, 256, ((3 * m + 1) // 2,), generator=g, dtype=torch.uint8)
        cw = cpu_ops.golay_encode_packed(nib, m)
        assert torch.equal(ops.golay_encode_packed(nib.to(gpu), m).cpu(), cw), case
        if ber:
            cw = cpu_ops.inject_bit_errors_triton(cw, ber, 8, seed=i)
        ref = cpu_ops.golay_decode_packed(cw, m, return_uncorrectable=True)
        got = ops.golay_decode_packed(cw.to(gpu), m, return_uncorrectable=True)
    else:
        nib = torch.randint(0, 256, ((m + 1) // 2,), generator=g, dtype=torch.uint8)
        cw = cpu_ops.hamming84_encode_packed(nib, m)
        assert torch.equal(ops.hamming84_encode_packed(nib.to(gpu), m).cpu(), cw), case
        if ber:
            cw = cpu_ops.inject_bit_errors_triton(cw, ber, 8, seed=i)
        ref = cpu_ops.hamming84_decode_packed(cw, return_error_types=True)
        got = ops.hamming84_decode_packed(cw.to(gpu), return_error_types=True)
    for a, b in zip(got, ref):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a.cpu(), b), case
        else:
            assert a == b, case


SHIM = _cases("shim", lambda r, i: (i, r.choice(["hamming84", "hamming74", "golay", "int4"]), r.choice([True, False]),
                                    r.choice([16, 20, 32, 48, 64, 100, 128, 256]), r.choice([1, 4, 8, 16, 32]),
                                    r.randint(1, 3), r.randint(1, 70), r.choice([1, 2, 4]), r.choice([1, 2]),
                                    r.choice(["float32", "float16", "bfloat16"]), r.choice([0.0, 1e-2, 5e-2]),
                                    r.choice(["div7", "mul_inv7"])))


@pytest.mark.parametrize("case", SHIM, ids=[f"s{c[0]}" for c in SHIM])
def test_fuzz_shim_write_read(gpu, case):
    """ECCBackend write + read (ecc_shim.py:557-721, 990-1071) on random cache
    geometries: the HIP backend's cache bits, scales, decoded K/V (attention
    dtype) and statistics equal the host backend's."""
    from kvecc.ecc_shim import ECCBackend, ECCShimConfig, SimpleBlockManager
    i, codec, interp, d, bs, batch, s, hk, groups, dtype, ber, rule = case
    interp = interp and codec == "hamming84"
    if codec != "golay" and d % 4:
        d += 4 - d % 4
    dt = getattr(torch, dtype)
    g = torch.Generator().manual_seed(7000 + i)
    k = torch.randn(batch, s, hk * d, generator=g).to(dt)
    v = torch.randn(batch, s, hk * d, generator=g).to(dt)
    res = []
    for dev, backend in ((gpu, "hip"), (torch.device("cpu"), "cpu")):
        cfg = ECCShimConfig(codec=codec, ber=ber, inject_errors=ber > 0, seed=11 + i, block_size=bs,
                            use_interpolation=interp, backend=backend, scale_rule=rule)
        nblk = (s + bs - 1) // bs + 1
        mgr = SimpleBlockManager(nblk, bs, 3, hk, d, device=dev, codec=codec)
        be = ECCBackend(mgr, cfg, num_heads=hk * groups)
        be._injection_count = i
        be.write(k.to(dev), v.to(dev), layer_idx=1)
        kt, vt = be.codec_backend.shim_read(mgr, 1, s, mgr.shim_codec, interp, dt, be._stats)
        res.append((mgr.k_cache.cpu(), mgr.v_cache.cpu(), mgr.k_scales.cpu(), mgr.v_scales.cpu(),
                    kt.cpu(), vt.cpu(), be._injection_count, be._errors_corrected, be._errors_detected))
    h, c = res
    for j in range(6):
        assert torch.equal(h[j], c[j]), (case, j)
    assert h[6:] == c[6:], (case, h[6:], c[6:])
