"""Sizes past 32-bit indexing on one MI355X (288 GB of HBM invites them).

Byte codecs run on 2^32 + a few elements, Golay on 2^31 + a few codewords.
Parity here is by size-independent properties: encode -> decode round trips,
planted errors at the far end of the buffer (past every 32-bit boundary)
corrected and counted exactly, interpolation of planted double errors against
the reference formula (interpolation_triton.py:120-159) on the neighbourhood,
and the fused quantizer against the oracle on sampled rows.  ~30 GB of HBM.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

BIG = (1 << 32) + 4101       # bytes / values
BIG_CW = (1 << 31) + 5       # Golay codewords


def _far_positions(n):
    return [n - 1, n - 2, (1 << 32) + 5 if n > (1 << 32) + 5 else n // 2, (1 << 31) + 3, 7]


def test_hamming84_past_4g(gpu):
    from kvecc import ops
    x = torch.randint(0, 16, (BIG,), dtype=torch.uint8, device=gpu)
    cw = torch.empty_like(x)
    ops.hamming84_encode_into(x, cw)
    pos = _far_positions(BIG)
    for i, p in enumerate(pos):  # data-bit singles (corrected), one double (kept, detected)
        cw[p] ^= 1 << (i % 4)
    cw[BIG - 3] ^= 0x03
    data, et = torch.empty_like(x), torch.empty_like(x)
    st = ops.new_stats(gpu)
    ops.hamming84_decode_into(cw, data, et, st)
    assert ops.read_stats(st) == [len(pos), 1]
    assert int((et == 1).sum()) == len(pos) and int(et[BIG - 3]) == 2
    data[BIG - 3] = x[BIG - 3]  # the double keeps corrupted data
    assert torch.equal(data, x)
    del data, et
    # Hamming(7,4) through the same buffers
    ops.hamming74_encode_into(x, cw)
    cw[BIG - 1] ^= 0x04
    data = torch.empty_like(x)
    st = ops.new_stats(gpu)
    ops.hamming74_decode_into(cw, data, None, st)
    assert ops.read_stats(st, 1) == [1] and torch.equal(data, x)


def test_golay_past_2g_codewords(gpu):
    from kvecc import ops
    trip = torch.randint(0, 16, (BIG_CW * 3,), dtype=torch.uint8, device=gpu)
    cw = torch.empty(BIG_CW, dtype=torch.int32, device=gpu)
    ops.golay_encode_into(trip, cw, BIG_CW)
    pos = [BIG_CW - 1, BIG_CW - 2, (1 << 31) + 1, 3]
    for p in pos:
        cw[p] ^= 0x800401  # 3-bit error: corrected
    cw[BIG_CW - 3] ^= 0xF  # 4 bits: uncorrectable
    out = torch.empty_like(trip)
    counts = torch.empty(BIG_CW, dtype=torch.uint8, device=gpu)
    st = ops.new_stats(gpu)
    ops.golay_decode_into(cw, out, counts, st)
    assert ops.read_stats(st) == [3 * len(pos), 1]
    assert int(counts[BIG_CW - 3]) == 4 and all(int(counts[p]) == 3 for p in pos)
    o = out.view(-1, 3)
    o[BIG_CW - 3] = trip.view(-1, 3)[BIG_CW - 3]
    assert torch.equal(out, trip)


def test_packed_golay_past_2g_codewords(gpu):
    from kvecc import ops
    m = BIG_CW
    nib = torch.randint(0, 256, ((3 * m + 1) // 2,), dtype=torch.uint8, device=gpu)
    if (3 * m) % 2:
        nib[-1] &= 0x0F  # the unused high nibble of the last byte stays zero
    cw3 = torch.empty(3 * m, dtype=torch.uint8, device=gpu)
    ops.golay_encode_packed_into(nib, cw3, m)
    cw3[3 * (m - 1)] ^= 0x05  # 2 bits in the last codeword
    back = torch.empty_like(nib)
    flags = torch.zeros((m + 7) // 8, dtype=torch.uint8, device=gpu)
    st = ops.new_stats(gpu)
    ops.golay_decode_packed_into(cw3, back, flags, m, st)
    assert ops.read_stats(st) == [2, 0] and int(flags.sum()) == 0
    assert torch.equal(back, nib)


def test_interpolation_and_gate_past_4g(gpu):
    from kvecc import ops
    q = torch.randint(0, 16, (BIG,), dtype=torch.uint8, device=gpu)
    err = torch.zeros_like(q)
    flag = torch.empty(1, dtype=torch.int32, device=gpu)
    ops.any_equal(err, 2, flag)
    assert int(flag) == 0
    pos = [BIG - 1, BIG - 2, (1 << 32) + 9, 11]
    for p in pos:
        err[p] = 2
    ops.any_equal(err, 2, flag)
    assert int(flag) == 1
    out = torch.empty_like(q)
    ops.interpolate_into(q, err, out, 1, BIG, 1)  # one row of length BIG
    for p in pos:
        left = int(q[max(p - 1, 0)])
        right = int(q[min(p + 1, BIG - 1)])
        exp = min(15, int(np.trunc(np.float32((left + right) * 0.5 + 0.5))))
        assert int(out[p]) == exp, p
    for p in pos:  # everything else is a (clamped, q <= 15) copy
        out[p] = q[p]
    assert torch.equal(out, q)


def test_fused_quantize_dequant_past_4g(gpu, oracle):
    from kvecc import ops
    d = 128
    rows = BIG // d + 1
    x = torch.randn(rows, d, device=gpu, dtype=torch.float16) * 3
    cw = torch.empty(rows, d, dtype=torch.uint8, device=gpu)
    sc = torch.empty(rows, dtype=torch.float32, device=gpu)
    ops.quantize_encode_rows_into(x, 2, cw, sc, scale_rule="div7")
    sample = [0, 1, rows // 2, (1 << 25) + 1, rows - 2, rows - 1]
    xs = x[sample].float().cpu().numpy()
    oq, os_ = oracle.quantize_rows(xs)
    assert np.array_equal(cw[sample].cpu().numpy(), oracle.hamming84_encode(oq))
    assert np.array_equal(sc[sample].cpu().numpy(), os_)
    out = torch.empty_like(x)
    st = ops.new_stats(gpu)
    ops.decode_dequant_h84_into(cw, sc, out, True, st)
    ref, _ = oracle.decode_dequant_h84(oracle.hamming84_encode(oq), os_)
    assert ops.read_stats(st) == [0, 0]
    assert torch.equal(out[sample].cpu(), torch.from_numpy(ref).to(torch.float16))


@pytest.mark.parametrize("codec", ["hamming84", "golay", "golay_packed"])
def test_paged_attention_cache_past_4g(gpu, codec):
    """Caches over 4 GiB take the 64-bit-addressed attention kernels (smaller
    ones use 32-bit buffer offsets).  The sequence's blocks sit past the 4 GiB
    mark; the result must equal the same blocks copied into a small cache,
    which runs the buffer-load kernels (~9 GB of HBM).  Hamming(8,4) uses fp32
    queries: fp16 MHA queries would send the small cache to the matrix-core
    kernel (different summation order), fp32 keeps both on the same kernel."""
    import math
    from kvecc import ops
    heads, d, bs, ctx, batch = 8, 128, 16, 1000, 2
    per = d if codec == "hamming84" else (d + 2) // 3
    if codec == "golay_packed":  # bytes per token row (KVECC_GOLAY_PACKED_ROW)
        per = (3 * per + 3) // 4 * 4
    cdt = torch.int32 if codec == "golay" else torch.uint8
    row_bytes = heads * bs * per * (4 if codec == "golay" else 1)
    num_blocks = (1 << 32) // row_bytes + 200                    # > 4 GiB per cache
    nb = (ctx + bs - 1) // bs
    g = torch.Generator(device=gpu).manual_seed(5)
    hi = 1 << 24 if codec == "golay" else 256
    used = torch.arange(num_blocks - batch * nb, num_blocks, device=gpu)   # the far end
    big_k = torch.zeros(num_blocks, 1, heads, bs * per, dtype=cdt, device=gpu)
    big_v = torch.zeros_like(big_k)
    small_k = torch.randint(0, hi, (batch * nb, 1, heads, bs * per), dtype=cdt, device=gpu, generator=g)
    small_v = torch.randint(0, hi, small_k.shape, dtype=cdt, device=gpu, generator=g)
    big_k[used] = small_k
    big_v[used] = small_v
    ks_small = torch.rand(batch * nb, 1, heads, bs, device=gpu, generator=g) + 0.1
    vs_small = torch.rand_like(ks_small) + 0.1
    ks_big = torch.zeros(num_blocks, 1, heads, bs, device=gpu)
    vs_big = torch.zeros_like(ks_big)
    ks_big[used] = ks_small
    vs_big[used] = vs_small
    perm = torch.randperm(batch * nb, device=gpu, generator=g).to(torch.int32).view(batch, nb)
    lens = torch.tensor([ctx, ctx - 37], dtype=torch.int32, device=gpu)
    q = torch.randn(batch, heads, d, device=gpu, generator=g)
    q = q if codec == "hamming84" else q.half()
    outs = []
    for kc, vc, ks, vs, table in ((big_k, big_v, ks_big, vs_big, perm + (num_blocks - batch * nb)),
                                  (small_k, small_v, ks_small, vs_small, perm)):
        out = torch.empty_like(q)
        ops.paged_attention_into(q, kc, vc, table.contiguous(), lens, ks, vs, out, 0, bs,
                                 1 / math.sqrt(d), codec, ctx)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])
