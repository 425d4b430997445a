"""Paged decode attention with inline ECC decode (attention_ecc.py:620-780)
against a plain torch fp32 reference of the same op.

The reference kernel walks tokens with an online softmax in fp32; the HIP
kernel splits the context and combines partials, so results agree to fp32
summation-order rounding: ATOL/RTOL below.  The host twin follows the
reference's sequential order.  Decoding itself is bit-exact (checked through
the oracle-pinned host backend).
"""

import math

import numpy as np
import pytest
import torch

ATOL = 2e-5
RTOL = 2e-4


def _cache(device, codec, batch, heads, kv_heads, d, ctx, ber, seed, layers=3, layer=1, bs=16):
    """Random paged caches written through the host backend (oracle-pinned)."""
    from kvecc import cpu_ops
    g = torch.Generator().manual_seed(seed)
    nblk_seq = (ctx + bs - 1) // bs
    num_blocks = batch * nblk_seq + 3
    per = d if codec == "hamming84" else (d + 2) // 3
    cdt = torch.uint8 if codec == "hamming84" else torch.int32
    kc = torch.zeros(num_blocks, layers, kv_heads, bs * per, dtype=cdt)
    vc = torch.zeros_like(kc)
    x = torch.randn(2, num_blocks, layers, kv_heads, bs, d, generator=g)
    for cache, xi in ((kc, x[0]), (vc, x[1])):
        q, s = cpu_ops.quantize_rows(xi)
        if codec == "hamming84":
            enc = cpu_ops.hamming84_encode(q)
        else:
            enc = cpu_ops.golay_encode_rows(q)
        if ber > 0:
            enc = cpu_ops.inject_bit_errors_triton(enc, ber, 8 if codec == "hamming84" else 24,
                                                   seed=seed)
        cache.copy_(enc.reshape(cache.shape))
    ks = torch.rand(num_blocks, layers, kv_heads, bs, generator=g) * 0.3 + 0.05
    vs = torch.rand(num_blocks, layers, kv_heads, bs, generator=g) * 0.3 + 0.05
    perm = torch.randperm(num_blocks, generator=g)[: batch * nblk_seq].to(torch.int32)
    max_blocks = nblk_seq + 2
    table = torch.full((batch, max_blocks), -1, dtype=torch.int32)
    table[:, :nblk_seq] = perm.view(batch, nblk_seq)
    lens = torch.tensor([max(1, ctx - 7 * b) for b in range(batch)], dtype=torch.int32)
    return kc, vc, table, lens, ks, vs


def _torch_reference(query, kc, vc, table, lens, ks, vs, layer, bs, codec):
    """fp32 torch restatement of paged_attention_ecc (per (b, h) softmax)."""
    from kvecc import cpu_ops
    b_, h_, d = query.shape
    kv_heads = kc.shape[2]
    groups = h_ // kv_heads
    out = torch.zeros(b_, h_, d)
    for b in range(b_):
        n = int(lens[b])
        pos = torch.arange(n)
        blk = table[b, pos // bs].long()
        slot = pos % bs
        ok = blk >= 0
        pos, blk, slot = pos[ok], blk[ok], slot[ok]
        if n and not bool(ok.any()):
            # no valid token: the reference's constant (DESIGN §1 quirk 14,
            # attention_ecc.py:342,391-423 / :806-807,885-886)
            out[b] = -8.0 if codec == "hamming84" else 0.0
            continue
        for side, cache, sc in ((0, kc, ks), (1, vc, vs)):
            rows = cache.view(cache.shape[0], cache.shape[1], kv_heads, bs, -1)[blk, layer, :, slot]
            if codec == "hamming84":
                dec, _ = cpu_ops.hamming84_decode(rows.contiguous())
            else:
                dec = cpu_ops.golay_decode_rows(rows.contiguous(), d)
            f = (dec.float() - 8.0) * sc[blk, layer, :, slot].unsqueeze(-1)  # [n, Hkv, d]
            if side == 0:
                kf = f
            else:
                vf = f
        for h in range(h_):
            hk = h // groups
            s = (query[b, h].float() @ kf[:, hk].T) / math.sqrt(d)
            w = torch.softmax(s, dim=0)
            out[b, h] = w @ vf[:, hk]
    return out


CASES = [("hamming84", 2, 4, 4, 64, 300, 0.01), ("hamming84", 1, 12, 12, 64, 1024, 0.0),
         ("hamming84", 3, 8, 2, 128, 700, 0.02), ("golay", 2, 4, 4, 128, 513, 0.02),
         ("golay", 1, 6, 3, 64, 77, 0.0), ("hamming84", 1, 2, 1, 32, 5, 0.05),
         # head_dim % 16 != 0: one-dword lane chunks (VEC 1) through the buffer-load kernel
         ("hamming84", 2, 4, 2, 100, 333, 0.01), ("hamming84", 1, 3, 3, 20, 90, 0.02),
         # GQA groups of 8 / 16 / 2 query heads at head_dim 64 / 128 / 32 (fp16
         # queries: the matrix-core kernel; fp32: the VALU kernels)
         ("hamming84", 2, 16, 2, 64, 257, 0.01), ("hamming84", 1, 32, 2, 128, 1000, 0.01),
         ("hamming84", 2, 8, 4, 32, 100, 0.0),
         # MHA at head_dim 128 / 32 (fp16 queries: the matrix-core kernel at one head per workgroup)
         ("hamming84", 2, 8, 8, 128, 700, 0.01), ("hamming84", 2, 4, 4, 32, 300, 0.01)]


@pytest.mark.parametrize("codec,batch,heads,kvh,d,ctx,ber", CASES)
def test_cpu_backend_vs_torch(codec, batch, heads, kvh, d, ctx, ber):
    from kvecc import cpu_ops
    kc, vc, table, lens, ks, vs = _cache("cpu", codec, batch, heads, kvh, d, ctx, ber, seed=ctx)
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(1))
    ref = _torch_reference(q, kc, vc, table, lens, ks, vs if codec == "hamming84" else ks, 1, 16,
                           codec)
    got = cpu_ops.paged_attention_ecc(q, kc, vc, table, lens, ks, 1, 16, codec=codec, v_scales=vs)
    assert torch.allclose(got, ref, atol=ATOL, rtol=RTOL), float((got - ref).abs().max())


def test_empty_context_and_missing_blocks():
    from kvecc import cpu_ops
    kc, vc, table, lens, ks, vs = _cache("cpu", "hamming84", 2, 2, 2, 32, 40, 0.0, seed=3)
    lens[1] = 0
    table[0, 1] = -1  # tokens 16..31 of sequence 0 are skipped
    q = torch.randn(2, 2, 32)
    got = cpu_ops.paged_attention_ecc(q, kc, vc, table, lens, ks, 1, 16, v_scales=vs)
    ref = _torch_reference(q, kc, vc, table, lens, ks, vs, 1, 16, "hamming84")
    # the reference kernel's empty-context value (attention_ecc.py:342,391-423)
    assert torch.equal(got[1], torch.full((2, 32), -8.0))
    assert torch.allclose(got[0], ref[0], atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
@pytest.mark.parametrize("codec,batch,heads,kvh,d,ctx,ber", CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_hip_vs_torch(gpu, codec, batch, heads, kvh, d, ctx, ber, dtype):
    from kvecc import ops
    kc, vc, table, lens, ks, vs = _cache("cpu", codec, batch, heads, kvh, d, ctx, ber, seed=ctx)
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(1)).to(dtype)
    ref = _torch_reference(q.float(), kc, vc, table, lens, ks, vs if codec == "hamming84" else ks,
                           1, 16, codec)
    dev = lambda t: t.to(gpu)  # noqa: E731
    got = ops.paged_attention_ecc(dev(q), dev(kc), dev(vc), dev(table), dev(lens), dev(ks), 1, 16,
                                  codec=codec, v_scales=dev(vs)).cpu()
    if codec == "golay" or dtype == torch.float32:
        assert got.dtype == torch.float32
        assert torch.allclose(got, ref, atol=ATOL, rtol=RTOL), float((got - ref).abs().max())
    else:  # fp16 output: within one fp16 ulp of the fp32 result
        assert got.dtype == dtype
        assert torch.allclose(got.float(), ref, atol=1e-3, rtol=1e-3), \
            float((got.float() - ref).abs().max())


def _pack_golay(cache, d):
    """int32 Golay cache [..., bs * g] -> the packed layout [..., bs * KVECC_GOLAY_PACKED_ROW(g)]
    (3 little-endian bytes per codeword, rows zero-padded to 4 bytes)."""
    g = (d + 2) // 3
    row = (3 * g + 3) // 4 * 4
    w = cache.view(*cache.shape[:-1], -1, g).numpy().astype(np.uint32)
    out = np.zeros(w.shape[:-1] + (row,), np.uint8)
    for byte in range(3):
        out[..., byte:3 * g:3] = (w >> (8 * byte)) & 0xFF
    return torch.from_numpy(out.reshape(*cache.shape[:-1], -1))


PACKED_CASES = [(2, 4, 4, 128, 513, 0.02), (1, 6, 3, 64, 77, 0.0), (3, 8, 2, 100, 300, 0.01),
                (2, 2, 1, 7, 41, 0.05), (1, 4, 4, 256, 2050, 0.01)]


@pytest.mark.parametrize("batch,heads,kvh,d,ctx,ber", PACKED_CASES[:3])
def test_cpu_packed_golay_equals_int32(batch, heads, kvh, d, ctx, ber):
    """The host twin reads the packed layout (KVECC_CODEC_GOLAY_PACKED) to the
    same bits as the int32 one."""
    from kvecc import cpu_ops
    kc, vc, table, lens, ks, vs = _cache("cpu", "golay", batch, heads, kvh, d, ctx, ber, seed=ctx)
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(1))
    outs = []
    for codec, k, v in (("golay", kc, vc), ("golay_packed", _pack_golay(kc, d), _pack_golay(vc, d))):
        out = torch.empty(batch, heads, d)
        cpu_ops.paged_attention_into(q, k, v, table, lens, ks, vs, out, 1, 16, 1 / math.sqrt(d), codec)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("batch,heads,kvh,d,ctx,ber", PACKED_CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_hip_packed_golay_vs_torch(gpu, batch, heads, kvh, d, ctx, ber, dtype):
    """kvecc_paged_attention on packed Golay caches (4 codewords per lane from
    one 12-byte buffer load) against the torch fp32 reference of the int32 layout."""
    from kvecc import ops
    kc, vc, table, lens, ks, vs = _cache("cpu", "golay", batch, heads, kvh, d, ctx, ber, seed=ctx)
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(1)).to(dtype)
    ref = _torch_reference(q.float(), kc, vc, table, lens, ks, vs, 1, 16, "golay")
    dev = lambda t: t.to(gpu)  # noqa: E731
    out = torch.empty(batch, heads, d, dtype=dtype, device=gpu)
    ops.paged_attention_into(dev(q), dev(_pack_golay(kc, d)), dev(_pack_golay(vc, d)), dev(table),
                             dev(lens), dev(ks), dev(vs), out, 1, 16, 1 / math.sqrt(d), "golay_packed")
    got = out.float().cpu()
    tol = (ATOL, RTOL) if dtype == torch.float32 else (1e-2, 1e-2)  # bf16 output rounding
    assert torch.allclose(got, ref, atol=tol[0], rtol=tol[1]), float((got - ref).abs().max())


GOLAY_FP16_CASES = [(2, 8, 2, 128, 300, 0.02), (1, 32, 2, 128, 1000, 0.01), (3, 4, 2, 128, 77, 0.0),
                    (2, 32, 16, 128, 513, 0.01), (1, 16, 4, 64, 200, 0.01), (2, 4, 4, 128, 129, 0.02)]


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["golay", "golay_packed"])
@pytest.mark.parametrize("batch,heads,kvh,d,ctx,ber", GOLAY_FP16_CASES)
def test_hip_golay_fp16_native_vs_torch(gpu, batch, heads, kvh, d, ctx, ber, codec):
    """The native entry (paged_attention_into) with fp16 queries over int32 and
    packed Golay caches, output fp16: GQA groups 4 / 16 / 2 / 2 at head_dim 128
    take the matrix-core kernel, head_dim 64 and MHA the VALU kernels."""
    from kvecc import ops
    kc, vc, table, lens, ks, vs = _cache("cpu", "golay", batch, heads, kvh, d, ctx, ber, seed=ctx + 3)
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(2)).half()
    ref = _torch_reference(q.float(), kc, vc, table, lens, ks, vs, 1, 16, "golay")
    if codec == "golay_packed":
        kc, vc = _pack_golay(kc, d), _pack_golay(vc, d)
    dev = lambda t: t.to(gpu)  # noqa: E731
    out = torch.empty(batch, heads, d, dtype=torch.float16, device=gpu)
    ops.paged_attention_into(dev(q), dev(kc), dev(vc), dev(table), dev(lens), dev(ks), dev(vs), out, 1, 16,
                             1 / math.sqrt(d), codec)
    got = out.float().cpu()
    # fp16 output: one fp16 ulp of the fp32 result
    assert torch.allclose(got, ref, atol=1e-3, rtol=1e-3), float((got - ref).abs().max())


# ---- reference-generated fixtures (tools/gen_golden.py gen_attention) ---------------
# Outputs of the reference's own paged_attention_ecc: the Triton H84 kernel
# (attention_ecc.py:264-427) under TRITON_INTERPRET=1 and the Golay
# reference_attention_ecc (:783-909).  fp32 tolerance: the reference walks the
# context sequentially, kvecc splits it (summation order only).


def _fixture_cases(manifest):
    return [c["name"] for c in manifest["attention"]["params"]["cases"]]


def _fixture(golden, manifest, name):
    z = golden("attention")
    meta = {c["name"]: c for c in manifest["attention"]["params"]["cases"]}[name]
    arr = {k: torch.from_numpy(z[f"{name}_{k}"]) for k in
           ("q", "k_cache", "v_cache", "block_table", "context_lens", "k_scales", "v_scales", "out")}
    return meta, arr


FIXTURES = ["h84_basic", "h84_empty", "h84_holes", "h84_all_missing", "h84_d100",
            "h84_vscales_none", "h84_fp16", "golay_basic", "golay_empty_holes", "golay_d100",
            # use_tiled=True: the reference's tiled kernel (empty contexts give 0)
            "h84_tiled_empty", "h84_tiled_holes", "h84_tiled_all_missing", "h84_tiled_small_block"]


def test_fixture_inventory(manifest):
    assert _fixture_cases(manifest) == FIXTURES


def _run_fixture(mod, meta, arr, dev=None):
    t = (lambda x: x.to(dev)) if dev is not None else (lambda x: x)
    return mod.paged_attention_ecc(t(arr["q"]), t(arr["k_cache"]), t(arr["v_cache"]),
                                   t(arr["block_table"]), t(arr["context_lens"]), t(arr["k_scales"]),
                                   meta["layer"], meta["block_size"], codec=meta["codec"],
                                   v_scales=t(arr["v_scales"]) if meta["v_scales"] else None,
                                   use_tiled=meta.get("use_tiled", False),
                                   block_m=meta.get("block_m", 4)).cpu()


def _assert_fixture(got, meta, arr):
    want = arr["out"]
    assert got.dtype == want.dtype, (got.dtype, want.dtype)
    if want.dtype == torch.float16:  # fp16 output: one fp16 ulp of the fp32 result
        assert torch.allclose(got.float(), want.float(), atol=1e-3, rtol=1e-3)
    else:
        assert torch.allclose(got, want, atol=ATOL, rtol=RTOL), float((got - want).abs().max())
    # empty / all-missing contexts reproduce the reference's exact value
    for b in range(got.shape[0]):
        if bool((want[b] == want[b].flatten()[0]).all()) and float(want[b].flatten()[0]) in (0.0, -8.0):
            assert torch.equal(got[b], want[b])


@pytest.mark.parametrize("name", FIXTURES)
def test_cpu_backend_vs_reference_fixture(golden, manifest, name):
    from kvecc import cpu_ops
    meta, arr = _fixture(golden, manifest, name)
    _assert_fixture(_run_fixture(cpu_ops, meta, arr), meta, arr)


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_hip_vs_reference_fixture(gpu, golden, manifest, name):
    from kvecc import ops
    meta, arr = _fixture(golden, manifest, name)
    _assert_fixture(_run_fixture(ops, meta, arr, gpu), meta, arr)


@pytest.mark.gpu
def test_hip_empty_context_values(gpu):
    """context_len 0 and an all -1 table: H84 -8.0, Golay 0 in every lane, for
    every output dtype and both cache layouts (the split and combine kernels)."""
    from kvecc import ops
    for codec in ("hamming84", "golay"):
        kc, vc, table, lens, ks, vs = _cache("cpu", codec, 3, 4, 2, 64, 40, 0.0, seed=5)
        lens[0] = 0
        table[2, :] = -1
        want = -8.0 if codec == "hamming84" else 0.0
        for dt in (torch.float32, torch.float16, torch.bfloat16):
            q = torch.randn(3, 4, 64).to(dt)
            g = lambda t: t.to(gpu)  # noqa: E731
            out = torch.empty(3, 4, 64, dtype=dt, device=gpu)
            ops.paged_attention_into(g(q), g(kc), g(vc), g(table), g(lens), g(ks), g(vs), out, 1, 16,
                                     0.125, codec)
            out = out.float().cpu()
            assert torch.equal(out[0], torch.full((4, 64), want)), (codec, dt)
            assert torch.equal(out[2], torch.full((4, 64), want)), (codec, dt)
            assert bool(torch.isfinite(out[1]).all()) and not torch.equal(out[1], out[0])


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["hamming84", "golay", "golay_packed"])
def test_hip_mfma_gqa_holes_and_buffer_end(gpu, codec):
    """The matrix-core GQA kernels (fp16 queries, head_dim 128, 4 query heads per
    cache head) with an empty context, a -1 block inside a context, and the cache
    buffer's last row in use (layer 2 of 3, last block, last cache head): the
    packed Golay loads read past a row's 129 bytes, which the buffer descriptor's
    range must absorb at the end of the allocation."""
    from kvecc import ops
    base = "hamming84" if codec == "hamming84" else "golay"
    batch, heads, kvh, d, ctx, layer = 3, 16, 4, 128, 90, 2
    kc, vc, table, lens, ks, vs = _cache("cpu", base, batch, heads, kvh, d, ctx, 1e-3, seed=11)
    lens[0] = 96                     # sequence 0 ends on row 15 of its sixth block ...
    table[0, 5] = kc.shape[0] - 1    # ... which is the buffer's last block
    table[1, 2] = -1                 # tokens 32..47 of sequence 1 are skipped
    lens[2] = 0
    q = torch.randn(batch, heads, d, generator=torch.Generator().manual_seed(4)).half()
    ref = _torch_reference(q.float(), kc, vc, table, lens, ks, vs, layer, 16, base)
    if codec == "golay_packed":
        kc, vc = _pack_golay(kc, d), _pack_golay(vc, d)
    dev = lambda t: t.to(gpu)  # noqa: E731
    out = torch.empty(batch, heads, d, dtype=torch.float16, device=gpu)
    ops.paged_attention_into(dev(q), dev(kc), dev(vc), dev(table), dev(lens), dev(ks), dev(vs), out, layer, 16,
                             1 / math.sqrt(d), codec)
    got = out.float().cpu()
    assert torch.equal(got[2], torch.full((heads, d), -8.0 if codec == "hamming84" else 0.0))
    assert torch.allclose(got[:2], ref[:2], atol=1e-3, rtol=1e-3), float((got[:2] - ref[:2]).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["golay", "golay_packed"])
def test_hip_golay_long_context_fold(gpu, codec):
    """The Golay kernel sums raw nibbles and folds the -8 out per split
    (acc - 8*psum).  At 32k tokens of small V values (n close to 8, the worst
    case for that cancellation) it stays within 2e-6 of an fp64 reference."""
    from kvecc import cpu_ops, ops
    g = torch.Generator().manual_seed(11)
    ctx, d, heads, bs = 32768, 128, 2, 16
    nblk = ctx // bs
    gw = (d + 2) // 3
    x = (torch.randn(2, nblk, 1, heads, bs, d, generator=g) * 0.02)
    x[..., 0] = 0.14  # row absmax pinned: values ~ +-0.02 quantize to n in 7..9
    caches, scales = [], []
    for side in range(2):
        q4, s = cpu_ops.quantize_rows(x[side])
        caches.append(cpu_ops.golay_encode_rows(q4).reshape(nblk, 1, heads, bs * gw))
        scales.append(s.reshape(nblk, 1, heads, bs))
    table = torch.randperm(nblk, generator=g).to(torch.int32).view(1, nblk)
    lens = torch.tensor([ctx], dtype=torch.int32)
    q = torch.randn(1, heads, d, generator=g)
    # fp64 reference over the decoded values
    rows = torch.arange(ctx)
    blk = table[0, rows // bs].long()
    slot = rows % bs
    ref = torch.zeros(1, heads, d, dtype=torch.float64)
    dec = []
    for side in range(2):
        c = caches[side].view(nblk, 1, heads, bs, gw)[blk, 0, :, slot]  # [ctx, heads, gw]
        n = cpu_ops.golay_decode_rows(c.contiguous(), d).double()
        dec.append((n - 8.0) * scales[side][blk, 0, :, slot].double().unsqueeze(-1))
    for h in range(heads):
        s = (q[0, h].double() @ dec[0][:, h].T) / math.sqrt(d)
        ref[0, h] = torch.softmax(s, 0) @ dec[1][:, h]
    kc, vc = caches
    if codec == "golay_packed":
        kc, vc = _pack_golay(kc, d), _pack_golay(vc, d)
    out = torch.empty(1, heads, d, device=gpu)
    t = lambda v: v.to(gpu)  # noqa: E731
    ops.paged_attention_into(t(q), t(kc), t(vc), t(table), t(lens), t(scales[0]), t(scales[1]), out,
                             0, bs, 1 / math.sqrt(d), codec)
    err = float((out.cpu().double() - ref).abs().max())
    assert err < 2e-6, err
