"""Generate golden input/output vectors from the reference implementation.

Runs the reference's own ``@triton.jit`` kernels on CPU under
``TRITON_INTERPRET=1`` and writes small ``.npz`` fixtures plus a
``MANIFEST.json`` (sha256 + parameters) into ``tests/golden/``.

This script runs ONLY in the development container, where the reference is
mounted read-only at /root/reference.  Nothing on the GPU box reads the
reference; the committed fixtures are data (inputs and expected outputs).

Usage (``-O`` strips the reference wrappers' ``assert x.is_cuda``)::

    python -O tools/gen_golden.py [--ref /root/reference] [--only NAME ...]
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

os.environ["TRITON_INTERPRET"] = "1"

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden")


def _save(name, manifest, params, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    with open(path, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    manifest[name] = {"file": name + ".npz", "sha256": digest, "params": params,
                      "arrays": {k: [list(v.shape), str(v.dtype)] for k, v in arrays.items()}}
    print(f"  wrote {name}.npz ({os.path.getsize(path)} B)")


def gen_hamming(manifest):
    import torch
    from ecc_codecs.triton_kernels import (hamming74_encode, hamming74_decode,
                                           hamming84_encode, hamming84_decode)
    allb = torch.arange(256, dtype=torch.int32).to(torch.uint8)
    e74 = hamming74_encode(allb)
    e84 = hamming84_encode(allb)
    d74, f74, (c74,) = hamming74_decode(allb, return_error_detected=True)
    d84, t84, (c84, det84) = hamming84_decode(allb, return_error_types=True)
    _save("hamming", manifest, {"inputs": "all 256 byte values, encode and decode"},
          inputs=allb.numpy(), enc74=e74.numpy(), enc84=e84.numpy(),
          dec74_data=d74.numpy(), dec74_flag=f74.numpy(),
          dec74_stats=np.array([c74], dtype=np.int64),
          dec84_data=d84.numpy(), dec84_type=t84.numpy(),
          dec84_stats=np.array([c84, det84], dtype=np.int64))


def gen_golay(manifest):
    import torch
    from ecc_codecs.triton_kernels import golay_encode, golay_decode
    from ecc_codecs.triton_kernels.config import (build_golay_syndrome_table,
                                                  GOLAY_H_ROW_MASKS)
    table = build_golay_syndrome_table().numpy().astype(np.int32)
    sha = hashlib.sha256(table.astype("<i4").tobytes()).hexdigest()
    # encode: all 4096 data words, then triplets whose high nibbles are dirty
    d = np.arange(4096, dtype=np.int64)
    trip = np.stack([d & 15, (d >> 4) & 15, (d >> 8) & 15], axis=1).astype(np.uint8)
    rng = np.random.default_rng(1234)
    dirty = rng.integers(0, 256, size=(1024, 3), dtype=np.int64).astype(np.uint8)
    enc_in = np.concatenate([trip, dirty], axis=0)
    enc_out = golay_encode(torch.from_numpy(enc_in)).numpy()
    # decode: codewords of random data with 0..7 random bit errors, plus garbage
    m = 16384
    data = rng.integers(0, 4096, size=m, dtype=np.int64)
    dtrip = np.stack([data & 15, (data >> 4) & 15, (data >> 8) & 15], axis=1).astype(np.uint8)
    clean = golay_encode(torch.from_numpy(dtrip)).numpy().astype(np.int64)
    nerr = rng.integers(0, 8, size=m)
    noisy = clean.copy()
    for i in range(m):
        pos = rng.choice(24, size=nerr[i], replace=False)
        for p in pos:
            noisy[i] ^= 1 << int(p)
    garbage = rng.integers(-(2**31), 2**31, size=2048, dtype=np.int64)
    dec_in = np.concatenate([noisy, garbage]).astype(np.int32)
    dtrips, dcounts, (bits, unc) = golay_decode(torch.from_numpy(dec_in), return_error_counts=True)
    _save("golay", manifest,
          {"table_sha256": sha, "decode": "16384 codewords with 0..7 random bit errors + 2048 random int32",
           "encode": "all 4096 data words + 1024 dirty triplets"},
          table=table, h_row_masks=np.array(GOLAY_H_ROW_MASKS, dtype=np.int64),
          enc_in=enc_in, enc_out=enc_out.astype(np.int32),
          dec_in=dec_in, dec_trip=dtrips.numpy(), dec_count=dcounts.numpy(),
          dec_stats=np.array([bits, unc], dtype=np.int64), dec_nerr=nerr.astype(np.int8))


INJECT_CASES = [
    # (dtype, n, n_bits, seed, ber)
    ("u8", 1000, 8, 42, 0.05),
    ("u8", 300, 7, 12345, 0.2),
    ("u8", 257, 4, 2**20 + 7, 0.3),
    ("u8", 4096, 8, 0, 1e-2),
    ("u8", 128, 8, 101, 0.5),
    ("u8", 64, 8, 997, 1.0),
    ("u8", 43, 1, 1, 0.5),
    ("u8", 100, 0, 3, 0.5),      # n_bits=0 still draws bit 0
    ("u8", 100, 12, 5, 0.3),     # n_bits>8 capped at 8 bits
    ("u8", 100000, 8, 31337, 1e-3),  # seed*N*n_bits overflows int32
    ("i32", 1000, 24, 42, 0.05),
    ("i32", 129, 24, 1, 0.01),
    ("i32", 43, 24, 31337, 0.2),
    ("i32", 60000, 24, 31337, 1e-2),  # overflow case
    ("i32", 200, 12, 7, 0.5),
    ("i32", 200, 30, 8, 0.3),   # n_bits>24 capped at 24
    ("i32", 64, 0, 9, 0.5),
]

VEC_CASES = [
    ("u8", 1000, 8, 42, 0.05),
    ("u8", 333, 5, 77, 0.3),
    ("u8", 200, 3, 2**24 + 1, 0.4),
    ("i32", 1000, 24, 42, 0.05),
    ("i32", 257, 13, 99, 0.3),
]


def gen_inject(manifest):
    import torch
    from ecc_codecs.triton_kernels import (inject_bit_errors_triton,
                                           inject_bit_errors_triton_vectorized)
    rng = np.random.default_rng(77)
    for tag, fn, cases in (("inject", inject_bit_errors_triton, INJECT_CASES),
                           ("inject_vec", inject_bit_errors_triton_vectorized, VEC_CASES)):
        arrays = {}
        params = []
        for idx, (dt, n, nb, seed, ber) in enumerate(cases):
            if dt == "u8":
                x = rng.integers(0, 256, size=n, dtype=np.int64).astype(np.uint8)
            else:
                x = rng.integers(0, 2**24, size=n, dtype=np.int64).astype(np.int32)
            t0 = time.time()
            out, (flips, affected) = fn(torch.from_numpy(x), ber, nb, seed=seed, return_stats=True)
            arrays[f"c{idx}_in"] = x
            arrays[f"c{idx}_out"] = out.numpy()
            arrays[f"c{idx}_stats"] = np.array([flips, affected], dtype=np.int64)
            params.append({"dtype": dt, "n": n, "n_bits": nb, "seed": seed, "ber": ber})
            print(f"    {tag} case {idx}: {dt} n={n} nb={nb} seed={seed} ber={ber} "
                  f"flips={flips} ({time.time() - t0:.1f}s)")
        _save(tag, manifest, {"cases": params}, **arrays)


def gen_interp(manifest):
    import torch
    from ecc_codecs.triton_kernels import interpolate_double_errors
    rng = np.random.default_rng(99)
    cases = []
    # reference KATs (tests/test_triton_interpolation.py)
    cases.append(("kat_mid", [4, 8, 12, 8, 4], [0, 0, 2, 0, 0], -1))
    cases.append(("kat_left", [15, 4, 8, 12], [2, 0, 0, 0], -1))
    cases.append(("kat_right", [4, 8, 12, 15], [0, 0, 0, 2], -1))
    cases.append(("kat_scatter", [0, 4, 8, 12, 8, 4, 0], [0, 2, 0, 2, 0, 2, 0], -1))
    cases.append(("kat_consec", [4, 0, 0, 0, 4], [0, 2, 2, 2, 0], -1))
    cases.append(("kat_single", [8], [2], -1))
    cases.append(("kat_none", [1, 5, 10, 15, 8], [0, 0, 0, 0, 0], -1))
    arrays = {}
    params = []
    for i, (name, q, e, sd) in enumerate(cases):
        arrays[f"c{i}_q"] = np.array(q, dtype=np.uint8)
        arrays[f"c{i}_err"] = np.array(e, dtype=np.uint8)
        params.append({"name": name, "seq_dim": sd})
    shapes = [((1000,), -1), ((16, 257), -1), ((16, 257), 0), ((37, 4, 24), 0),
              ((5, 6, 7, 8), 1), ((9, 3, 32), -1), ((64, 2, 48), 0)]
    for j, (shape, sd) in enumerate(shapes):
        q = rng.integers(0, 16, size=shape, dtype=np.int64).astype(np.uint8)
        if j == 1:
            q[0, :5] = [200, 17, 16, 255, 99]  # values >15 get clamped
        err = rng.choice(np.array([0, 1, 2, 3], dtype=np.uint8), size=shape, p=[0.7, 0.1, 0.15, 0.05])
        k = len(cases) + j
        arrays[f"c{k}_q"] = q
        arrays[f"c{k}_err"] = err
        params.append({"name": f"rand{j}", "seq_dim": sd, "shape": list(shape)})
    # no-double case with values >15: fast path returns the input unchanged
    k = len(cases) + len(shapes)
    qn = rng.integers(0, 256, size=(8, 40), dtype=np.int64).astype(np.uint8)
    arrays[f"c{k}_q"] = qn
    arrays[f"c{k}_err"] = rng.choice(np.array([0, 1, 3], dtype=np.uint8), size=(8, 40))
    params.append({"name": "nodouble_big", "seq_dim": -1})
    for idx, p in enumerate(params):
        q = torch.from_numpy(arrays[f"c{idx}_q"])
        e = torch.from_numpy(arrays[f"c{idx}_err"])
        out = interpolate_double_errors(q, e, seq_dim=p["seq_dim"])
        arrays[f"c{idx}_out"] = out.contiguous().numpy()
    _save("interp", manifest, {"cases": params}, **arrays)


def gen_fused(manifest):
    """Pin quantize+encode against the shim's torch path and the fused decode.

    The fused quantize kernels call ``libdevice.rint``, which the Triton
    interpreter cannot run; their parity target is the torch path of the shim
    (ecc_shim.py:572-580), so codewords are hamming8x_encode(torch-path q).
    ``fused_decode_dequantize_hamming84`` runs as-is.
    """
    import torch
    from ecc_codecs.triton_kernels import (hamming84_encode, hamming74_encode,
                                           fused_decode_dequantize_hamming84)
    from kv_cache.paged_cache_ecc import compute_quantization_scales
    g = torch.Generator().manual_seed(5)
    arrays = {}
    params = []
    for i, (rows, d) in enumerate([(64, 128), (37, 64), (5, 100), (3, 7)]):
        x = torch.randn(rows, d, generator=g) * (1.0 + i)
        x[0, :] = 0.0  # zero row -> scale 1.0
        # torch path of the shim (ecc_shim.py:572-580)
        sc = compute_quantization_scales(x.float(), dim=-1)
        q = (torch.round(x.float() / sc.unsqueeze(-1)).clamp(-8, 7) + 8).to(torch.uint8)
        cw84, s84 = hamming84_encode(q), sc
        cw74, s74 = hamming74_encode(q), sc
        # corrupt a few codewords to exercise the decode path
        cwn = cw84.clone()
        flat = cwn.view(-1)
        flat[::7] ^= 0x01
        flat[::11] ^= 0x03
        out, ncorr = fused_decode_dequantize_hamming84(cwn, s84)
        arrays[f"c{i}_x"] = x.numpy()
        arrays[f"c{i}_cw84"] = cw84.numpy()
        arrays[f"c{i}_s84"] = s84.numpy()
        arrays[f"c{i}_cw74"] = cw74.numpy()
        arrays[f"c{i}_s74"] = s74.numpy()
        arrays[f"c{i}_torch_q"] = q.numpy()
        arrays[f"c{i}_torch_scale"] = sc.numpy()
        arrays[f"c{i}_cw_noisy"] = cwn.numpy()
        arrays[f"c{i}_dq"] = out.numpy()
        arrays[f"c{i}_ncorr"] = np.array([ncorr], dtype=np.int64)
        params.append({"rows": rows, "d": d})
    _save("fused", manifest, {"cases": params}, **arrays)


def gen_shim(manifest):
    """End-to-end shim on an offline random-init 2-layer GPT-2 (ecc_shim.py)."""
    import torch
    from transformers import GPT2Config, GPT2LMHeadModel
    from kv_cache.ecc_shim import (ECCShimConfig, patch_model_with_ecc_attention,
                                   reset_ecc_cache, get_ecc_stats)
    torch.manual_seed(0)
    cfg = GPT2Config(n_layer=2, n_head=4, n_embd=64, n_positions=64, vocab_size=97)
    model = GPT2LMHeadModel(cfg).eval()
    state = {k: v.clone() for k, v in model.state_dict().items()}
    ids = torch.randint(0, 97, (1, 24), generator=torch.Generator().manual_seed(3))
    arrays = {"input_ids": ids.numpy()}
    for k, v in state.items():
        arrays["w_" + k.replace(".", "__")] = v.numpy()
    params = []
    runs = [("hamming84", 0.0, False), ("hamming84", 1e-2, False), ("hamming84", 5e-2, True),
            ("hamming74", 5e-2, False), ("golay", 5e-2, False), ("int4", 5e-2, False),
            ("fp16", 0.0, False)]
    for i, (codec, ber, interp) in enumerate(runs):
        sc = ECCShimConfig(codec=codec, ber=ber, inject_errors=ber > 0, seed=42,
                           block_size=16, use_interpolation=interp)
        t0 = time.time()
        with torch.no_grad(), patch_model_with_ecc_attention(model, sc, num_blocks=16):
            reset_ecc_cache(model)
            out = model(ids)
            st = get_ecc_stats(model)
        arrays[f"r{i}_logits"] = out.logits.float().numpy()
        params.append({"codec": codec, "ber": ber, "use_interpolation": interp,
                       "stats": {k: int(v) for k, v in st.items()}})
        print(f"    shim {codec} ber={ber} interp={interp}: {st} ({time.time() - t0:.1f}s)")
    _save("shim_gpt2", manifest, {"model": cfg.to_dict(), "runs": params, "seq_len": 24}, **arrays)


def gen_shim_fp16(manifest):
    """SURVEY config 4 in its own dtype: the reference shim on an offline
    random-init fp16 GPT-2 (2 layers, head_dim 32, 40 tokens = 2.5 blocks of 16),
    Hamming(8,4) + interpolation at BER 1e-2 and 1e-3, and Golay at 1e-2.  Besides
    logits and get_ecc_stats() it records, per layer, what ECCBackend.write was
    given (the fp16 K/V projections) and the dequantized K/V that attend handed
    to _run_attention (fp32 (q - 8) * scale, ecc_shim.py:1067-1071, before its
    .to(q.dtype)), so the decode -> interpolate -> dequantize data path can be
    pinned bit for bit, not only through the statistics."""
    import torch
    from transformers import GPT2Config, GPT2LMHeadModel
    import kv_cache.ecc_shim as es
    torch.manual_seed(1)
    cfg = GPT2Config(n_layer=2, n_head=2, n_embd=64, n_positions=64, vocab_size=97)
    model = GPT2LMHeadModel(cfg).eval().half()
    ids = torch.randint(0, 97, (1, 40), generator=torch.Generator().manual_seed(5))
    arrays = {"input_ids": ids.numpy()}
    for k, v in model.state_dict().items():
        arrays["w_" + k.replace(".", "__")] = v.numpy()
    rec = {"write": [], "kv": []}
    orig_write, orig_run = es.ECCBackend.write, es.ECCBackend._run_attention

    def write(self, k, v, layer_idx, seq_id=0):
        rec["write"].append((layer_idx, k.detach().clone(), v.detach().clone()))
        return orig_write(self, k, v, layer_idx, seq_id)

    def run_attention(self, q, k_float, v_float, device):
        rec["kv"].append((k_float.detach().clone(), v_float.detach().clone()))
        return orig_run(self, q, k_float, v_float, device)

    es.ECCBackend.write, es.ECCBackend._run_attention = write, run_attention
    params = []
    try:
        runs = [("hamming84", 1e-2, True), ("hamming84", 1e-3, True), ("golay", 1e-2, False)]
        for i, (codec, ber, interp) in enumerate(runs):
            rec["write"].clear()
            rec["kv"].clear()
            sc = es.ECCShimConfig(codec=codec, ber=ber, inject_errors=ber > 0, seed=42,
                                  block_size=16, use_interpolation=interp)
            t0 = time.time()
            with torch.no_grad(), es.patch_model_with_ecc_attention(model, sc, num_blocks=16):
                es.reset_ecc_cache(model)
                out = model(ids)
                st = es.get_ecc_stats(model)
            assert out.logits.dtype == torch.float16
            arrays[f"r{i}_logits"] = out.logits.numpy()
            assert len(rec["write"]) == len(rec["kv"]) == cfg.n_layer
            for (layer, k, v), (kf, vf) in zip(rec["write"], rec["kv"]):
                assert k.dtype == torch.float16 and kf.dtype == torch.float32
                arrays[f"r{i}_l{layer}_k_in"] = k.numpy()
                arrays[f"r{i}_l{layer}_v_in"] = v.numpy()
                arrays[f"r{i}_l{layer}_k_deq"] = kf.numpy()
                arrays[f"r{i}_l{layer}_v_deq"] = vf.numpy()
            params.append({"codec": codec, "ber": ber, "use_interpolation": interp,
                           "stats": {k: int(v) for k, v in st.items()}})
            print(f"    shim fp16 {codec} ber={ber} interp={interp}: {st} ({time.time() - t0:.1f}s)")
    finally:
        es.ECCBackend.write, es.ECCBackend._run_attention = orig_write, orig_run
    _save("shim_gpt2_fp16", manifest, {"model": cfg.to_dict(), "runs": params, "seq_len": 40,
                                       "dtype": "float16"}, **arrays)


def gen_attention(manifest):
    """Pin paged_attention_ecc (kv_cache/attention_ecc.py:620-780).

    hamming84 runs the reference's ``paged_attention_ecc_kernel`` (:264-427)
    under the interpreter; golay runs its Python ``reference_attention_ecc``
    (:783-909) through the interpreted golay_decode.  Cases cover what the
    reference's own tests leave at "shape only": empty contexts (H84 -> -8.0 in
    every lane, golay -> zeros), -1 blocks before and after valid ones, a
    table of only -1 blocks, head_dim 100 (BLOCK_HEAD_DIM 128), v_scales=None,
    an fp16 query, and random (mostly noisy) codewords so every decode branch
    runs.  No GQA: the reference indexes cache head = query head.
    """
    import torch
    from ecc_codecs.triton_kernels import golay_encode
    from kv_cache.attention_ecc import paged_attention_ecc
    rng = np.random.default_rng(2024)
    arrays = {}
    params = []

    def golay_cache(shape, g):
        # codewords of random data with 0..4 random bit errors (every decode outcome)
        m = int(np.prod(shape[:-1])) * shape[-1]
        data = rng.integers(0, 4096, size=m, dtype=np.int64)
        trip = np.stack([data & 15, (data >> 4) & 15, (data >> 8) & 15], 1).astype(np.uint8)
        cw = golay_encode(torch.from_numpy(trip)).numpy().astype(np.int64)
        nerr = rng.integers(0, 5, size=m)
        for i in range(m):
            for b in rng.choice(24, size=nerr[i], replace=False):
                cw[i] ^= 1 << int(b)
        return cw.astype(np.int32).reshape(shape)

    cases = [
        # name, codec, batch, heads, d, layers, layer, bs, nblocks, table, ctx, qdtype, v_scales
        ("h84_basic", "hamming84", 2, 2, 32, 2, 1, 4, 8, [[3, 0, 6, -1], [5, 1, 2, 7]], [13, 16],
         "f32", True),
        ("h84_empty", "hamming84", 2, 2, 32, 1, 0, 4, 6, [[0, 1, -1, -1], [2, 3, -1, -1]], [0, 6],
         "f32", True),
        ("h84_holes", "hamming84", 2, 3, 32, 2, 0, 4, 8, [[-1, 3, 5, -1], [4, -1, 0, 2]], [16, 15],
         "f32", True),
        ("h84_all_missing", "hamming84", 1, 2, 16, 1, 0, 4, 3, [[-1, -1, -1]], [9], "f32", True),
        ("h84_d100", "hamming84", 1, 2, 100, 1, 0, 4, 4, [[2, 0, 3]], [10], "f32", True),
        ("h84_vscales_none", "hamming84", 2, 2, 64, 2, 1, 4, 6, [[1, 4, -1], [0, 5, 2]], [7, 12],
         "f32", False),
        ("h84_fp16", "hamming84", 1, 4, 64, 1, 0, 4, 4, [[3, 1, 0]], [11], "f16", True),
        ("golay_basic", "golay", 2, 2, 64, 2, 1, 4, 6, [[2, 0, 5], [1, 4, 3]], [9, 12], "f32", True),
        ("golay_empty_holes", "golay", 2, 2, 32, 1, 0, 4, 6, [[0, 1, -1], [-1, 3, 2]], [0, 11],
         "f32", True),
        ("golay_d100", "golay", 1, 2, 100, 1, 0, 4, 4, [[1, 3, 0]], [12], "f32", True),
    ]
    # use_tiled=True (:430-617, taken when block_size >= block_m, :693): the
    # tiled kernel masks the normaliser with token_valid and returns 0 for a
    # context with no valid token, where the default kernel gives -8.0.
    # (Appended after the cases above, so their random inputs are unchanged.)
    tiled = {"h84_tiled_empty": 4, "h84_tiled_holes": 4, "h84_tiled_all_missing": 2,
             "h84_tiled_small_block": 4}
    cases += [
        ("h84_tiled_empty", "hamming84", 2, 2, 32, 1, 0, 4, 6, [[0, 1, -1, -1], [2, 3, -1, -1]], [0, 6],
         "f32", True),
        ("h84_tiled_holes", "hamming84", 2, 3, 32, 2, 0, 8, 8, [[-1, 3, 5, -1], [4, -1, 0, 2]], [30, 29],
         "f32", True),
        ("h84_tiled_all_missing", "hamming84", 1, 2, 16, 1, 0, 4, 3, [[-1, -1, -1]], [9], "f32", True),
        # block_size 2 < block_m 4: the default kernel runs (empty -> -8.0)
        ("h84_tiled_small_block", "hamming84", 2, 2, 16, 1, 0, 2, 4, [[-1, -1], [1, 3]], [3, 4], "f32", True),
    ]
    for (name, codec, batch, heads, d, layers, layer, bs, nblocks, table, ctx, qdt,
         with_vs) in cases:
        per = d if codec == "hamming84" else (d + 2) // 3
        shape = (nblocks, layers, heads, bs * per)
        if codec == "hamming84":
            kc = rng.integers(0, 256, size=shape, dtype=np.int64).astype(np.uint8)
            vc = rng.integers(0, 256, size=shape, dtype=np.int64).astype(np.uint8)
        else:
            kc, vc = golay_cache(shape, per), golay_cache(shape, per)
        ks = (rng.random((nblocks, layers, heads, bs)) * 0.3 + 0.05).astype(np.float32)
        vs = (rng.random((nblocks, layers, heads, bs)) * 0.3 + 0.05).astype(np.float32)
        q = rng.standard_normal((batch, heads, d)).astype(np.float32)
        if qdt == "f16":
            q = q.astype(np.float16)
        tab = np.array(table, dtype=np.int32)
        lens = np.array(ctx, dtype=np.int32)
        out = paged_attention_ecc(torch.from_numpy(q), torch.from_numpy(kc), torch.from_numpy(vc),
                                  torch.from_numpy(tab), torch.from_numpy(lens), torch.from_numpy(ks),
                                  layer, bs, codec=codec,
                                  v_scales=torch.from_numpy(vs) if with_vs else None,
                                  use_tiled=name in tiled, block_m=tiled.get(name, 4))
        for k, v in (("q", q), ("k_cache", kc), ("v_cache", vc), ("block_table", tab),
                     ("context_lens", lens), ("k_scales", ks), ("v_scales", vs),
                     ("out", out.numpy())):
            arrays[f"{name}_{k}"] = v
        params.append({"name": name, "codec": codec, "layer": layer, "block_size": bs,
                       "v_scales": with_vs, "q_dtype": qdt, "out_dtype": str(out.dtype),
                       "use_tiled": name in tiled, "block_m": tiled.get(name, 4)})
        print(f"    {name}: out {tuple(out.shape)} {out.dtype}, "
              f"range [{float(out.min()):.4f}, {float(out.max()):.4f}]")
    _save("attention", manifest, {"cases": params}, **arrays)


GENERATORS = {"hamming": gen_hamming, "golay": gen_golay, "inject": gen_inject,
              "interp": gen_interp, "fused": gen_fused, "shim": gen_shim, "shim_fp16": gen_shim_fp16,
              "attention": gen_attention}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    if __debug__:
        sys.exit("run with `python -O` (the reference wrappers assert is_cuda)")
    sys.path.insert(0, args.ref)
    os.makedirs(OUT, exist_ok=True)
    mpath = os.path.join(OUT, "MANIFEST.json")
    manifest = {}
    if os.path.exists(mpath):
        with open(mpath) as f:
            manifest = json.load(f)
    for name, fn in GENERATORS.items():
        if args.only and name not in args.only:
            continue
        print(f"[{name}]")
        t0 = time.time()
        fn(manifest)
        print(f"  done in {time.time() - t0:.1f}s")
    manifest["_generator"] = {"script": "tools/gen_golden.py", "mode": "TRITON_INTERPRET=1",
                              "reference_snapshot": "2026-01-28"}
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
