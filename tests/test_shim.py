"""The ECC shim (patch_model_with_ecc_attention) against the reference's run.

tests/golden/shim_gpt2.npz holds the reference shim's logits and
get_ecc_stats() for a random-init 2-layer GPT-2 (weights stored in the
fixture) at seq_len 24, for each codec (tools/gen_golden.py:gen_shim).
Statistics must match exactly (they depend only on the bits of the cache);
logits are float outputs of HF matmuls + SDPA and are compared with a
tolerance (GPU vs CPU summation order).
"""

import numpy as np
import pytest
import torch

LOGIT_ATOL = 2e-3
LOGIT_RTOL = 2e-3


def test_config_validation():
    from kvecc.ecc_shim import ECCShimConfig
    with pytest.raises(ValueError):
        ECCShimConfig(codec="reed-solomon")
    c = ECCShimConfig(codec="golay", ber=1e-3, backend="hip")
    assert c.backend == "hip" and c.block_size == 16 and c.seed == 42
    assert c.golay_storage == "int32"
    with pytest.raises(ValueError):
        ECCShimConfig(codec="golay", golay_storage="int24")
    with pytest.raises(ValueError):
        ECCShimConfig(codec="golay", golay_storage="packed", fused=False)


def test_block_manager_layout_cpu():
    from kvecc.ecc_shim import SimpleBlockManager
    m = SimpleBlockManager(8, 16, 3, 4, 128, device="cpu", codec="golay")
    assert m.k_cache.shape == (8, 3, 4, 16 * 43) and m.k_cache.dtype == torch.int32
    mp = SimpleBlockManager(8, 16, 3, 4, 128, device="cpu", codec="golay", golay_storage="packed")
    assert mp.k_cache.shape == (8, 3, 4, 16 * 132) and mp.k_cache.dtype == torch.uint8
    assert mp.shim_codec == "golay_packed" and m.shim_codec == "golay"
    mp = SimpleBlockManager(8, 16, 3, 4, 64, device="cpu", codec="golay", golay_storage="packed")
    assert mp.k_cache.shape == (8, 3, 4, 16 * 68)  # 22 codewords = 66 B, padded to 68
    m2 = SimpleBlockManager(8, 16, 3, 4, 64, device="cpu", codec="hamming84")
    assert m2.k_cache.shape == (8, 3, 4, 16 * 64) and m2.k_scales.shape == (8, 3, 4, 16)
    m2.allocate(0, 40)
    assert m2.block_table[0, :3].tolist() == [0, 1, 2] and m2.get_context_len(0) == 40
    blk, slot = m2.slots(0, 40)
    assert blk.tolist() == [0] * 16 + [1] * 16 + [2] * 8 and slot[17].item() == 1
    with pytest.raises(RuntimeError):
        m2.allocate(1, 16 * 6)
    m2.reset()
    assert len(m2.free_blocks) == 8 and int(m2.block_table.max()) == -1


def _model(golden, manifest, device):
    from transformers import GPT2Config, GPT2LMHeadModel
    g = golden("shim_gpt2")
    cfg = GPT2Config(**{k: v for k, v in manifest["shim_gpt2"]["params"]["model"].items()
                        if k in ("n_layer", "n_head", "n_embd", "n_positions", "vocab_size")})
    model = GPT2LMHeadModel(cfg).eval()
    state = {k[2:].replace("__", "."): torch.from_numpy(v) for k, v in g.items()
             if k.startswith("w_")}
    model.load_state_dict(state, strict=True)
    return model.to(device), torch.from_numpy(g["input_ids"]).to(device), g


def _shim_matches_reference(device, backend, golden, manifest, golay_storage="int32"):
    from kvecc.ecc_shim import (ECCShimConfig, get_ecc_stats, patch_model_with_ecc_attention,
                                reset_ecc_cache)
    model, ids, g = _model(golden, manifest, device)
    runs = list(enumerate(manifest["shim_gpt2"]["params"]["runs"]))
    if golay_storage != "int32":
        runs = [(i, r) for i, r in runs if r["codec"] == "golay"]
        assert runs
    for i, run in runs:
        # the fixtures come from the reference run on CPU tensors: IEEE scale division
        cfg = ECCShimConfig(codec=run["codec"], ber=run["ber"], inject_errors=run["ber"] > 0,
                            seed=42, block_size=16, use_interpolation=run["use_interpolation"],
                            backend=backend, scale_rule="div7", golay_storage=golay_storage)
        with torch.no_grad(), patch_model_with_ecc_attention(model, cfg, num_blocks=16):
            reset_ecc_cache(model)
            out = model(ids)
            st = get_ecc_stats(model)
        assert st == run["stats"], (run["codec"], st, run["stats"])
        ref = g[f"r{i}_logits"]
        got = out.logits.float().cpu().numpy()
        assert np.allclose(got, ref, atol=LOGIT_ATOL, rtol=LOGIT_RTOL), \
            (run["codec"], float(np.abs(got - ref).max()))


@pytest.mark.gpu
def test_shim_gpt2_matches_reference(gpu, golden, manifest):
    _shim_matches_reference(gpu, "hip", golden, manifest)


def test_shim_gpt2_matches_reference_cpu_backend(golden, manifest):
    """The same end-to-end run on the host backend (model and cache on the CPU)."""
    _shim_matches_reference(torch.device("cpu"), "cpu", golden, manifest)


def test_shim_gpt2_packed_golay_matches_reference_cpu_backend(golden, manifest):
    """The packed Golay cache layout reproduces the reference shim's Golay runs
    (statistics exactly, logits within the float tolerance)."""
    _shim_matches_reference(torch.device("cpu"), "cpu", golden, manifest, golay_storage="packed")


@pytest.mark.gpu
def test_shim_gpt2_packed_golay_matches_reference(gpu, golden, manifest):
    _shim_matches_reference(gpu, "hip", golden, manifest, golay_storage="packed")


def _cache_bits_match_oracle(gpu, backend):
    from oracle import oracle
    from kvecc.ecc_shim import ECCBackend, ECCShimConfig, SimpleBlockManager
    torch.manual_seed(0)
    b, s, hk, d = 2, 20, 3, 64
    for codec, nb in (("hamming84", 8), ("golay", 24), ("hamming74", 7), ("int4", 4)):
        cfg = ECCShimConfig(codec=codec, ber=0.05, inject_errors=True, seed=7, backend=backend)
        mgr = SimpleBlockManager(4, 16, 2, hk, d, device=gpu, codec=codec)
        be = ECCBackend(mgr, cfg, num_heads=hk)
        k = torch.randn(b, s, hk * d, device=gpu, dtype=torch.float16)
        v = torch.randn(b, s, hk * d, device=gpu, dtype=torch.float16)
        be._injection_count = 5
        be.write(k, v, layer_idx=1)
        assert be._injection_count == 5 + b * s * hk
        for which, x, cache in ((0, k, mgr.k_cache), (1, v, mgr.v_cache)):
            # default scale rule: the reference on this backend's device
            q, _ = oracle.quantize_rows(x.float().cpu().numpy().reshape(b, s, hk, d),
                                        rule=1 if backend == "hip" else 0)
            last = q[-1]  # last batch wins
            for pos in range(s):
                for h in range(hk):
                    r = ((b - 1) * s + pos) * hk + h
                    row = last[pos, h]
                    if codec == "golay":
                        pad = np.zeros(66, np.uint8)
                        pad[:d] = row
                        enc = oracle.golay_encode(pad.reshape(-1, 3))
                    elif codec == "hamming84":
                        enc = oracle.hamming84_encode(row)
                    elif codec == "hamming74":
                        enc = oracle.hamming74_encode(row)
                    else:
                        enc = row
                    exp, _, _ = oracle.inject(enc, 0.05, nb, 7 + 5 + r + which)
                    blk, slot = pos // 16, pos % 16
                    per = exp.size
                    got = cache[blk, 1, h, slot * per:(slot + 1) * per].cpu().numpy()
                    assert np.array_equal(got, exp), (codec, which, pos, h)


@pytest.mark.gpu
def test_shim_cache_bits_match_oracle(gpu):
    """Cache codewords after one write equal the reference loop restated with
    the oracle: quantize rows, encode, per-row seeds (K: s+r, V: s+r+1)."""
    _cache_bits_match_oracle(gpu, "hip")


def test_shim_cache_bits_match_oracle_cpu_backend():
    _cache_bits_match_oracle(torch.device("cpu"), "cpu")


def _fused_equals_composed(device, backend):
    """The one-launch write/read (shim.hip / its host twin) leaves the same cache
    bits and scales, returns the same attention output and counts the same
    statistics as the per-op composition, for every fused codec."""
    from kvecc.ecc_shim import ECCBackend, ECCShimConfig, SimpleBlockManager
    torch.manual_seed(1)
    cases = [("hamming84", True, 64, torch.float16), ("hamming84", False, 128, torch.float32),
             ("hamming74", False, 64, torch.bfloat16), ("golay", False, 128, torch.float16),
             ("golay", False, 100, torch.float32), ("int4", False, 64, torch.float16)]
    for codec, interp, d, dt in cases:
        b, s, hk, nh = 2, 37, 2, 4  # GQA: 2 query heads per cache head
        res = []
        for fused in (True, False):
            cfg = ECCShimConfig(codec=codec, ber=0.02, inject_errors=True, seed=11,
                                use_interpolation=interp, backend=backend)
            mgr = SimpleBlockManager(6, 16, 3, hk, d, device=device, codec=codec)
            be = ECCBackend(mgr, cfg, num_heads=nh, fused=fused)
            g = torch.Generator().manual_seed(3)
            k = torch.randn(b, s, hk * d, generator=g).to(device=device, dtype=dt)
            v = torch.randn(b, s, hk * d, generator=g).to(device=device, dtype=dt)
            q = torch.randn(b, nh, s, d, generator=g).to(device=device, dtype=dt)
            be._injection_count = 9
            be.write(k, v, layer_idx=2)
            out = be.attend(q, layer_idx=2)
            q1 = q[:, :, :1]
            out1 = be.attend(q1, layer_idx=2)  # seq_len==1 path
            res.append((mgr.k_cache.cpu(), mgr.v_cache.cpu(), mgr.k_scales.cpu(),
                        mgr.v_scales.cpu(), out.float().cpu(), out1.float().cpu(),
                        be._injection_count, be._errors_corrected, be._errors_detected))
        f, c = res
        for i in range(4):
            assert torch.equal(f[i], c[i]), (codec, d, i)
        assert f[6:] == c[6:], (codec, f[6:], c[6:])
        assert codec == "int4" or f[7] > 0, codec  # errors were injected and corrected
        assert torch.allclose(f[4], c[4], atol=1e-3, rtol=1e-3), codec
        assert torch.allclose(f[5], c[5], atol=1e-3, rtol=1e-3), codec


def test_fused_equals_composed_cpu_backend():
    _fused_equals_composed(torch.device("cpu"), "cpu")


@pytest.mark.gpu
def test_fused_equals_composed(gpu):
    _fused_equals_composed(gpu, "hip")


@pytest.mark.gpu
@pytest.mark.parametrize("rule", ["div7", "mul_inv7"])
def test_hip_and_cpu_backends_write_identical_caches(gpu, rule):
    """Under either scale rule the two backends write the same cache bytes and
    scales and read back the same dequantized K/V and statistics (fp16, fp32
    and bf16 models; every fused codec; injection on)."""
    from kvecc.ecc_shim import ECCBackend, ECCShimConfig, SimpleBlockManager
    cases = [("hamming84", True, 64, torch.float16), ("hamming74", False, 128, torch.float32),
             ("golay", False, 128, torch.bfloat16), ("golay", False, 100, torch.float16),
             ("int4", False, 64, torch.float32)]
    for codec, interp, d, dt in cases:
        b, s, hk = 2, 29, 3
        g = torch.Generator().manual_seed(d)
        k = (torch.randn(b, s, hk * d, generator=g) * 2).to(dt)
        v = (torch.randn(b, s, hk * d, generator=g) * 2).to(dt)
        res = []
        for backend, dev in (("hip", gpu), ("cpu", torch.device("cpu"))):
            cfg = ECCShimConfig(codec=codec, ber=0.02, inject_errors=True, seed=5,
                                use_interpolation=interp, backend=backend, scale_rule=rule)
            mgr = SimpleBlockManager(4, 16, 2, hk, d, device=dev, codec=codec)
            be = ECCBackend(mgr, cfg, num_heads=hk)
            be.write(k.to(dev), v.to(dev), layer_idx=1)
            k_t, v_t = be.codec_backend.shim_read(mgr, 1, s, codec, interp, torch.float32, be._stats)
            res.append((mgr.k_cache.cpu(), mgr.v_cache.cpu(), mgr.k_scales.cpu(),
                        mgr.v_scales.cpu(), k_t.cpu(), v_t.cpu(),
                        be.codec_backend.read_stats(be._stats, 2)))
        hip, cpu = res
        for i in range(6):
            assert torch.equal(hip[i], cpu[i]), (codec, rule, i)
        assert hip[6] == cpu[6], (codec, rule)


@pytest.mark.gpu
def test_strided_write_equals_contiguous(gpu):
    """kvecc_shim_write_strided reads the projections' views in place: a slice of
    a fused [b, s, 3*hidden] QKV output (GPT-2) and a transposed [b, h, s, d]
    tensor (Llama after RoPE) leave the same cache bytes and scales as the
    reference's .transpose(1, 2).contiguous() copies (ecc_shim.py:1290-1291)."""
    from kvecc import ops
    from kvecc.ecc_shim import SimpleBlockManager
    b, s, hk, d = 3, 37, 4, 64
    for codec, nb in (("hamming84", 8), ("golay", 24), ("int4", 4)):
        g = torch.Generator().manual_seed(nb)
        qkv = torch.randn(b, s, 3 * hk * d, generator=g).to(gpu, torch.float16)
        _, k, v = qkv.split(hk * d, dim=2)                      # GPT-2: strided slices
        kh = k.view(b, s, hk, d).transpose(1, 2).contiguous()   # Llama: [b, h, s, d]
        variants = {"contiguous": (k.contiguous(), v.contiguous()),
                    "qkv_slice": (k, v),
                    "heads_first": (kh.transpose(1, 2), v.view(b, s, hk, d))}
        res = {}
        for name, (kk, vv) in variants.items():
            mgr = SimpleBlockManager(4, 16, 2, hk, d, device=gpu, codec=codec)
            mgr.allocate(0, s)
            ops.shim_write(kk, vv, mgr, 1, codec, nb, True, 0.03, 17)
            res[name] = (mgr.k_cache.cpu(), mgr.v_cache.cpu(), mgr.k_scales.cpu(), mgr.v_scales.cpu())
        for name in ("qkv_slice", "heads_first"):
            for i in range(4):
                assert torch.equal(res[name][i], res["contiguous"][i]), (codec, name, i)
        assert res["contiguous"][2].abs().sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("codec,interp", [("hamming84", True), ("golay", False), ("golay_packed", False)])
def test_patched_forward_replays_in_a_hip_graph(gpu, codec, interp):
    """The whole patched forward (cache reset included) captures in one HIP graph:
    no host sync or host-to-device copy in a steady-state forward.  Replays give
    the eager forward's logits and ECC statistics (same seeds: the reset restarts
    the injection counter, as the reference's per-text reset does)."""
    from transformers import GPT2Config, GPT2LMHeadModel
    from kvecc.ecc_shim import (ECCShimConfig, get_ecc_stats, patch_model_with_ecc_attention,
                                reset_ecc_cache)
    torch.manual_seed(0)
    cfg_m = GPT2Config(n_layer=2, n_head=4, n_embd=256, n_positions=128)
    model = GPT2LMHeadModel(cfg_m).half().to(gpu).eval()
    ids = torch.randint(0, cfg_m.vocab_size, (1, 96), generator=torch.Generator().manual_seed(1)).to(gpu)
    storage = "packed" if codec == "golay_packed" else "int32"
    cfg = ECCShimConfig(codec=codec.replace("_packed", ""), ber=1e-2, inject_errors=True, seed=42,
                        block_size=16, use_interpolation=interp, golay_storage=storage)
    with torch.no_grad(), patch_model_with_ecc_attention(model, cfg, num_blocks=6):
        def fwd():
            reset_ecc_cache(model)
            return model(ids).logits
        eager = fwd().clone()
        eager_stats = get_ecc_stats(model)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                fwd()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = fwd()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
        st = get_ecc_stats(model)
        assert st["errors_corrected"] == eager_stats["errors_corrected"] > 0
        assert st["errors_detected"] == eager_stats["errors_detected"]


def _packed_equals_int32(device, backend):
    """golay_storage="packed" keeps the low 3 bytes of every int32 codeword the
    reference layout stores (row padding zero), the same scales, and reads back
    the same attention outputs and statistics (prefill and seq_len==1)."""
    from kvecc.ecc_shim import ECCBackend, ECCShimConfig, SimpleBlockManager
    for d, dt in ((128, torch.float16), (100, torch.float32), (64, torch.bfloat16), (7, torch.float16)):
        b, s, hk, nh = 2, 37, 2, 4
        res = {}
        for storage in ("int32", "packed"):
            cfg = ECCShimConfig(codec="golay", ber=0.02, inject_errors=True, seed=11,
                                backend=backend, golay_storage=storage)
            mgr = SimpleBlockManager(6, 16, 3, hk, d, device=device, codec="golay",
                                     golay_storage=storage)
            be = ECCBackend(mgr, cfg, num_heads=nh)
            g = torch.Generator().manual_seed(d)
            k = torch.randn(b, s, hk * d, generator=g).to(device=device, dtype=dt)
            v = torch.randn(b, s, hk * d, generator=g).to(device=device, dtype=dt)
            q = torch.randn(b, nh, s, d, generator=g).to(device=device, dtype=dt)
            be.write(k, v, layer_idx=2)
            out = be.attend(q, layer_idx=2)
            out1 = be.attend(q[:, :, :1], layer_idx=2)
            res[storage] = (mgr, out.float().cpu(), out1.float().cpu(), be._errors_corrected,
                            be._errors_detected)
        m32, mpk = res["int32"][0], res["packed"][0]
        gw = (d + 2) // 3
        row = (3 * gw + 3) // 4 * 4
        for c32, cpk in ((m32.k_cache, mpk.k_cache), (m32.v_cache, mpk.v_cache)):
            w = m32.view5(c32).cpu().numpy().astype(np.uint32)           # [..., gw]
            exp = np.zeros(w.shape[:-1] + (row,), np.uint8)
            for byte in range(3):
                exp[..., byte:3 * gw:3] = (w >> (8 * byte)) & 0xFF
            assert np.array_equal(mpk.view5(cpk).cpu().numpy(), exp), d
        assert torch.equal(m32.k_scales.cpu(), mpk.k_scales.cpu())
        assert torch.equal(m32.v_scales.cpu(), mpk.v_scales.cpu())
        assert res["int32"][3:] == res["packed"][3:] and res["int32"][3] > 0, d
        assert torch.equal(res["int32"][1], res["packed"][1]), d
        assert torch.equal(res["int32"][2], res["packed"][2]), d


def test_golay_packed_storage_cpu_backend():
    _packed_equals_int32(torch.device("cpu"), "cpu")


@pytest.mark.gpu
def test_golay_packed_storage(gpu):
    _packed_equals_int32(gpu, "hip")


@pytest.mark.gpu
def test_golay_packed_storage_hip_equals_cpu(gpu):
    """The HIP and host shim kernels write the same packed cache bytes and read
    back the same K/V and statistics."""
    from kvecc.ecc_shim import ECCBackend, ECCShimConfig, SimpleBlockManager
    for d, dt in ((128, torch.bfloat16), (100, torch.float16), (5, torch.float32)):
        b, s, hk = 2, 29, 3
        g = torch.Generator().manual_seed(d)
        k = (torch.randn(b, s, hk * d, generator=g) * 2).to(dt)
        v = (torch.randn(b, s, hk * d, generator=g) * 2).to(dt)
        res = []
        for backend, dev in (("hip", gpu), ("cpu", torch.device("cpu"))):
            cfg = ECCShimConfig(codec="golay", ber=0.02, inject_errors=True, seed=5,
                                backend=backend, scale_rule="div7", golay_storage="packed")
            mgr = SimpleBlockManager(4, 16, 2, hk, d, device=dev, codec="golay",
                                     golay_storage="packed")
            be = ECCBackend(mgr, cfg, num_heads=hk)
            be.write(k.to(dev), v.to(dev), layer_idx=1)
            k_t, v_t = be.codec_backend.shim_read(mgr, 1, s, mgr.shim_codec, False, torch.float32,
                                                  be._stats)
            res.append((mgr.k_cache.cpu(), mgr.v_cache.cpu(), mgr.k_scales.cpu(),
                        mgr.v_scales.cpu(), k_t.cpu(), v_t.cpu(),
                        be.codec_backend.read_stats(be._stats, 2)))
        hip, cpu = res
        for i in range(6):
            assert torch.equal(hip[i], cpu[i]), (d, i)
        assert hip[6] == cpu[6] and hip[6][0] > 0, d


@pytest.mark.gpu
def test_config4_full_size_hip_equals_cpu_backend(gpu):
    """BASELINE config 4 at its size: random-init GPT-2 (12 layers, 12 heads,
    768 hidden) over seq_len 1024 inside patch_model_with_ecc_attention,
    Hamming(8,4) + interpolation, BER 1e-3 (ecc_shim.py:1396-1481, stats
    :1627-1642).  fp32 model on both backends with one scale rule, so both
    write the same cache bytes: get_ecc_stats must be equal and the logits
    agree to fp32 matmul rounding (GPU vs host GEMMs)."""
    from transformers import GPT2Config, GPT2LMHeadModel
    from kvecc.ecc_shim import ECCShimConfig, get_ecc_stats, patch_model_with_ecc_attention, reset_ecc_cache
    torch.manual_seed(0)
    cpu_model = GPT2LMHeadModel(GPT2Config(n_positions=1024)).eval()
    gpu_model = GPT2LMHeadModel(GPT2Config(n_positions=1024)).eval()
    gpu_model.load_state_dict(cpu_model.state_dict())
    gpu_model = gpu_model.to(gpu)
    ids = torch.randint(0, 50257, (1, 1024), generator=torch.Generator().manual_seed(0))
    res = {}
    for backend, model, dev in (("hip", gpu_model, gpu), ("cpu", cpu_model, torch.device("cpu"))):
        cfg = ECCShimConfig(codec="hamming84", ber=1e-3, inject_errors=True, seed=42, block_size=16,
                            use_interpolation=True, backend=backend, scale_rule="div7")
        with torch.no_grad(), patch_model_with_ecc_attention(model, cfg, num_blocks=64):
            reset_ecc_cache(model)
            out = model(ids.to(dev), labels=ids.to(dev))
            res[backend] = (out.logits.float().cpu(), float(out.loss), get_ecc_stats(model))
    (lh, loss_h, st_h), (lc, loss_c, st_c) = res["hip"], res["cpu"]
    assert st_h == st_c, (st_h, st_c)
    assert st_h["errors_corrected"] > 0 and st_h["errors_detected"] > 0
    assert torch.allclose(lh, lc, rtol=1e-3, atol=1e-3), float((lh - lc).abs().max())
    assert abs(loss_h - loss_c) < 1e-3 * max(1.0, abs(loss_c))
