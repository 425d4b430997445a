"""The shim on a LLaMA-architecture model (RoPE, GQA: 4 query heads over 2 KV
heads), after the reference's TestPatchModelWithECCAttention
(tests/test_ecc_shim.py:310-445), which loads TinyLlama from the hub; here a
random-init LlamaForCausalLM (no network)."""

import pytest
import torch

LOGIT_ATOL = 2e-3


def _llama():
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=101, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128)
    return LlamaForCausalLM(cfg).eval(), torch.randint(0, 101, (1, 20),
                                                       generator=torch.Generator().manual_seed(1))


def _run(model, ids, backend, codec, ber, interp=False):
    from kvecc.ecc_shim import (ECCShimConfig, get_ecc_stats, patch_model_with_ecc_attention,
                                reset_ecc_cache)
    cfg = ECCShimConfig(codec=codec, ber=ber, inject_errors=ber > 0, seed=42, backend=backend,
                        use_interpolation=interp)
    with torch.no_grad(), patch_model_with_ecc_attention(model, cfg, num_blocks=16):
        reset_ecc_cache(model)
        logits = model(ids).logits.float()
        return logits, get_ecc_stats(model)


def test_patch_replace_restore_and_rope_cpu():
    from kvecc.ecc_shim import ECCPagedAttentionShim, ECCShimConfig, patch_model_with_ecc_attention
    model, ids = _llama()
    orig_type = type(model.model.layers[0].self_attn)
    with torch.no_grad():
        ref = model(ids).logits
    with patch_model_with_ecc_attention(model, ECCShimConfig(codec="hamming84", backend="cpu"),
                                        num_blocks=16):
        assert isinstance(model.model.layers[0].self_attn, ECCPagedAttentionShim)
    assert type(model.model.layers[0].self_attn) is orig_type
    # fp16 storage: only fp16 rounding of K/V, so RoPE and GQA must match the model exactly-ish
    out, _ = _run(model, ids, "cpu", "fp16", 0.0)
    assert torch.allclose(out, ref, atol=1e-3)
    for codec in ("hamming84", "golay", "int4"):  # INT4 quantization noise only
        out, st = _run(model, ids, "cpu", codec, 0.0, interp=codec == "hamming84")
        cos = torch.nn.functional.cosine_similarity(out.flatten()[None], ref.flatten()[None]).item()
        assert cos > 0.98, (codec, cos)
        assert st["errors_corrected"] == 0 and st["total_values"] == 2 * 2 * 20 * 2 * 32


def test_errors_corrected_cpu():
    model, ids = _llama()
    clean, _ = _run(model, ids, "cpu", "golay", 0.0)
    noisy, st = _run(model, ids, "cpu", "golay", 1e-2)
    assert st["injection_count"] == 2 * 20 * 2 and st["errors_corrected"] > 0
    if st["errors_detected"] == 0:  # everything corrected -> identical logits
        assert torch.equal(noisy, clean)


@pytest.mark.gpu
@pytest.mark.parametrize("codec,interp", [("hamming84", True), ("hamming84", False),
                                          ("golay", False), ("hamming74", False)])
def test_hip_equals_cpu_backend(gpu, codec, interp):
    model, ids = _llama()
    cpu_logits, cpu_st = _run(model, ids, "cpu", codec, 1e-2, interp)
    model = model.to(gpu)
    hip_logits, hip_st = _run(model, ids.to(gpu), "hip", codec, 1e-2, interp)
    assert hip_st == cpu_st
    assert torch.allclose(hip_logits.cpu(), cpu_logits, atol=LOGIT_ATOL, rtol=LOGIT_ATOL)
