"""The reference's own codec-level tests, ported over backend in {cpu, hip}.

Mirrors tests/test_triton_fault_injection.py:5-224 (statistical BER fidelity,
determinism, untouched high bits, sizes, statistics, the batched API),
tests/test_kv_cache.py:130-190,244-287 (scales KAT, write/decode round trip,
full encode -> inject -> decode pipelines) and tests/test_fused_kernels.py:110-123
(all-zero rows: scale 1.0, nibble 8) of the reference.  The exact flip patterns
are pinned elsewhere (tests/test_gpu_parity.py, tests/test_cpu_backend.py:
golden vectors from the reference's own kernels); these are the reference's
invariants, run as it states them.
"""

import pytest
import torch

BACKENDS = [pytest.param("cpu", id="cpu"), pytest.param("hip", id="hip", marks=pytest.mark.gpu)]


@pytest.fixture(params=BACKENDS)
def be(request):
    """(backend module, device) -- the hip case needs a GPU, the cpu case runs here."""
    from kvecc.backends import get_codec_backend
    if request.param == "hip":
        request.getfixturevalue("gpu")
        return get_codec_backend("hip"), torch.device("cuda:0")
    return get_codec_backend("cpu"), torch.device("cpu")


def _randint(hi, n, dtype, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, hi, n if isinstance(n, tuple) else (n,), generator=g, dtype=dtype).to(dev)


# ---- fault injection (test_triton_fault_injection.py) ---------------------------

def test_zero_ber_no_errors(be):
    ops, dev = be
    data = _randint(256, 10000, torch.uint8, dev)
    corrupted, stats = ops.inject_bit_errors_triton(data, ber=0.0, n_bits=8, seed=42, return_stats=True)
    assert torch.equal(data, corrupted) and stats[0] == 0


@pytest.mark.parametrize("target_ber", [0.01, 0.05, 0.10, 0.20])
def test_ber_fidelity_uint8(be, target_ber):
    ops, dev = be
    n, nb = 100_000, 8
    data = torch.zeros(n, dtype=torch.uint8, device=dev)
    _, stats = ops.inject_bit_errors_triton(data, ber=target_ber, n_bits=nb, seed=42, return_stats=True)
    assert abs(stats[0] / (n * nb) - target_ber) < max(target_ber * 0.1, 0.01)


@pytest.mark.parametrize("target_ber", [0.01, 0.05, 0.10])
def test_ber_fidelity_int32_24bit(be, target_ber):
    ops, dev = be
    n, nb = 50_000, 24
    data = torch.zeros(n, dtype=torch.int32, device=dev)
    _, stats = ops.inject_bit_errors_triton(data, ber=target_ber, n_bits=nb, seed=42, return_stats=True)
    assert abs(stats[0] / (n * nb) - target_ber) < max(target_ber * 0.1, 0.01)


def test_same_seed_same_result(be):
    ops, dev = be
    d8 = _randint(256, 10000, torch.uint8, dev)
    d32 = _randint(2**20, 10000, torch.int32, dev)
    assert torch.equal(ops.inject_bit_errors_triton(d8, ber=0.1, n_bits=8, seed=42),
                       ops.inject_bit_errors_triton(d8, ber=0.1, n_bits=8, seed=42))
    assert torch.equal(ops.inject_bit_errors_triton(d32, ber=0.1, n_bits=24, seed=42),
                       ops.inject_bit_errors_triton(d32, ber=0.1, n_bits=24, seed=42))


def test_different_seed_different_result(be):
    ops, dev = be
    data = torch.zeros(10000, dtype=torch.uint8, device=dev)
    assert not torch.equal(ops.inject_bit_errors_triton(data, ber=0.1, n_bits=8, seed=42),
                           ops.inject_bit_errors_triton(data, ber=0.1, n_bits=8, seed=99))


def test_only_active_bits_affected(be):
    ops, dev = be
    data = torch.full((10000,), 0x80, dtype=torch.uint8, device=dev)
    corrupted = ops.inject_bit_errors_triton(data, ber=0.5, n_bits=4, seed=42)
    assert bool((((corrupted >> 7) & 1) == 1).all())
    assert int(((corrupted ^ data) & 0x70).sum()) == 0  # bits 4..6 too
    assert bool((corrupted != data).any())


def test_xor_relationship(be):
    ops, dev = be
    data = torch.arange(256, dtype=torch.uint8, device=dev)
    corrupted = ops.inject_bit_errors_triton(data.clone(), ber=0.1, n_bits=8, seed=42)
    assert torch.equal(corrupted ^ (data ^ corrupted), data)


@pytest.mark.parametrize("size", [0, 1, 100, 1024, 10000, 100000])
def test_various_sizes(be, size):
    ops, dev = be
    for dtype, nb, hi in ((torch.uint8, 8, 256), (torch.int32, 24, 2**20)):
        data = _randint(hi, size, dtype, dev) if size else torch.empty(0, dtype=dtype, device=dev)
        corrupted = ops.inject_bit_errors_triton(data, ber=0.1, n_bits=nb, seed=42)
        assert corrupted.shape == data.shape and corrupted.dtype == data.dtype


def test_stats_match_actual_errors(be):
    ops, dev = be
    data = torch.zeros(10000, dtype=torch.uint8, device=dev)
    corrupted, stats = ops.inject_bit_errors_triton(data, ber=0.1, n_bits=8, seed=42, return_stats=True)
    actual = sum(int(((corrupted >> b) & 1).sum()) for b in range(8))
    assert stats[0] == actual
    assert stats[1] == int((corrupted != data).sum())


def test_batched_api_returns_error_count(be):
    ops, dev = be
    data = torch.zeros(10000, dtype=torch.uint8, device=dev)
    corrupted, total = ops.inject_bit_errors_triton_batched(data, ber=0.1, n_bits=8, seed=42)
    assert corrupted.shape == data.shape and isinstance(total, int) and total > 0


# ---- pipelines and cache helpers (test_kv_cache.py) --------------------------------

def test_full_ecc_pipeline_hamming84(be):
    ops, dev = be
    original = _randint(16, 10_000, torch.uint8, dev)
    corrupted = ops.inject_bit_errors_triton(ops.hamming84_encode(original), ber=0.001, n_bits=8, seed=42)
    decoded, _ = ops.hamming84_decode(corrupted)
    assert float((decoded == original).float().mean()) > 0.99


def test_full_ecc_pipeline_golay(be):
    ops, dev = be
    original = _randint(16, (3_333, 3), torch.uint8, dev)
    corrupted = ops.inject_bit_errors_triton(ops.golay_encode(original), ber=0.01, n_bits=24, seed=42)
    decoded, _ = ops.golay_decode(corrupted)
    assert float((decoded == original).float().mean()) > 0.98


def test_compute_quantization_scales_kat(be):
    from kvecc.paged_cache import compute_quantization_scales
    _, dev = be
    t = torch.tensor([[1.0, -2.0, 3.0, -4.0], [0.5, -0.5, 0.1, -0.1]], device=dev)
    s = compute_quantization_scales(t, dim=-1)
    assert s.shape == (2,)
    assert s[0].item() == pytest.approx(4.0 / 7, rel=0.01)
    assert s[1].item() == pytest.approx(0.5 / 7, rel=0.01)


def test_write_kv_roundtrip_hamming84(be):
    from kvecc.paged_cache import compute_quantization_scales, write_kv_to_cache_simple
    ops, dev = be
    g = torch.Generator().manual_seed(0)
    kv = torch.randn(2, 16, 32, generator=g).to(dev, torch.float16)
    scales = compute_quantization_scales(kv.float(), dim=-1)
    encoded, _ = write_kv_to_cache_simple(kv, codec="hamming84", scale=scales)
    decoded, _ = ops.hamming84_decode(encoded.flatten())
    deq = (decoded.view(encoded.shape).float() - 8) * scales.unsqueeze(-1)
    assert float(((kv.float() - deq) ** 2).mean()) < 1.0


# ---- fused kernels (test_fused_kernels.py) --------------------------------------------

def test_fused_zero_rows(be):
    ops, dev = be
    x = torch.zeros(4, 64, dtype=torch.float16, device=dev)
    cw, scales = ops.fused_quantize_encode_hamming84(x)
    assert bool((scales == 1.0).all())
    decoded, _ = ops.hamming84_decode(cw)
    assert bool((decoded == 8).all())
