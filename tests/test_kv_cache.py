"""kv_cache/memory_layout.py and paged_cache_ecc.py helpers and the benchmark
harness API, after the reference's tests/test_kv_cache.py (CPU variants run
here; the GPU variants on the box)."""

import pytest
import torch


@pytest.mark.parametrize("codec,dtype,cpb,overhead", [
    ("hamming84", torch.uint8, 16 * 128, 2.0), ("golay", torch.int32, (16 * 128 + 2) // 3, 32 / 12)])
def test_ecc_cache_config(codec, dtype, cpb, overhead):
    from kvecc.memory_layout import ECCCacheConfig
    c = ECCCacheConfig(num_heads=32, head_size=128, num_layers=32, block_size=16, num_blocks=256,
                       codec=codec)
    assert c.dtype == dtype and c.values_per_block == 16 * 128
    assert c.codewords_per_block == cpb and c.storage_overhead == pytest.approx(overhead)


def test_allocate_and_block_tables():
    from kvecc.memory_layout import (ECCCacheConfig, allocate_blocks, allocate_ecc_kv_cache,
                                     compute_slot_mapping, create_block_table, get_physical_block)
    c = ECCCacheConfig(num_heads=8, head_size=64, num_layers=4, block_size=16, num_blocks=32)
    k, v = allocate_ecc_kv_cache(c, device="cpu")
    assert k.shape == v.shape == (32, 4, 8, c.codewords_per_block) and k.dtype == torch.uint8
    t = create_block_table(4, 512, 16, device="cpu")
    assert t.shape == (4, 32) and t.dtype == torch.int32 and bool((t == -1).all())
    t = create_block_table(2, 256, 16, device="cpu")
    assert allocate_blocks(t, 0, 5, torch.arange(64), 0) == 5
    assert t[0, :5].tolist() == [0, 1, 2, 3, 4] and bool((t[0, 5:] == -1).all())
    assert get_physical_block(t, 0, 3) == 3
    with pytest.raises(RuntimeError):
        allocate_blocks(t, 1, 10, torch.arange(12), 5)
    t = create_block_table(1, 256, 16, device="cpu")
    allocate_blocks(t, 0, 4, torch.arange(100), 0)
    sm = compute_slot_mapping(50, 16, t, batch_idx=0)
    assert sm.shape == (50, 2) and sm[0].tolist() == [0, 0] and sm[16].tolist() == [1, 0]


def _write_simple_checks(device):
    from kvecc.cpu_ops import hamming84_decode as cpu_h84_decode
    from kvecc.paged_cache import compute_quantization_scales, write_kv_to_cache_simple
    t = torch.tensor([[1.0, -2.0, 3.0, -4.0], [0.5, -0.5, 0.1, -0.1]], device=device)
    s = compute_quantization_scales(t, dim=-1)
    assert s.shape == (2,) and s[0].item() == pytest.approx(4 / 7) and s[1].item() == pytest.approx(0.5 / 7)
    g = torch.Generator().manual_seed(0)
    kv = torch.randn(2, 32, 64, generator=g).to(device=device, dtype=torch.float16)
    enc, sc = write_kv_to_cache_simple(kv, codec="hamming84")
    assert enc.shape == kv.shape and enc.dtype == torch.uint8 and sc.shape == (2, 32)
    # bit-exact against the reference formula restated in torch
    q = (torch.round(kv / sc.unsqueeze(-1)).clamp(-8, 7) + 8).to(torch.uint8)
    dec, _ = cpu_h84_decode(enc.cpu())
    assert torch.equal(dec, q.cpu())
    mse = ((kv.float().cpu() - (dec.float() - 8) * sc.float().cpu().unsqueeze(-1)) ** 2).mean()
    assert mse < 1.0
    genc, _ = write_kv_to_cache_simple(kv[:, :5, :7], codec="golay")
    assert genc.dtype == torch.int32 and genc.numel() == (2 * 5 * 7 + 2) // 3


def test_write_kv_simple_cpu():
    _write_simple_checks("cpu")


@pytest.mark.gpu
def test_write_kv_simple_gpu(gpu):
    _write_simple_checks(gpu)


@pytest.mark.gpu
def test_benchmark_harness(gpu):
    from kvecc import benchmark_harness as bh
    assert 0 < bh.cuda_timer(lambda: torch.randn(1000, device=gpu) + 1, warmup=5, repeat=50) < 1000
    r = bh.benchmark_hamming84_encode(n_elements=10_000, warmup=5, repeat=20)
    assert r.name == "hamming84_encode" and r.n_elements == 10_000 and r.latency_us > 0
    assert bh.benchmark_golay_encode(n_triplets=3_333, warmup=5, repeat=20).throughput_mvals_sec > 0
    r = bh.benchmark_fault_injection(n_elements=10_000, ber=0.05, warmup=5, repeat=20)
    assert "fault_injection" in r.name and r.extra["ber"] == 0.05
    r = bh.benchmark_encode_inject_decode(codec="hamming84", n_elements=10_000, ber=0.01, warmup=5,
                                          repeat=20)
    assert "pipeline" in r.name and r.extra["codec"] == "hamming84"
    r = bh.benchmark_encode_inject_decode(codec="golay", n_elements=9_999, ber=0.01, warmup=2,
                                          repeat=5)
    assert r.latency_us > 0


def test_kv_cache_pair_layout():
    """K and V are contiguous, zeroed, 256-byte aligned views of one allocation,
    V skewed past K (memory_layout.kv_cache_pair); SimpleBlockManager uses it."""
    import torch
    from kvecc.ecc_shim import SimpleBlockManager
    from kvecc.memory_layout import KV_SKEW_BYTES, kv_cache_pair
    for dtype, shape in ((torch.uint8, (5, 2, 3, 16 * 7)), (torch.int32, (4, 1, 2, 16 * 43))):
        k, v = kv_cache_pair(shape, dtype, "cpu")
        assert k.shape == v.shape == shape and k.dtype == v.dtype == dtype
        assert k.is_contiguous() and v.is_contiguous()
        assert not k.any() and not v.any()
        gap = v.data_ptr() - k.data_ptr() - k.numel() * k.element_size()
        assert gap >= KV_SKEW_BYTES and (v.data_ptr() - k.data_ptr()) % 256 == 0
        k.fill_(1)
        assert not v.any()  # disjoint
    mgr = SimpleBlockManager(8, 16, 2, 4, 64, device="cpu", codec="golay")
    assert mgr.v_cache.data_ptr() - mgr.k_cache.data_ptr() >= mgr.k_cache.numel() * 4 + KV_SKEW_BYTES
