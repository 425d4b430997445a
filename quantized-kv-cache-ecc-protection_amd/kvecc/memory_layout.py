"""Paged ECC cache configuration and block-table helpers.

Same API as kv_cache/memory_layout.py:5-111 (ECCCacheConfig, CacheBlock,
allocate_ecc_kv_cache, create_block_table, get_physical_block,
allocate_blocks, compute_slot_mapping).  Note the reference's two Golay
packings: ECCCacheConfig counts FLAT codewords per block,
ceil(block_size*head_size/3) (:31-37), while the shim packs per head,
block_size*ceil(head_size/3) (ecc_shim.py:261); both are reproduced as stated.
"""

from __future__ import annotations

import torch

from .config import get_physical_dtype

# V starts this many bytes past the 256-byte-rounded end of K (see kv_cache_pair)
KV_SKEW_BYTES = 12800


def kv_cache_pair(shape, dtype, device):
    """Zeroed K and V caches of one shape as two views of ONE allocation, V
    starting KV_SKEW_BYTES past K's 256-byte-rounded end.

    Paged decode attention reads K row r and V row r together.  In two separate
    equal-size allocations those rows sit exactly one allocation apart, which on
    MI355X maps them onto the same HBM channels and banks: Hamming(8,4) / Golay /
    packed Golay attention at [8,4096,32,128] ran 62.6 / 80.7 / 74.2 us with V
    right after K against 56.1 / 74.2 / 71.5 us with a 12,800-byte skew
    (tools/exp/attn_alias.py, profiles/r02/attention/kv_skew.log).  Both views
    are contiguous and 256-byte aligned; nothing else about the layout changes.

    V is handed out as its OWN storage over its bytes of the allocation
    (re-imported through DLPack, which keeps the allocation alive), not as a
    view of K's storage.  The two never overlap, but torch.compile's
    functionalization sees two views of one storage as aliased inputs: the
    shim's cache-write operator, which mutates both, then got a synthetic base
    and inductor cloned the WHOLE allocation around every layer's write (and
    copied it back), instead of writing the caches in place."""
    n = 1
    for x in shape:
        n *= int(x)
    esz = torch.empty((), dtype=dtype).element_size()
    v_off = ((n * esz + 255) // 256 * 256 + KV_SKEW_BYTES) // esz
    buf = torch.zeros(v_off + n, dtype=dtype, device=device)
    return buf[:n].view(shape), torch.from_dlpack(buf[v_off:v_off + n].view(shape))


class ECCCacheConfig:
    def __init__(self, num_heads, head_size, num_layers, block_size=16, num_blocks=256,
                 codec="hamming84"):
        self.num_heads = num_heads
        self.head_size = head_size
        self.num_layers = num_layers
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.codec = codec

    @property
    def dtype(self):
        return get_physical_dtype(self.codec)

    @property
    def values_per_block(self):
        return self.block_size * self.head_size

    @property
    def codewords_per_block(self):
        if self.codec == "golay":
            return (self.values_per_block + 2) // 3  # flat packing (memory_layout.py:31-37)
        return self.values_per_block

    @property
    def storage_overhead(self):
        """Stored bits per INT4 data bit: 8/4 (H84), 32/12 (Golay in int32), else 1."""
        if self.codec == "hamming84":
            return 8 / 4
        if self.codec == "golay":
            return 32 / 12
        return 1.0


class CacheBlock:
    def __init__(self, physical_idx, codec, dtype):
        self.physical_idx = physical_idx
        self.codec = codec
        self.dtype = dtype


def allocate_ecc_kv_cache(config: ECCCacheConfig, device="cuda"):
    """Zeroed K and V caches [num_blocks, num_layers, num_heads, codewords_per_block]."""
    shape = (config.num_blocks, config.num_layers, config.num_heads, config.codewords_per_block)
    return (torch.zeros(shape, dtype=config.dtype, device=device),
            torch.zeros(shape, dtype=config.dtype, device=device))


def create_block_table(batch_size, max_seq_len, block_size, device="cuda"):
    """int32 [batch, ceil(max_seq_len / block_size)] filled with -1 (no block)."""
    max_blocks = (max_seq_len + block_size - 1) // block_size
    return torch.full((batch_size, max_blocks), -1, dtype=torch.int32, device=device)


def get_physical_block(block_table, batch_idx, logical_block_idx):
    return int(block_table[batch_idx, logical_block_idx].item())


def allocate_blocks(block_table, batch_idx, num_blocks_needed, free_blocks, next_free_idx):
    """Take the next `num_blocks_needed` entries of free_blocks for row
    batch_idx; returns the new next_free_idx (RuntimeError when exhausted)."""
    if next_free_idx + num_blocks_needed > len(free_blocks):
        raise RuntimeError("Out of physical blocks")
    block_table[batch_idx, :num_blocks_needed] = free_blocks[
        next_free_idx:next_free_idx + num_blocks_needed].to(block_table.dtype)
    return next_free_idx + num_blocks_needed


def compute_slot_mapping(seq_len, block_size, block_table, batch_idx):
    """[seq_len, 2] = (physical block, slot within block) of every position."""
    pos = torch.arange(seq_len, device=block_table.device)
    physical = block_table[batch_idx, pos // block_size]
    return torch.stack([physical, (pos % block_size).to(physical.dtype)], dim=1)
