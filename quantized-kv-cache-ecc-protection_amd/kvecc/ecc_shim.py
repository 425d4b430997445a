"""ECC-protected paged KV cache shim for HuggingFace models (drop-in).

Mirrors kv_cache/ecc_shim.py of the reference (ECCShimConfig :134-186,
SimpleBlockManager :189-360, ECCBackend :363-1164, ECCPagedAttentionShim
:1167-1392, patch_model_with_ecc_attention :1395-1481, reset_ecc_cache /
get_ecc_stats :1614-1642) with identical cache layout, injection seeds and
statistics, plus the codec-backend selector the reference lacks
(``ECCShimConfig(backend="hip")``).

What changes is how the work is issued.  The reference runs a Python loop
over every (batch, position, kv-head) row with 2 encode + 2 inject Triton
launches and a ``.item()`` per position (ecc_shim.py:626-737), and stacks
cache slices one token at a time in attend (:931-977).  Here a layer's write
is one quantize, one encode, one per-row-seeded injection and one scatter per
K/V tensor (a handful of HIP launches for the whole layer), and attend is one
gather, one decode (+ interpolation) and one dequantization; error counters
accumulate on the device and are read only when asked for (get_ecc_stats).
"""

from __future__ import annotations

import math
from contextlib import contextmanager

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._lib import golay_packed_row_bytes
from .backends import get_codec_backend
from .memory_layout import kv_cache_pair

try:  # optional, as in the reference (:54)
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding
except Exception:  # pragma: no cover
    LlamaRotaryEmbedding = None


def compute_injection_seed(base_seed: int, layer_idx: int, injection_count: int) -> int:
    """base_seed + layer_idx*10000 + injection_count (ecc_shim.py:57-80)."""
    return base_seed + layer_idx * 10000 + injection_count


class ECCDummyCache:
    """Placeholder satisfying the transformers cache interface (ecc_shim.py:83-131)."""

    def __init__(self, num_layers=0):
        self.key_cache = []
        self.value_cache = []
        self._num_layers = num_layers
        self._seen_tokens = 0

    def __len__(self):
        return self._num_layers

    def __iter__(self):
        for i in range(len(self.key_cache)):
            yield (self.key_cache[i], self.value_cache[i])

    def __getitem__(self, layer_idx):
        if layer_idx < len(self.key_cache):
            return (self.key_cache[layer_idx], self.value_cache[layer_idx])
        return (None, None)

    def to_legacy_cache(self):
        return ()

    def get_seq_length(self, layer_idx=0):
        return self._seen_tokens

    def get_max_length(self):
        return None

    def get_usable_length(self, new_seq_length, layer_idx=0):
        return self._seen_tokens

    def update(self, key_states, value_states, layer_idx, cache_kwargs=None):
        self._seen_tokens += key_states.shape[-2]
        return key_states, value_states

    @property
    def seen_tokens(self):
        return self._seen_tokens


class ECCShimConfig:
    """Codec / BER / injection settings of the shim (ecc_shim.py:134-186).

    ``backend`` selects the codec implementation from kvecc.backends
    (default "hip"; unknown names raise ValueError).  ``fused`` runs the cache
    write and read as one launch each (kvecc_shim_write / kvecc_shim_read);
    False composes the per-op kernels (identical bits, kept for A/B tests).
    ``scale_rule`` picks how the INT4 row scale absmax / 7 is rounded:
    "mul_inv7" (absmax * RN(1/7), what the reference computes on GPU tensors),
    "div7" (IEEE division, the reference on CPU tensors) or None for the
    backend's device (kvecc.h KVECC_SCALE_*).
    ``golay_storage`` is the Golay cache layout: "int32" (the reference's, one
    int32 per codeword) or "packed" (3-byte codewords, token rows padded to 4
    bytes: 132 instead of 172 B per row at head_dim 128).  "packed" needs the
    fused write / read.
    """

    SUPPORTED_CODECS = {"fp16", "fp8", "int4", "hamming74", "hamming84", "golay"}

    def __init__(self, codec="hamming84", ber=0.0, block_size=16, num_blocks=256,
                 inject_errors=False, seed=42, use_interpolation=False, backend="hip",
                 fused=True, scale_rule=None, golay_storage="int32"):
        if codec not in self.SUPPORTED_CODECS:
            raise ValueError(f"Unsupported codec: '{codec}'. "
                             f"Supported codecs: {sorted(self.SUPPORTED_CODECS)}")
        self.codec = codec
        self.ber = ber
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.inject_errors = inject_errors
        self.seed = seed
        self.use_interpolation = use_interpolation
        self.backend = backend
        self.fused = fused  # one-launch cache write / read (False: per-op kernels)
        self.scale_rule = scale_rule
        if golay_storage not in ("int32", "packed"):
            raise ValueError(f"golay_storage must be 'int32' or 'packed', not {golay_storage!r}")
        if golay_storage == "packed" and not fused:
            raise ValueError("golay_storage='packed' needs fused=True")
        self.golay_storage = golay_storage


class SimpleBlockManager:
    """Paged KV storage, layout identical to ecc_shim.py:189-360.

    k_cache / v_cache: [num_blocks, num_layers, num_kv_heads, codewords_per_head]
    with codewords_per_head = block_size * head_dim (uint8 codewords, fp16,
    fp8) or block_size * ceil(head_dim/3) (int32 Golay codewords), or with
    golay_storage="packed" block_size * KVECC_GOLAY_PACKED_ROW(ceil(head_dim/3))
    uint8 (3-byte Golay codewords, not a reference layout);
    k_scales / v_scales: fp32 [num_blocks, num_layers, num_kv_heads, block_size].
    """

    def __init__(self, num_blocks, block_size, num_layers, num_kv_heads, head_dim, device="cuda",
                 codec="hamming84", golay_storage="int32"):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.num_layers = num_layers
        self.num_kv_heads = num_kv_heads
        self.head_dim = head_dim
        self.device = device
        self.codec = codec
        self.needs_scales = codec not in ("fp16", "fp8")
        self.golay_packed = codec == "golay" and golay_storage == "packed"
        # the codec name the fused shim kernels take (ops.SHIM_CODECS)
        self.shim_codec = "golay_packed" if self.golay_packed else codec
        if self.golay_packed:
            self.values_per_head = block_size * golay_packed_row_bytes((head_dim + 2) // 3)
            self.cache_dtype = torch.uint8
        elif codec == "golay":
            self.values_per_head = block_size * ((head_dim + 2) // 3)
            self.cache_dtype = torch.int32
        else:
            self.values_per_head = block_size * head_dim
            self.cache_dtype = {"fp16": torch.float16, "fp8": torch.float8_e4m3fn}.get(
                codec, torch.uint8)
        self.codewords_per_head = self.values_per_head
        shape = (num_blocks, num_layers, num_kv_heads, self.codewords_per_head)
        # one allocation, V skewed off K's HBM channels (memory_layout.kv_cache_pair)
        self.k_cache, self.v_cache = kv_cache_pair(shape, self.cache_dtype, device)
        sshape = (num_blocks, num_layers, num_kv_heads, block_size)
        self.k_scales = torch.zeros(sshape, dtype=torch.float32, device=device)
        self.v_scales = torch.zeros(sshape, dtype=torch.float32, device=device)
        self.free_blocks = list(range(num_blocks))
        self.seq_to_blocks = {}
        self.seq_to_len = {}
        self.max_seqs = 32
        self.max_blocks_per_seq = num_blocks
        self.block_table = torch.full((self.max_seqs, self.max_blocks_per_seq), -1,
                                      dtype=torch.int32, device=device)
        self._host_table = {}  # seq_id -> list of physical blocks (mirror, no device reads)
        # physical block ids on the device: a contiguous run of new blocks is
        # written into the table with a device-to-device copy, so allocation in
        # a steady-state forward issues no host-to-device transfer and the
        # whole patched forward can be captured in a HIP graph
        self._block_ids = torch.arange(num_blocks, dtype=torch.int32, device=device)

    def allocate(self, seq_id, num_tokens):
        need = (num_tokens + self.block_size - 1) // self.block_size
        existing = self.seq_to_blocks.get(seq_id, [])
        new_needed = max(0, need - len(existing))
        if new_needed > len(self.free_blocks):
            raise RuntimeError(f"Out of blocks: need {new_needed}, have {len(self.free_blocks)}")
        new = [self.free_blocks.pop(0) for _ in range(new_needed)]
        blocks = existing + new
        self.seq_to_blocks[seq_id] = blocks
        self.seq_to_len[seq_id] = num_tokens
        if new:
            dst = self.block_table[seq_id, len(existing):len(blocks)]
            if new == list(range(new[0], new[0] + len(new))):
                dst.copy_(self._block_ids[new[0]:new[0] + len(new)])
            else:
                dst.copy_(torch.tensor(new, dtype=torch.int32, device=self.block_table.device))
        self._host_table[seq_id] = blocks
        return self.block_table[seq_id], num_tokens

    def get_block_table(self, seq_id):
        return self.block_table[seq_id]

    def get_context_len(self, seq_id):
        return self.seq_to_len.get(seq_id, 0)

    def reset(self):
        # every block back in ascending order.  The reference appends the
        # returned blocks to the free list (ecc_shim.py:349-353), so each reset
        # rotates the physical ids the next forward gets; nothing observable
        # depends on them (the caches are zeroed here), but torch.compile
        # specialises a traced forward's allocation on the free list, and a
        # rotating list recompiled the patched model on every forward
        for blocks in self.seq_to_blocks.values():
            self.free_blocks.extend(blocks)
        self.free_blocks.sort()
        self.seq_to_blocks.clear()
        self.seq_to_len.clear()
        self._host_table.clear()
        self.block_table.fill_(-1)
        self.k_cache.zero_()
        self.v_cache.zero_()
        self.k_scales.zero_()
        self.v_scales.zero_()

    # ---- vectorised slot addressing -------------------------------------------
    def slots(self, seq_id, positions: int):
        """(physical block, slot) index tensors of token positions [0, positions)."""
        blocks = self._host_table.get(seq_id, [])
        pos = torch.arange(positions, device=self.k_cache.device)
        tab = torch.tensor(blocks or [0], dtype=torch.long, device=self.k_cache.device)
        return tab[pos // self.block_size], pos % self.block_size

    def view5(self, cache):
        """[blocks, layers, heads, block_size, per_token] view of a cache tensor."""
        return cache.view(self.num_blocks, self.num_layers, self.num_kv_heads, self.block_size, -1)


_N_BITS = {"hamming74": 7, "hamming84": 8, "golay": 24, "int4": 4, "fp8": 8}


class ECCBackend:
    """Quantize/encode/inject on write, decode/correct/dequantize on attend.

    Same observable behaviour as ecc_shim.py:363-1164: per-row injection seeds
    (K: seed + count, V: seed + count + 1, count += 1 per (batch, pos, head)
    row), last-batch-wins cache writes, statistics semantics per codec.
    """

    # codecs whose write / read run as one fused launch each (shim.hip)
    FUSED_CODECS = ("int4", "hamming74", "hamming84", "golay")

    def __init__(self, manager, config, num_heads, fused=None):
        self.manager = manager
        self.config = config
        self.codec_backend = get_codec_backend(getattr(config, "backend", "hip"))
        # fused=False composes the per-op kernels instead (same bits; A/B tests)
        self.fused = getattr(config, "fused", True) if fused is None else fused
        self.num_heads = num_heads
        self.num_kv_heads = manager.num_kv_heads
        self.head_dim = manager.head_dim
        if manager.golay_packed and not self._fused_ok():
            raise ValueError("packed Golay storage needs the fused shim write / read "
                             "(fused=True, a backend with shim_write, head_dim <= 512)")
        self.num_kv_groups = num_heads // self.num_kv_heads
        self._injection_count = 0
        self._total_values = 0
        self._stats = self.codec_backend.new_stats(manager.k_cache.device)  # backend counters

    # counters read lazily (one sync) -------------------------------------------
    @property
    def _errors_corrected(self):
        return self.codec_backend.read_stats(self._stats, 2)[0]

    @property
    def _errors_detected(self):
        return self.codec_backend.read_stats(self._stats, 2)[1]

    def reset_stats(self):
        self._injection_count = 0
        self._total_values = 0
        self._stats.zero_()

    def _inject_rows(self, enc, rows, row_len, seed_base):
        """Per-row injection of the reference's write loop, in place."""
        flat = enc.view(-1) if enc.dtype != torch.float8_e4m3fn else enc.view(torch.uint8).view(-1)
        self.codec_backend.inject_rows_into(flat, flat, rows, row_len, self.config.ber,
                             _N_BITS[self.config.codec], seed_base)

    def write(self, k, v, layer_idx, seq_id=0):
        """Store K, V [batch, seq, kv_heads*head_dim] (or a [batch, seq, kv_heads,
        head_dim] view, which the fused path reads in place) for layer `layer_idx`."""
        cfg, mgr = self.config, self.manager
        batch, seq_len = k.shape[0], k.shape[1]
        d, hk = self.head_dim, self.num_kv_heads
        self._total_values += 2 * batch * seq_len * hk * d
        if mgr.get_context_len(seq_id) < seq_len:
            mgr.allocate(seq_id, seq_len)
        rows = batch * seq_len * hk
        inject = cfg.inject_errors and cfg.ber > 0
        seed0 = cfg.seed + self._injection_count
        if self._fused_ok(k) and k.dtype == v.dtype:
            if self._traced():  # torch.compile: the dispatcher operator (no graph break)
                torch.ops.kvecc.shim_write(k, v, mgr.k_cache, mgr.v_cache, mgr.k_scales, mgr.v_scales,
                                           mgr.block_table[seq_id], mgr.num_layers, mgr.block_size,
                                           mgr.num_kv_heads, mgr.head_dim, layer_idx, mgr.shim_codec,
                                           _N_BITS[cfg.codec], inject, cfg.ber, seed0, cfg.scale_rule)
            else:
                self.codec_backend.shim_write(k, v, mgr, layer_idx, mgr.shim_codec, _N_BITS[cfg.codec],
                                              inject, cfg.ber, seed0, seq_id, cfg.scale_rule)
            if inject:
                self._injection_count += rows
            return
        if mgr.golay_packed:
            raise TypeError(f"packed Golay storage: K/V dtype {k.dtype}/{v.dtype} has no fused write")
        blk, slot = mgr.slots(seq_id, seq_len)
        kr = k.reshape(batch, seq_len, hk, d)
        vr = v.reshape(batch, seq_len, hk, d)
        codec = cfg.codec
        ops = self.codec_backend
        for which, x, cache, scales in ((0, kr, mgr.k_cache, mgr.k_scales),
                                        (1, vr, mgr.v_cache, mgr.v_scales)):
            if codec == "fp16":
                enc = x.to(torch.float16)
            elif codec == "fp8":
                enc = x.to(torch.float8_e4m3fn).contiguous()
                if inject:
                    self._inject_rows(enc, rows, d, seed0 + which)
            else:
                q, sc = ops.quantize_rows(x, cfg.scale_rule)  # the shim's torch rounding
                if codec == "golay":
                    enc = ops.golay_encode_rows(q)
                    row_len = enc.shape[-1]
                elif codec == "hamming74":
                    enc = ops.hamming74_encode(q)
                    row_len = d
                elif codec == "hamming84":
                    enc = ops.hamming84_encode(q)
                    row_len = d
                else:  # int4: raw nibbles
                    enc = q
                    row_len = d
                if inject:
                    self._inject_rows(enc, rows, row_len, seed0 + which)
                # last batch wins (every batch writes the same seq_id slots)
                mgr.view5(scales)[blk, layer_idx, :, slot, 0] = sc[-1]
            mgr.view5(cache)[blk, layer_idx, :, slot, :] = enc[-1].to(cache.dtype)
        if inject:
            self._injection_count += rows

    def _traced(self):
        """True while torch.compile traces this backend and it is one whose
        kernels are registered as torch.ops.kvecc operators (hip, cpu): calls
        then go through the dispatcher, eager calls straight to the C ABI."""
        return torch.compiler.is_compiling() and self.codec_backend.__name__ in ("kvecc.ops", "kvecc.cpu_ops")

    def _fused_ok(self, x=None):
        if not self.fused or self.config.codec not in self.FUSED_CODECS:
            return False
        if not hasattr(self.codec_backend, "shim_write"):
            return False
        d = self.head_dim
        if self.config.codec != "golay" and d % 4:
            return False
        if d > 512:
            return False
        return x is None or x.dtype in (torch.float32, torch.float16, torch.bfloat16)

    def _gather(self, cache, blk, slot, layer_idx):
        return self.manager.view5(cache)[blk, layer_idx, :, slot, :]  # [ctx, heads, per_token]

    def _decode(self, enc, stats):
        """Codewords [ctx, heads, *] -> INT4 [ctx, heads, head_dim] (stats += ...)."""
        codec, d = self.config.codec, self.head_dim
        ops = self.codec_backend
        if codec == "golay":
            return ops.golay_decode_rows(enc, d, stats=stats)
        flat = enc.reshape(-1)
        out = torch.empty_like(flat)
        if codec == "hamming74":
            ops.hamming74_decode_into(flat, out, None, stats)
            return out.view(enc.shape)
        if codec == "hamming84":
            if self.config.use_interpolation:
                et = torch.empty_like(flat)
                ops.hamming84_decode_into(flat, out, et, stats)
                ctx = enc.shape[0]
                res = torch.empty_like(flat)
                # temporal neighbours along the context axis (ecc_shim.py:1048-1059)
                ops.interpolate_into(out, et, res, 1, ctx, flat.numel() // max(ctx, 1))
                return res.view(enc.shape)
            ops.hamming84_decode_into(flat, out, None, stats)
            return out.view(enc.shape)
        return enc  # int4: raw nibbles

    def attend(self, q, layer_idx, seq_id=0):
        """Attention of q [batch, heads, seq, head_dim] over the decoded cache."""
        cfg, mgr = self.config, self.manager
        ctx = mgr.get_context_len(seq_id)
        if ctx == 0:
            return torch.zeros_like(q)
        q_len = q.shape[2]
        fast = cfg.codec == "hamming84" and not cfg.use_interpolation and q_len == 1
        if self._fused_ok() and fast:
            return self._paged_decode_attention(q, layer_idx, seq_id, ctx)
        if self._fused_ok():
            # the reference's seq_len==1 Triton path (ecc_shim.py:791-800) keeps no statistics
            interp = cfg.use_interpolation and cfg.codec == "hamming84"
            out_dtype, stats = (torch.float32, None) if fast else (q.dtype, self._stats)
            if self._traced():
                k_t, v_t = torch.ops.kvecc.shim_read(
                    mgr.k_cache, mgr.v_cache, mgr.k_scales, mgr.v_scales, mgr.block_table[seq_id], ctx,
                    mgr.num_kv_heads, mgr.head_dim, mgr.num_layers, mgr.block_size, layer_idx, mgr.shim_codec,
                    interp, out_dtype, stats)
            else:
                k_t, v_t = self.codec_backend.shim_read(mgr, layer_idx, ctx, mgr.shim_codec, interp,
                                                        out_dtype, stats, seq_id)
            if fast:
                return self._decode_step_attention(q, k_t, v_t)
            return self._run_attention_hd(q, k_t, v_t)
        blk, slot = mgr.slots(seq_id, ctx)
        k_enc = self._gather(mgr.k_cache, blk, slot, layer_idx)
        v_enc = self._gather(mgr.v_cache, blk, slot, layer_idx)
        if cfg.codec == "fp16":
            return self._run_attention(q, k_enc, v_enc)
        if cfg.codec == "fp8":
            return self._run_attention(q, k_enc.to(torch.float16), v_enc.to(torch.float16))
        # the reference's seq_len==1 Triton path (ecc_shim.py:791-800) keeps no statistics
        stats = None if fast else self._stats
        k_dec = self._decode(k_enc, stats)
        v_dec = self._decode(v_enc, stats)
        k_sc = mgr.view5(mgr.k_scales)[blk, layer_idx, :, slot, 0]
        v_sc = mgr.view5(mgr.v_scales)[blk, layer_idx, :, slot, 0]
        k_f = (k_dec.float() - 8.0) * k_sc.unsqueeze(-1)
        v_f = (v_dec.float() - 8.0) * v_sc.unsqueeze(-1)
        if fast:
            return self._decode_step_attention(q, k_f.transpose(0, 1), v_f.transpose(0, 1))
        return self._run_attention(q, k_f, v_f)

    def _paged_decode_attention(self, q, layer_idx, seq_id, ctx):
        """seq_len==1 Hamming(8,4) path: paged attention with inline decode
        (attention_ecc.py:620-780 via ecc_shim.py:1091-1136), no statistics.
        Every batch row attends over the same seq_id context (the reference
        passes one block-table row, ecc_shim.py:1117-1129)."""
        mgr = self.manager
        b, h, _, d = q.shape
        q1 = q[:, :, 0, :].contiguous()
        table = mgr.block_table[seq_id].unsqueeze(0).expand(b, -1).contiguous()
        lens = torch.full((b,), ctx, dtype=torch.int32, device=q.device)
        if self._traced():
            out = torch.ops.kvecc.paged_attention(q1, mgr.k_cache, mgr.v_cache, table, lens, mgr.k_scales,
                                                  mgr.v_scales, layer_idx, mgr.block_size, 1.0 / math.sqrt(d),
                                                  "hamming84", ctx)
            return out.unsqueeze(2)
        out = torch.empty_like(q1)
        self.codec_backend.paged_attention_into(
            q1, mgr.k_cache, mgr.v_cache, table, lens, mgr.k_scales, mgr.v_scales, out,
            layer_idx, mgr.block_size, 1.0 / math.sqrt(d), "hamming84", max_context_len=ctx)
        return out.unsqueeze(2)

    def _decode_step_attention(self, q, k_f, v_f):
        """seq_len==1 path of paged_attention_ecc (attention_ecc.py:264-427): fp32
        softmax over the context, output in q's dtype.  K/V are head-major
        [Hkv, ctx, D]; query head h reads cache head h // groups (the reference
        indexes cache head h directly, which only agrees without GQA)."""
        if self.num_kv_groups > 1:
            k_f = k_f.repeat_interleave(self.num_kv_groups, dim=0)
            v_f = v_f.repeat_interleave(self.num_kv_groups, dim=0)
        scale = 1.0 / math.sqrt(self.head_dim)
        qf = q[:, :, 0, :].float()                                # [B, H, D]
        scores = torch.einsum("bhd,htd->bht", qf, k_f) * scale     # [B, H, ctx]
        w = torch.softmax(scores, dim=-1)
        out = torch.einsum("bht,htd->bhd", w, v_f)
        return out.to(q.dtype).unsqueeze(2)

    def _run_attention_hd(self, q, k, v):
        """_run_attention on head-major K/V [Hkv, ctx, D] already in q's dtype."""
        if self.num_kv_groups > 1:
            k = k.repeat_interleave(self.num_kv_groups, dim=0)
            v = v.repeat_interleave(self.num_kv_groups, dim=0)
        return F.scaled_dot_product_attention(q, k.unsqueeze(0), v.unsqueeze(0),
                                              is_causal=q.shape[2] > 1)

    def _run_attention(self, q, k_float, v_float, device=None):
        """GQA expand + SDPA, causal for prefill (ecc_shim.py:1138-1164)."""
        if self.num_kv_groups > 1:
            k_float = k_float.repeat_interleave(self.num_kv_groups, dim=1)
            v_float = v_float.repeat_interleave(self.num_kv_groups, dim=1)
        k = k_float.permute(1, 0, 2).unsqueeze(0).to(q.dtype)
        v = v_float.permute(1, 0, 2).unsqueeze(0).to(q.dtype)
        return F.scaled_dot_product_attention(q, k, v, is_causal=q.shape[2] > 1)


class ECCPagedAttentionShim(nn.Module):
    """Replacement attention module (ecc_shim.py:1167-1392)."""

    def __init__(self, original_attn, layer_idx, backend, rotary_emb, model_type="llama"):
        super().__init__()
        self.model_type = model_type
        if model_type == "gpt2":
            for name in ("c_attn", "c_proj"):
                if not hasattr(original_attn, name):
                    avail = [a for a in dir(original_attn) if not a.startswith("_")]
                    raise ValueError(f"GPT-2 attention module missing '{name}'. Available: {avail}")
                setattr(self, name, getattr(original_attn, name))
            if hasattr(original_attn, "attn_dropout"):
                self.attn_dropout = original_attn.attn_dropout
            if hasattr(original_attn, "resid_dropout"):
                self.resid_dropout = original_attn.resid_dropout
        else:
            for name in ("q_proj", "k_proj", "v_proj", "o_proj"):
                if not hasattr(original_attn, name):
                    avail = [a for a in dir(original_attn) if not a.startswith("_")]
                    raise ValueError(f"Attention module {type(original_attn).__name__} missing "
                                     f"'{name}'. Available attributes: {avail}")
                proj = getattr(original_attn, name)
                if proj is None:
                    raise ValueError(f"'{name}' is None in {type(original_attn).__name__}. "
                                     "This attention implementation may not be compatible.")
                setattr(self, name, proj)
        self.num_heads, self.num_kv_heads, self.head_dim = _get_attention_params(original_attn)
        self.hidden_size = self.num_heads * self.head_dim
        if hasattr(original_attn, "split_size"):
            self.split_size = original_attn.split_size
        self.backend = backend
        self.layer_idx = layer_idx
        self.rotary_emb = rotary_emb
        self.scale = 1.0 / math.sqrt(self.head_dim)

    def forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_value=None,
                output_attentions=False, use_cache=False, cache_position=None, layer_past=None,
                head_mask=None, encoder_hidden_states=None, encoder_attention_mask=None, **kwargs):
        if self.model_type == "gpt2":
            return self._forward_gpt2(hidden_states, use_cache=use_cache,
                                      output_attentions=output_attentions)
        return self._forward_llama(hidden_states, position_ids=position_ids)

    def _forward_gpt2(self, hidden_states, use_cache=False, output_attentions=False):
        b, s, _ = hidden_states.shape
        q, k, v = self.c_attn(hidden_states).split(self.split_size, dim=2)
        q = q.view(b, s, self.num_heads, self.head_dim).transpose(1, 2)
        k = k.view(b, s, self.num_kv_heads, self.head_dim).transpose(1, 2)
        v = v.view(b, s, self.num_kv_heads, self.head_dim).transpose(1, 2)
        self._write(k, v, b, s)
        out = self.backend.attend(q, self.layer_idx, seq_id=0)
        out = self.c_proj(out.transpose(1, 2).contiguous().view(b, s, self.hidden_size))
        if hasattr(self, "resid_dropout"):
            out = self.resid_dropout(out)
        outputs = (out, (k, v) if use_cache else None)
        if output_attentions:
            outputs = outputs + (None,)
        return outputs

    def _forward_llama(self, hidden_states, position_ids=None):
        b, s, _ = hidden_states.shape
        q = self.q_proj(hidden_states).view(b, s, self.num_heads, self.head_dim).transpose(1, 2)
        k = self.k_proj(hidden_states).view(b, s, self.num_kv_heads, self.head_dim).transpose(1, 2)
        v = self.v_proj(hidden_states).view(b, s, self.num_kv_heads, self.head_dim).transpose(1, 2)
        if position_ids is None:
            position_ids = torch.arange(s, device=hidden_states.device).unsqueeze(0).expand(b, -1)
        cos, sin = self.rotary_emb(v, position_ids)
        q, k = self._apply_rotary_pos_emb(q, k, cos, sin)
        self._write(k, v, b, s)
        out = self.backend.attend(q, self.layer_idx, seq_id=0)
        out = self.o_proj(out.transpose(1, 2).contiguous().view(b, s, self.hidden_size))
        return out, None

    def _write(self, k, v, b, s):
        """backend.write of K/V [b, heads, s, d].  The reference copies them to
        [b, s, heads*d] first (ecc_shim.py:1290-1291, :1351-1352); the fused
        write reads the [b, s, heads, d] views in place."""
        if self.backend._fused_ok(k) and k.dtype == v.dtype:
            self.backend.write(k.transpose(1, 2), v.transpose(1, 2), self.layer_idx, seq_id=0)
        else:
            self.backend.write(k.transpose(1, 2).contiguous().view(b, s, -1),
                               v.transpose(1, 2).contiguous().view(b, s, -1), self.layer_idx,
                               seq_id=0)

    def _apply_rotary_pos_emb(self, q, k, cos, sin):
        def rotate_half(x):
            h = x.shape[-1] // 2
            return torch.cat((-x[..., h:], x[..., :h]), dim=-1)

        q_heads = q.shape[1]
        while cos.dim() < 4:
            cos = cos.unsqueeze(0 if cos.dim() < 2 else 1)
            sin = sin.unsqueeze(0 if sin.dim() < 2 else 1)
        if cos.shape[1] != 1 and cos.shape[1] != q_heads:
            cos, sin = cos[:, :1], sin[:, :1]
        return q * cos + rotate_half(q) * sin, k * cos + rotate_half(k) * sin


def _get_attention_params(attn_module):
    """(num_heads, num_kv_heads, head_dim) of an HF attention module (ecc_shim.py:1556-1611)."""
    cfg = getattr(attn_module, "config", None)
    num_heads = None
    for attr in ("num_heads", "num_attention_heads"):
        if hasattr(attn_module, attr):
            num_heads = getattr(attn_module, attr)
            break
    if num_heads is None and cfg is not None:
        for attr in ("num_attention_heads", "num_heads", "n_head"):
            if hasattr(cfg, attr):
                num_heads = getattr(cfg, attr)
                break
    head_dim = None
    for attr in ("head_dim", "head_size"):
        if hasattr(attn_module, attr):
            head_dim = getattr(attn_module, attr)
            break
    if head_dim is None and cfg is not None:
        if getattr(cfg, "head_dim", None):
            head_dim = cfg.head_dim
        elif hasattr(cfg, "hidden_size") and num_heads:
            head_dim = cfg.hidden_size // num_heads
    num_kv_heads = None
    for attr in ("num_key_value_heads", "num_kv_heads"):
        if hasattr(attn_module, attr):
            num_kv_heads = getattr(attn_module, attr)
            break
    if num_kv_heads is None and cfg is not None:
        for attr in ("num_key_value_heads", "num_kv_heads"):
            if hasattr(cfg, attr):
                num_kv_heads = getattr(cfg, attr)
                break
    if num_kv_heads is None:
        num_kv_heads = num_heads
    if (num_heads is None or head_dim is None) and hasattr(attn_module, "q_proj") and \
            hasattr(attn_module.q_proj, "weight"):
        out_features = attn_module.q_proj.weight.shape[0]
        for cand in (128, 64, 32, 96, 256):
            if out_features % cand == 0:
                head_dim = head_dim or cand
                num_heads = num_heads or out_features // cand
                break
    if num_heads is None:
        raise ValueError("Could not determine num_heads from attention module")
    if head_dim is None:
        raise ValueError("Could not determine head_dim from attention module")
    return num_heads, num_kv_heads, head_dim


def _find_rotary_embedding(model, layers):
    """Locate (or build) the rotary embedding module (ecc_shim.py:1484-1553)."""
    if hasattr(layers[0].self_attn, "rotary_emb"):
        return layers[0].self_attn.rotary_emb
    if hasattr(layers[0], "rotary_emb"):
        return layers[0].rotary_emb
    if hasattr(model, "model") and hasattr(model.model, "rotary_emb"):
        return model.model.rotary_emb
    if hasattr(model, "rotary_emb"):
        return model.rotary_emb
    device = next(model.parameters()).device
    config = getattr(model, "config", None)
    if LlamaRotaryEmbedding is not None and config is not None:
        try:
            return LlamaRotaryEmbedding(config=config, device=device)
        except TypeError:
            pass

    class SimpleRotaryEmbedding(nn.Module):
        def __init__(self, dim, base=10000.0):
            super().__init__()
            inv = 1.0 / (base ** (torch.arange(0, dim, 2).float() / dim))
            self.register_buffer("inv_freq", inv, persistent=False)

        def forward(self, x, position_ids):
            freqs = torch.einsum("i,j->ij", position_ids[0].float(),
                                 self.inv_freq.to(position_ids.device))
            emb = torch.cat((freqs, freqs), dim=-1)
            return emb.cos()[None, None], emb.sin()[None, None]

    _, _, head_dim = _get_attention_params(layers[0].self_attn)
    return SimpleRotaryEmbedding(head_dim).to(device)


@contextmanager
def patch_model_with_ecc_attention(model, config, num_blocks=256):
    """Swap every attention module of an HF model for the ECC shim
    (ecc_shim.py:1395-1481); restored on exit."""
    if hasattr(model, "model") and hasattr(model.model, "layers"):
        layers, model_type = model.model.layers, "llama"
    elif hasattr(model, "layers"):
        layers, model_type = model.layers, "llama"
    elif hasattr(model, "transformer") and hasattr(model.transformer, "h"):
        layers, model_type = model.transformer.h, "gpt2"
    else:
        raise ValueError("Unsupported model architecture")
    attn_attr = "attn" if model_type == "gpt2" else "self_attn"
    num_heads, num_kv_heads, head_dim = _get_attention_params(getattr(layers[0], attn_attr))
    manager = SimpleBlockManager(num_blocks=num_blocks, block_size=config.block_size,
                                 num_layers=len(layers), num_kv_heads=num_kv_heads,
                                 head_dim=head_dim, device=next(model.parameters()).device,
                                 codec=config.codec,
                                 golay_storage=getattr(config, "golay_storage", "int32"))
    backend = ECCBackend(manager, config, num_heads)
    rotary = None if model_type == "gpt2" else _find_rotary_embedding(model, layers)
    originals = {}
    try:
        for i, layer in enumerate(layers):
            originals[i] = getattr(layer, attn_attr)
            setattr(layer, attn_attr, ECCPagedAttentionShim(originals[i], i, backend, rotary,
                                                            model_type))
        model._ecc_block_manager = manager
        model._ecc_backend = backend
        model._ecc_model_type = model_type
        model._ecc_attn_attr = attn_attr
        yield model
    finally:
        for i, orig in originals.items():
            setattr(layers[i], attn_attr, orig)
        for name in ("_ecc_block_manager", "_ecc_backend", "_ecc_model_type", "_ecc_attn_attr"):
            if hasattr(model, name):
                delattr(model, name)


def reset_ecc_cache(model):
    """Fresh cache and counters for a new text (ecc_shim.py:1614-1624)."""
    if hasattr(model, "_ecc_block_manager"):
        model._ecc_block_manager.reset()
    if hasattr(model, "_ecc_backend"):
        model._ecc_backend.reset_stats()


def get_ecc_stats(model):
    """Block and error counters (ecc_shim.py:1627-1642); one device sync."""
    stats = {}
    if hasattr(model, "_ecc_block_manager"):
        m = model._ecc_block_manager
        stats["allocated_blocks"] = sum(len(b) for b in m.seq_to_blocks.values())
        stats["free_blocks"] = len(m.free_blocks)
        stats["sequences"] = len(m.seq_to_blocks)
    if hasattr(model, "_ecc_backend"):
        be = model._ecc_backend
        corrected, detected = be.codec_backend.read_stats(be._stats, 2)
        stats["injection_count"] = be._injection_count
        stats["errors_corrected"] = corrected
        stats["errors_detected"] = detected
        stats["total_values"] = be._total_values
    return stats
