"""The codec path as torch dispatcher operators: ``torch.ops.kvecc.*``.

The reference's functions are plain torch-callable Python functions
(ecc_codecs/triton_kernels/__init__.py:58-99, imported by the shim at
kv_cache/ecc_shim.py:42-51) that return Python ints for their statistics, so
every call is a device sync and a graph break under torch.compile.  Here each
codec step is also registered with the dispatcher (torch.library.custom_op):

  * a CUDA (HIP) kernel -- libkvecc.so through kvecc.ops -- and a CPU kernel --
    the host twin kvecc.cpu_ops -- chosen by the dispatcher from the inputs'
    device;
  * a fake (meta) kernel with the reference's shapes and dtypes (Golay
    [M,3] uint8 <-> [M] int32, uint8 flags / error types / counts), so
    torch.compile traces through the op without running it;
  * statistics as int64 tensors instead of Python ints (no sync), and the
    in-place / accumulating forms declared as mutations (``inject_bit_errors_``
    writes its input; the shim ops write the caches and accumulate statistics).

The reference-named Python functions (kvecc.hamming84_decode etc.) stay the
public API with the reference's return conventions; ECCBackend routes its
cache write / read and decode-step attention through these operators while
torch.compile traces it, so a patched attention forward compiles with no graph
break.  Registered on import of kvecc.
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib, cpu_ops, ops

_DEV = ("cuda", "cpu")


def _be(t: Tensor):
    """The backend module of a tensor's device: HIP kernels for GPU tensors,
    the host twin for CPU tensors (never a fallback from one to the other)."""
    return ops if t.is_cuda else cpu_ops


def _stats(t: Tensor):
    return _be(t).new_stats(t.device)


def _totals(t: Tensor, st: Tensor, n: int) -> Tensor:
    return _be(t).stats_totals(st, n).to(torch.int64).clone()


def _u8_flat(t: Tensor) -> Tensor:
    return t.reshape(-1).to(torch.uint8).contiguous()


# ---- Hamming(7,4) / Hamming(8,4) ---------------------------------------------

@torch.library.custom_op("kvecc::hamming74_encode", mutates_args=(), device_types=_DEV)
def hamming74_encode(int4_values: Tensor) -> Tensor:
    """hamming74_triton.py:170-201"""
    return _be(int4_values).hamming74_encode(int4_values)


@torch.library.custom_op("kvecc::hamming84_encode", mutates_args=(), device_types=_DEV)
def hamming84_encode(int4_values: Tensor) -> Tensor:
    """hamming84_triton.py:217-254"""
    return _be(int4_values).hamming84_encode(int4_values)


@hamming74_encode.register_fake
@hamming84_encode.register_fake
def _(int4_values):
    return torch.empty_like(int4_values, dtype=torch.uint8)


@torch.library.custom_op("kvecc::hamming74_decode", mutates_args=(), device_types=_DEV)
def hamming74_decode(codewords: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """hamming74_triton.py:218-277 -> (decoded, error_detected, int64[1] corrected)."""
    be, flat = _be(codewords), _u8_flat(codewords)
    data, flag, st = torch.empty_like(flat), torch.empty_like(flat), _stats(codewords)
    be.hamming74_decode_into(flat, data, flag, st)
    return data.view(codewords.shape), flag.view(codewords.shape), _totals(codewords, st, 1)


@hamming74_decode.register_fake
def _(codewords):
    u = torch.empty_like(codewords, dtype=torch.uint8)
    return u, torch.empty_like(u), codewords.new_empty(1, dtype=torch.int64)


@torch.library.custom_op("kvecc::hamming84_decode", mutates_args=(), device_types=_DEV)
def hamming84_decode(codewords: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """hamming84_triton.py:281-351 -> (decoded, error_types, int64[2] (corrected, detected))."""
    be, flat = _be(codewords), _u8_flat(codewords)
    data, et, st = torch.empty_like(flat), torch.empty_like(flat), _stats(codewords)
    be.hamming84_decode_into(flat, data, et, st)
    return data.view(codewords.shape), et.view(codewords.shape), _totals(codewords, st, 2)


@hamming84_decode.register_fake
def _(codewords):
    u = torch.empty_like(codewords, dtype=torch.uint8)
    return u, torch.empty_like(u), codewords.new_empty(2, dtype=torch.int64)


# ---- Golay(24,12) --------------------------------------------------------------

@torch.library.custom_op("kvecc::golay_encode", mutates_args=(), device_types=_DEV)
def golay_encode(triplets: Tensor) -> Tensor:
    """golay_triton.py:382-422: uint8 [M,3] (or [3]) -> int32 [M]."""
    return _be(triplets).golay_encode(triplets)


@golay_encode.register_fake
def _(triplets):
    m = 1 if triplets.dim() == 1 else triplets.shape[0]
    return triplets.new_empty(m, dtype=torch.int32)


@torch.library.custom_op("kvecc::golay_decode", mutates_args=(), device_types=_DEV)
def golay_decode(codewords: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """golay_triton.py:425-498 -> (uint8 [M,3] triplets, uint8 [M] error counts,
    int64[2] (bits corrected, uncorrectable))."""
    be = _be(codewords)
    flat = codewords.reshape(-1).to(torch.int32).contiguous()
    n = flat.numel()
    trip = torch.empty(n * 3, dtype=torch.uint8, device=codewords.device)
    counts = torch.empty(n, dtype=torch.uint8, device=codewords.device)
    st = _stats(codewords)
    be.golay_decode_into(flat, trip, counts, st)
    return trip.view(n, 3), counts, _totals(codewords, st, 2)


@golay_decode.register_fake
def _(codewords):
    n = codewords.numel()
    return (codewords.new_empty((n, 3), dtype=torch.uint8), codewords.new_empty(n, dtype=torch.uint8),
            codewords.new_empty(2, dtype=torch.int64))


@torch.library.custom_op("kvecc::golay_encode_rows", mutates_args=(), device_types=_DEV)
def golay_encode_rows(nibbles: Tensor) -> Tensor:
    """The shim's per-head packing (ecc_shim.py:623-682): [..., D] -> int32 [..., ceil(D/3)]."""
    return _be(nibbles).golay_encode_rows(nibbles)


@golay_encode_rows.register_fake
def _(nibbles):
    return nibbles.new_empty((*nibbles.shape[:-1], (nibbles.shape[-1] + 2) // 3), dtype=torch.int32)


@torch.library.custom_op("kvecc::golay_decode_rows", mutates_args=(), device_types=_DEV)
def golay_decode_rows(codewords: Tensor, d: int) -> Tuple[Tensor, Tensor]:
    """Inverse of golay_encode_rows -> (uint8 [..., d], int64[2] statistics)."""
    st = _stats(codewords)
    out = _be(codewords).golay_decode_rows(codewords, d, stats=st)
    return out, _totals(codewords, st, 2)


@golay_decode_rows.register_fake
def _(codewords, d):
    return (codewords.new_empty((*codewords.shape[:-1], d), dtype=torch.uint8),
            codewords.new_empty(2, dtype=torch.int64))


# ---- fault injection -----------------------------------------------------------

def _check_inject_dtype(data):
    if data.dtype not in (torch.uint8, torch.int32):
        raise ValueError(f"Unsupported dtype: {data.dtype}. Use uint8 or int32.")


@torch.library.custom_op("kvecc::inject_bit_errors", mutates_args=(), device_types=_DEV)
def inject_bit_errors(data: Tensor, ber: float, n_bits: int, seed: int) -> Tuple[Tensor, Tensor]:
    """fault_injection_triton.py:337-424 -> (corrupted copy, int64[2] (flips, elements
    affected)).  Unlike the Python API, ber <= 0 returns a copy (an operator's
    output may not alias its input)."""
    _check_inject_dtype(data)
    st = _stats(data)
    if ber <= 0:
        return data.clone(), _totals(data, st, 2)
    flat = data.reshape(-1).contiguous()
    out = torch.empty_like(flat)
    _be(data).inject_into(flat, out, ber, n_bits, seed, stats=st)
    return out.view(data.shape), _totals(data, st, 2)


@inject_bit_errors.register_fake
def _(data, ber, n_bits, seed):
    _check_inject_dtype(data)
    return torch.empty_like(data), data.new_empty(2, dtype=torch.int64)


@torch.library.custom_op("kvecc::inject_bit_errors_", mutates_args=("data",), device_types=_DEV)
def inject_bit_errors_(data: Tensor, ber: float, n_bits: int, seed: int, global_n: int = -1,
                       offset0: int = 0) -> Tensor:
    """In-place injection (kvecc_inject_*: out == in) of a contiguous tensor, sharded
    by (global_n, offset0) like the Monte-Carlo sweep -> int64[2] (flips, affected)."""
    _check_inject_dtype(data)
    if not data.is_contiguous():
        raise ValueError("inject_bit_errors_ needs a contiguous tensor")
    st = _stats(data)
    if ber > 0:
        flat = data.view(-1)
        _be(data).inject_into(flat, flat, ber, n_bits, seed, stats=st,
                              global_n=None if global_n < 0 else global_n, offset0=offset0)
    return _totals(data, st, 2)


@inject_bit_errors_.register_fake
def _(data, ber, n_bits, seed, global_n=-1, offset0=0):
    return data.new_empty(2, dtype=torch.int64)


# ---- interpolation ---------------------------------------------------------------

@torch.library.custom_op("kvecc::interpolate_double_errors", mutates_args=(), device_types=_DEV)
def interpolate_double_errors(q: Tensor, error_type: Tensor, seq_dim: int = -1) -> Tensor:
    """interpolation_triton.py:162-265 on uint8 q (for other dtypes the reference's
    result dtype depends on the data, which an operator cannot express: use the
    Python API)."""
    if q.dtype != torch.uint8:
        raise TypeError("kvecc::interpolate_double_errors takes uint8 q")
    return _be(q).interpolate_double_errors(q, error_type, seq_dim=seq_dim)


@interpolate_double_errors.register_fake
def _(q, error_type, seq_dim=-1):
    if q.dtype != torch.uint8:
        raise TypeError("kvecc::interpolate_double_errors takes uint8 q")
    return torch.empty_like(q)


# ---- fused quantize + encode / decode + dequantize --------------------------------

@torch.library.custom_op("kvecc::fused_quantize_encode", mutates_args=(), device_types=_DEV)
def fused_quantize_encode(x: Tensor, codec: str, scale_rule: Optional[str] = None) -> Tuple[Tensor, Tensor]:
    """fused_kernels.py:18-160 (hamming84) / :163-269 (hamming74); codec "int4" =
    quantize only -> (uint8 codewords shaped like x, fp32 row scales)."""
    be = _be(x)
    fn = {"hamming84": be.fused_quantize_encode_hamming84, "hamming74": be.fused_quantize_encode_hamming74,
          "int4": be.quantize_rows}[codec]
    return fn(x, scale_rule)


@fused_quantize_encode.register_fake
def _(x, codec, scale_rule=None):
    sshape = x.shape[:-1] if x.dim() > 1 else (1,)
    return torch.empty_like(x, dtype=torch.uint8), x.new_empty(sshape, dtype=torch.float32)


@torch.library.custom_op("kvecc::fused_decode_dequantize_hamming84", mutates_args=(), device_types=_DEV)
def fused_decode_dequantize_hamming84(codewords: Tensor, scales: Tensor,
                                      output_dtype: torch.dtype = torch.float32) -> Tuple[Tensor, Tensor]:
    """fused_kernels.py:372-437 -> (dequantized, int64[1] errors corrected)."""
    be = _be(codewords)
    d = codewords.shape[-1]
    cw = codewords.reshape(-1, d).contiguous()
    sc = scales.reshape(-1).to(torch.float32).contiguous()
    dt = output_dtype if output_dtype in (torch.float32, torch.float16, torch.bfloat16) else torch.float32
    out = torch.empty(cw.shape, dtype=dt, device=codewords.device)
    st = _stats(codewords)
    be.decode_dequant_h84_into(cw, sc, out, True, st)
    return out.view(codewords.shape).to(output_dtype), _totals(codewords, st, 1)


@fused_decode_dequantize_hamming84.register_fake
def _(codewords, scales, output_dtype=torch.float32):
    return torch.empty_like(codewords, dtype=output_dtype), codewords.new_empty(1, dtype=torch.int64)


# ---- ECC shim: cache write / read, decode-step paged attention ----------------------

@torch.library.custom_op("kvecc::shim_write", mutates_args=("k_cache", "v_cache", "k_scales", "v_scales"),
                         device_types=_DEV)
def shim_write(k: Tensor, v: Tensor, k_cache: Tensor, v_cache: Tensor, k_scales: Tensor, v_scales: Tensor,
               table: Tensor, num_layers: int, block_size: int, hkv: int, d: int, layer: int, codec: str,
               n_bits: int, inject: bool, ber: float, seed0: int, scale_rule: Optional[str] = None) -> None:
    """ECCBackend.write of one layer (ecc_shim.py:557-721) into the paged caches."""
    _be(k).shim_write_tensors(k, v, k_cache, v_cache, k_scales, v_scales, table, num_layers, block_size,
                              hkv, d, layer, codec, n_bits, inject, ber, seed0, scale_rule)


@shim_write.register_fake
def _(k, v, k_cache, v_cache, k_scales, v_scales, table, num_layers, block_size, hkv, d, layer, codec,
      n_bits, inject, ber, seed0, scale_rule=None):
    return None


@torch.library.custom_op("kvecc::shim_read", mutates_args=("stats",), device_types=_DEV)
def shim_read(k_cache: Tensor, v_cache: Tensor, k_scales: Tensor, v_scales: Tensor, table: Tensor, ctx: int,
              hkv: int, d: int, num_layers: int, block_size: int, layer: int, codec: str, interp: bool,
              out_dtype: torch.dtype, stats: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """ECCBackend.attend's decode side (ecc_shim.py:990-1071) -> K, V [hkv, ctx, d];
    statistics accumulate into `stats` (the backend's sharded counter buffer)."""
    return _be(k_cache).shim_read_tensors(k_cache, v_cache, k_scales, v_scales, table, ctx, hkv, d,
                                          num_layers, block_size, layer, codec, interp, out_dtype, stats)


@shim_read.register_fake
def _(k_cache, v_cache, k_scales, v_scales, table, ctx, hkv, d, num_layers, block_size, layer, codec, interp,
      out_dtype, stats):
    shape = (hkv, ctx, d)
    return k_cache.new_empty(shape, dtype=out_dtype), k_cache.new_empty(shape, dtype=out_dtype)


@torch.library.custom_op("kvecc::paged_attention", mutates_args=(), device_types=_DEV)
def paged_attention(query: Tensor, k_cache: Tensor, v_cache: Tensor, block_table: Tensor,
                    context_lens: Tensor, k_scales: Tensor, v_scales: Tensor, layer_idx: int, block_size: int,
                    sm_scale: float, codec: str, max_context_len: int = 0) -> Tensor:
    """Decode-step paged attention with inline ECC decode (attention_ecc.py:620-780)."""
    out = torch.empty_like(query)
    _be(query).paged_attention_into(query, k_cache, v_cache, block_table, context_lens, k_scales, v_scales,
                                    out, layer_idx, block_size, sm_scale, codec,
                                    max_context_len=max_context_len)
    return out


@paged_attention.register_fake
def _(query, k_cache, v_cache, block_table, context_lens, k_scales, v_scales, layer_idx, block_size, sm_scale,
      codec, max_context_len=0):
    return torch.empty_like(query)


OPS: List[str] = ["hamming74_encode", "hamming84_encode", "hamming74_decode", "hamming84_decode",
                  "golay_encode", "golay_decode", "golay_encode_rows", "golay_decode_rows",
                  "inject_bit_errors", "inject_bit_errors_", "interpolate_double_errors",
                  "fused_quantize_encode", "fused_decode_dequantize_hamming84", "shim_write", "shim_read",
                  "paged_attention"]
_ = _lib  # the operators bind libkvecc.so lazily, on first call
