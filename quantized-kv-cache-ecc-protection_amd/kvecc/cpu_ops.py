"""Host ("cpu") codec backend: the reference's codec function set on CPU tensors.

The reference has no CPU codec backend -- every Triton wrapper asserts
``x.is_cuda`` (hamming74_triton.py:185,246; hamming84_triton.py:237,316;
golay_triton.py:399,456; fault_injection_triton.py:369; interpolation_triton.py:195;
fused_kernels.py:117,234,388).  BASELINE config 1 (``backend="cpu"``) needs one, so this module
runs the ``kvecc_cpu_*`` entry points of libkvecc.so: the same codec algebra
as the gfx950 kernels (csrc/codec_math.h is compiled for both), on host
memory, over ``std::thread`` workers.  Return values and error behaviour
mirror kvecc.ops (and therefore the reference wrappers) exactly.

This is an explicitly selected backend (``get_codec_backend("cpu")``), never a
fallback of the "hip" one; it needs libkvecc.so but no GPU.
"""

from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from .config import ErrorType

_VP = ctypes.c_void_p

# worker threads per call; <= 0 means every host core.  Defaults to
# OMP_NUM_THREADS when set (the process's CPU share), like torch's own pool.
NUM_THREADS = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)


def set_num_threads(n: int) -> None:
    global NUM_THREADS
    NUM_THREADS = int(n)


def _ptr(t):
    return _VP(t.data_ptr()) if t is not None else _VP(0)


def _check_cpu(t, what="Input"):
    if t.device.type != "cpu":
        raise AssertionError(f"{what} must be a CPU tensor for the 'cpu' codec backend")


def _flat(t, dtype):
    f = t.reshape(-1)
    if f.dtype != dtype:
        f = f.to(dtype)
    return f.contiguous()


def _stats():
    return torch.zeros(2, dtype=torch.int64)


# ---- statistics (host twin of ops.new_stats / read_stats) -------------------
def new_stats(device=None):
    """Host statistics buffer: int64 [2], stats[k] += ... by every *_into call."""
    return _stats()


def stats_totals(stats, n=2):
    return stats[:n].clone()


def read_stats(stats, n=2):
    return [int(v) for v in stats[:n].tolist()]


# ============================================================================
# Hamming
# ============================================================================

def hamming74_encode_into(flat_in, out):
    _lib.call("kvecc_cpu_hamming74_encode", _ptr(flat_in), _ptr(out), flat_in.numel(), NUM_THREADS)
    return out


def hamming84_encode_into(flat_in, out):
    _lib.call("kvecc_cpu_hamming84_encode", _ptr(flat_in), _ptr(out), flat_in.numel(), NUM_THREADS)
    return out


def hamming74_decode_into(flat_cw, data, flag=None, stats=None):
    _lib.call("kvecc_cpu_hamming74_decode", _ptr(flat_cw), _ptr(data), _ptr(flag), flat_cw.numel(),
              _ptr(stats), NUM_THREADS)
    return data


def hamming84_decode_into(flat_cw, data, error_type=None, stats=None):
    _lib.call("kvecc_cpu_hamming84_decode", _ptr(flat_cw), _ptr(data), _ptr(error_type),
              flat_cw.numel(), _ptr(stats), NUM_THREADS)
    return data


def hamming74_encode(int4_values: torch.Tensor) -> torch.Tensor:
    """INT4 -> Hamming(7,4) codewords (host twin of ops.hamming74_encode)."""
    _check_cpu(int4_values)
    flat = _flat(int4_values, torch.uint8)
    out = torch.empty_like(flat)
    _lib.call("kvecc_cpu_hamming74_encode", _ptr(flat), _ptr(out), flat.numel(), NUM_THREADS)
    return out.view(int4_values.shape)


def hamming74_decode(codewords: torch.Tensor, return_error_detected: bool = False):
    """-> (decoded, (n_corrected,)) or (decoded, error_detected, (n_corrected,))"""
    _check_cpu(codewords)
    flat = _flat(codewords, torch.uint8)
    data = torch.empty_like(flat)
    flag = torch.empty_like(flat)
    st = _stats()
    _lib.call("kvecc_cpu_hamming74_decode", _ptr(flat), _ptr(data), _ptr(flag), flat.numel(),
              _ptr(st), NUM_THREADS)
    n = int(st[0])
    data = data.view(codewords.shape)
    if return_error_detected:
        return data, flag.view(codewords.shape), (n,)
    return data, (n,)


def hamming84_encode(int4_values: torch.Tensor) -> torch.Tensor:
    _check_cpu(int4_values)
    flat = _flat(int4_values, torch.uint8)
    out = torch.empty_like(flat)
    _lib.call("kvecc_cpu_hamming84_encode", _ptr(flat), _ptr(out), flat.numel(), NUM_THREADS)
    return out.view(int4_values.shape)


def hamming84_decode(codewords: torch.Tensor, return_error_types: bool = False):
    """-> (decoded, (corrected, detected)) or (decoded, error_types, (corrected, detected))"""
    _check_cpu(codewords)
    flat = _flat(codewords, torch.uint8)
    data = torch.empty_like(flat)
    etype = torch.empty_like(flat)
    st = _stats()
    _lib.call("kvecc_cpu_hamming84_decode", _ptr(flat), _ptr(data), _ptr(etype), flat.numel(),
              _ptr(st), NUM_THREADS)
    corrected, detected = int(st[0]), int(st[1])
    data = data.view(codewords.shape)
    if return_error_types:
        return data, etype.view(codewords.shape), (corrected, detected)
    return data, (corrected, detected)


# ============================================================================
# Golay(24,12)
# ============================================================================

def golay_encode_into(flat_triplets, codewords, m):
    _lib.call("kvecc_cpu_golay_encode", _ptr(flat_triplets), _ptr(codewords), m, NUM_THREADS)
    return codewords


def golay_decode_into(flat_cw, triplets, counts=None, stats=None):
    _lib.call("kvecc_cpu_golay_decode", _ptr(flat_cw), _ptr(triplets), _ptr(counts),
              flat_cw.numel(), _ptr(stats), NUM_THREADS)
    return triplets


def golay_encode(triplets: torch.Tensor) -> torch.Tensor:
    """INT4 triplets [N,3] (or [3]) -> int32 codewords [N]."""
    _check_cpu(triplets)
    if triplets.dim() == 1:
        triplets = triplets.unsqueeze(0)
    n = triplets.shape[0]
    flat = _flat(triplets, torch.uint8)
    if flat.numel() < 3 * n:
        raise ValueError(f"golay_encode needs 3 values per codeword, got shape {tuple(triplets.shape)}")
    out = torch.empty(n, dtype=torch.int32)
    _lib.call("kvecc_cpu_golay_encode", _ptr(flat), _ptr(out), n, NUM_THREADS)
    return out


def golay_decode(codewords: torch.Tensor, return_error_counts: bool = False):
    """-> (triplets [N,3], (bits_corrected, uncorrectable)) or
       (triplets, error_counts [N], (bits_corrected, uncorrectable))"""
    _check_cpu(codewords)
    n = codewords.numel()
    flat = _flat(codewords, torch.int32)
    trip = torch.empty(n * 3, dtype=torch.uint8)
    counts = torch.empty(n, dtype=torch.uint8)
    st = _stats()
    _lib.call("kvecc_cpu_golay_decode", _ptr(flat), _ptr(trip), _ptr(counts), n, _ptr(st),
              NUM_THREADS)
    trip = trip.view(n, 3)
    if return_error_counts:
        return trip, counts, (int(st[0]), int(st[1]))
    return trip, (int(st[0]), int(st[1]))


def golay_encode_rows(nibbles: torch.Tensor) -> torch.Tensor:
    """Per-head packing of the shim (ecc_shim.py:623-682): [..., D] nibbles ->
    [..., ceil(D/3)] codewords, each row zero-padded to a multiple of 3."""
    _check_cpu(nibbles)
    d = nibbles.shape[-1]
    g = (d + 2) // 3
    flat = _flat(nibbles, torch.uint8)
    rows = flat.numel() // d if d else 0
    out = torch.empty(*nibbles.shape[:-1], g, dtype=torch.int32)
    _lib.call("kvecc_cpu_golay_encode_rows", _ptr(flat), _ptr(out), rows, d, NUM_THREADS)
    return out


def golay_decode_rows(codewords: torch.Tensor, d: int, stats=None) -> torch.Tensor:
    """Inverse of golay_encode_rows: [..., ceil(d/3)] -> [..., d] nibbles."""
    _check_cpu(codewords)
    g = codewords.shape[-1]
    if g != (d + 2) // 3:
        raise ValueError(f"{g} codewords per row do not hold {d} values")
    flat = _flat(codewords, torch.int32)
    rows = flat.numel() // g if g else 0
    out = torch.empty(*codewords.shape[:-1], d, dtype=torch.uint8)
    _lib.call("kvecc_cpu_golay_decode_rows", _ptr(flat), _ptr(out), rows, d, _ptr(stats),
              NUM_THREADS)
    return out

def golay_encode_rows_into(nibbles: torch.Tensor, out: torch.Tensor) -> None:
    """golay_encode_rows into a caller buffer: contiguous uint8 [..., D] nibbles ->
    contiguous int32 [..., ceil(D/3)] codewords (asynchronous on the stream)."""
    d = nibbles.shape[-1]
    g = (d + 2) // 3
    if (nibbles.dtype != torch.uint8 or out.dtype != torch.int32 or not nibbles.is_contiguous()
            or not out.is_contiguous() or out.shape[-1] != g or out.shape[:-1] != nibbles.shape[:-1]
            or out.device != nibbles.device):
        raise ValueError("golay_encode_rows_into: contiguous uint8 [..., D] -> int32 [..., ceil(D/3)]")
    rows = nibbles.numel() // d if d else 0
    _lib.call("kvecc_cpu_golay_encode_rows", _ptr(nibbles), _ptr(out), rows, d, NUM_THREADS)


def golay_decode_rows_into(codewords: torch.Tensor, out: torch.Tensor, stats=None) -> None:
    """golay_decode_rows into a caller buffer: contiguous int32 [..., ceil(D/3)] ->
    contiguous uint8 [..., D]; statistics accumulate into `stats` (asynchronous)."""
    d = out.shape[-1]
    g = (d + 2) // 3
    if (codewords.dtype != torch.int32 or out.dtype != torch.uint8 or not codewords.is_contiguous()
            or not out.is_contiguous() or codewords.shape[-1] != g or codewords.numel() // max(g, 1) * d != out.numel()
            or out.device != codewords.device):
        raise ValueError("golay_decode_rows_into: contiguous int32 [..., ceil(D/3)] -> uint8 [..., D]")
    rows = codewords.numel() // g if g else 0
    _lib.call("kvecc_cpu_golay_decode_rows", _ptr(codewords), _ptr(out), rows, d, _ptr(stats), NUM_THREADS)



# ============================================================================
# Fault injection
# ============================================================================

def inject_into(flat_in, out, ber, n_bits, seed=0, counts=None, stats=None, global_n=None,
                offset0=0, threads=None):
    """Host twin of ops.inject_into; `stats` is an int64 [2] host tensor."""
    n = flat_in.numel()
    gn = n if global_n is None else int(global_n)
    if flat_in.dtype == torch.uint8:
        name = "kvecc_cpu_inject_u8"
    elif flat_in.dtype == torch.int32:
        name = "kvecc_cpu_inject_i32"
    else:
        raise ValueError(f"Unsupported dtype: {flat_in.dtype}. Use uint8 or int32.")
    _lib.call(name, _ptr(flat_in), _ptr(out), _ptr(counts), n, int(n_bits), int(seed), float(ber),
              gn, int(offset0), _ptr(stats), NUM_THREADS if threads is None else int(threads))
    return out


def inject_rows_into(flat_in, out, rows, row_len, ber, n_bits, seed_base, stats=None):
    """Per-row injection: row r uses seed_base + r and N = row_len (shim scheme)."""
    if flat_in.dtype == torch.uint8:
        name = "kvecc_cpu_inject_rows_u8"
    elif flat_in.dtype == torch.int32:
        name = "kvecc_cpu_inject_rows_i32"
    else:
        raise ValueError(f"Unsupported dtype: {flat_in.dtype}. Use uint8 or int32.")
    _lib.call(name, _ptr(flat_in), _ptr(out), int(rows), int(row_len), int(n_bits), int(seed_base),
              float(ber), _ptr(stats), NUM_THREADS)
    return out


def inject_bit_errors_triton(data, ber, n_bits, seed=0, return_stats=False):
    """Bernoulli bit flips on the reference's Philox stream; ber <= 0 returns `data`.
    -> corrupted, or (corrupted, (total_flips, elements_affected))"""
    _check_cpu(data)
    if ber <= 0:
        if return_stats:
            return data, (0, 0)
        return data
    flat = data.reshape(-1)
    if flat.dtype not in (torch.uint8, torch.int32):
        raise ValueError(f"Unsupported dtype: {flat.dtype}. Use uint8 or int32.")
    flat = flat.contiguous()
    out = torch.empty_like(flat)
    st = _stats()
    inject_into(flat, out, ber, n_bits, seed, stats=st)
    out = out.view(data.shape)
    if return_stats:
        return out, (int(st[0]), int(st[1]))
    return out


inject_bit_errors = inject_bit_errors_triton


def inject_bit_errors_triton_batched(data, ber, n_bits, seed=0):
    corrupted, (total, _) = inject_bit_errors_triton(data, ber, n_bits, seed, return_stats=True)
    return corrupted, total


def inject_bit_errors_triton_vectorized(data, ber, n_bits, seed=0, return_stats=False):
    """rand4x variant (fault_injection_triton.py:434-496), host twin."""
    _check_cpu(data)
    if ber <= 0:
        if return_stats:
            return data, (0, 0)
        return data
    flat = data.reshape(-1)
    if flat.dtype == torch.uint8:
        name = "kvecc_cpu_inject_u8_vectorized"
    elif flat.dtype == torch.int32:
        name = "kvecc_cpu_inject_i32_vectorized"
    else:
        raise ValueError(f"Unsupported dtype: {flat.dtype}. Use uint8 or int32.")
    flat = flat.contiguous()
    out = torch.empty_like(flat)
    st = _stats()
    _lib.call(name, _ptr(flat), _ptr(out), _VP(0), flat.numel(), int(n_bits), int(seed), float(ber),
              _ptr(st), NUM_THREADS)
    out = out.view(data.shape)
    if return_stats:
        return out, (int(st[0]), int(st[1]))
    return out


# ============================================================================
# Interpolation
# ============================================================================

def _seq_layout(shape, seq_dim):
    from .ops import _seq_layout as layout  # pure shape arithmetic, no device code
    return layout(shape, seq_dim)


def count_ne_into(a, b, stats):
    """Host twin of ops.count_ne_into: stats[0] += count of positions where a != b."""
    if a.dtype != torch.uint8 or b.dtype != torch.uint8 or a.numel() != b.numel():
        raise ValueError("count_ne_into: two uint8 tensors of one size")
    a, b = a.contiguous(), b.contiguous()
    _lib.call("kvecc_cpu_count_ne_u8", _ptr(a), _ptr(b), a.numel(), _ptr(stats), NUM_THREADS)
    return stats


def any_equal(x, value, flag=None):
    """int32 flag [1] = any(x == value) (host twin of ops.any_equal)."""
    if flag is None:
        flag = torch.empty(1, dtype=torch.int32)
    flag.fill_(int(bool((x == value).any())))
    return flag


def interpolate_into(q, err, out, outer, length, inner, gate=None):
    """Host twin of ops.interpolate_into; `gate` (a host int32 flag) == 0 copies q."""
    if gate is not None and int(gate.reshape(-1)[0]) == 0:
        out.copy_(q)
        return out
    _lib.call("kvecc_cpu_interpolate", _ptr(q), _ptr(err), _ptr(out), outer, length, inner,
              NUM_THREADS)
    return out


def interpolate_double_errors(q, error_type, original_shape=None, seq_dim=-1):
    """Host twin of ops.interpolate_double_errors (interpolation_triton.py:162-265)."""
    _check_cpu(q)
    _check_cpu(error_type, "Error type")
    assert q.shape == error_type.shape, "Shape mismatch between q and error_type"
    if q.numel() == 0:
        return q.clone()
    err = _flat(error_type, torch.uint8)
    if not bool((err == ErrorType.DOUBLE_DETECTED).any()):
        return q.clone()
    qf = _flat(q, torch.uint8)
    outer, length, inner = _seq_layout(tuple(q.shape), seq_dim)
    out = torch.empty_like(qf)
    _lib.call("kvecc_cpu_interpolate", _ptr(qf), _ptr(err), _ptr(out), outer, length, inner,
              NUM_THREADS)
    return out.view(q.shape)


def interpolate_double_errors_1d(q, error_type):
    return interpolate_double_errors(q, error_type, seq_dim=-1)


def interpolate_double_errors_autotuned(q, error_type, original_shape=None, seq_dim=-1):
    return interpolate_double_errors(q, error_type, original_shape, seq_dim)


# ============================================================================
# Fused quantize + encode / decode + dequantize
# ============================================================================

_DT = {torch.float32: _lib.F32, torch.float16: _lib.F16, torch.bfloat16: _lib.BF16}

# Row-scale rule when the caller names none: the reference's `abs_max / 7.0` as
# torch evaluates it on this backend's device (CPU tensors: IEEE division;
# kvecc.h KVECC_SCALE_*).  Pass scale_rule="mul_inv7" to reproduce the reference run
# on a GPU.
DEFAULT_SCALE_RULE = "div7"


def quantize_encode_rows_into(x2d, codec_code, cw, scales, scale_rule=None):
    if x2d.dtype not in _DT:
        raise TypeError(f"unsupported input dtype {x2d.dtype}")
    rows, d = x2d.shape
    _lib.call("kvecc_cpu_quantize_encode_rows", _ptr(x2d), _DT[x2d.dtype], int(codec_code),
              _lib.scale_rule_code(scale_rule, DEFAULT_SCALE_RULE), _ptr(cw),
              _ptr(scales), rows, d, NUM_THREADS)
    return cw, scales


def decode_dequant_h84_into(cw2d, scales, out, zero_doubles=True, stats=None):
    rows, d = cw2d.shape
    _lib.call("kvecc_cpu_decode_dequant_h84_rows", _ptr(cw2d), _ptr(scales), _ptr(out),
              _DT[out.dtype], rows, d, int(bool(zero_doubles)), _ptr(stats), NUM_THREADS)
    return out


def _fused_quantize_encode(input_tensor, codec_code, scale_rule=None):
    _check_cpu(input_tensor)
    if input_tensor.dtype not in _DT:
        raise TypeError(f"unsupported input dtype {input_tensor.dtype}")
    shape = input_tensor.shape
    d = shape[-1]
    x = input_tensor.reshape(-1, d).contiguous()
    rows = x.shape[0]
    cw = torch.empty(rows, d, dtype=torch.uint8)
    scales = torch.empty(rows, dtype=torch.float32)
    _lib.call("kvecc_cpu_quantize_encode_rows", _ptr(x), _DT[x.dtype], int(codec_code),
              _lib.scale_rule_code(scale_rule, DEFAULT_SCALE_RULE), _ptr(cw),
              _ptr(scales), rows, d, NUM_THREADS)
    if input_tensor.dim() == 1:
        return cw.squeeze(0), scales
    return cw.view(shape), scales.view(shape[:-1])


def fused_quantize_encode_hamming84(input_tensor, scale_rule=None):
    return _fused_quantize_encode(input_tensor, _lib.CODEC_H84, scale_rule)


def fused_quantize_encode_hamming74(input_tensor, scale_rule=None):
    return _fused_quantize_encode(input_tensor, _lib.CODEC_H74, scale_rule)


def quantize_rows(input_tensor, scale_rule=None):
    return _fused_quantize_encode(input_tensor, _lib.CODEC_NONE, scale_rule)


def fused_decode_dequantize_hamming84(codewords, scales, output_dtype=torch.float32):
    """-> (dequantized, errors_corrected); double errors become 0 (fused_kernels.py:344)."""
    _check_cpu(codewords)
    _check_cpu(scales, "Scales")
    shape = codewords.shape
    d = shape[-1]
    cw = codewords.reshape(-1, d).contiguous()
    sc = scales.reshape(-1).to(torch.float32).contiguous()
    dtype = output_dtype if output_dtype in _DT else torch.float32
    out = torch.empty(cw.shape, dtype=dtype)
    st = _stats()
    _lib.call("kvecc_cpu_decode_dequant_h84_rows", _ptr(cw), _ptr(sc), _ptr(out), _DT[dtype],
              cw.shape[0], d, 1, _ptr(st), NUM_THREADS)
    out = out.squeeze(0) if codewords.dim() == 1 else out.view(shape)
    if output_dtype != dtype:
        out = out.to(output_dtype)
    return out, int(st[0])


# ============================================================================
# ECC shim: paged KV-cache write / read (host twins of ops.shim_write / shim_read)
# ============================================================================

SHIM_CODECS = {"int4": _lib.CODEC_NONE, "hamming74": _lib.CODEC_H74, "hamming84": _lib.CODEC_H84,
               "golay": _lib.CODEC_GOLAY, "golay_packed": _lib.CODEC_GOLAY_PACKED}


def shim_write(k, v, manager, layer, codec, n_bits, inject, ber, seed0, seq_id=0,
               scale_rule=None):
    shim_write_tensors(k, v, manager.k_cache, manager.v_cache, manager.k_scales, manager.v_scales,
                       manager.block_table[seq_id], manager.num_layers, manager.block_size,
                       manager.num_kv_heads, manager.head_dim, layer, codec, n_bits, inject, ber, seed0,
                       scale_rule)


def shim_write_tensors(k, v, k_cache, v_cache, k_scales, v_scales, table, num_layers, block_size, hkv, d,
                       layer, codec, n_bits, inject, ber, seed0, scale_rule=None):
    batch, seq = k.shape[0], k.shape[1]
    if k.dtype not in _DT or v.dtype != k.dtype:
        raise TypeError(f"unsupported K/V dtype {k.dtype}/{v.dtype}")
    _check_cpu(k)
    k, v = k.reshape(batch, seq, -1).contiguous(), v.reshape(batch, seq, -1).contiguous()
    _lib.call("kvecc_cpu_shim_write", _ptr(k), _ptr(v), _DT[k.dtype], batch, seq, int(hkv), int(d),
              SHIM_CODECS[codec], _lib.scale_rule_code(scale_rule, DEFAULT_SCALE_RULE), int(n_bits),
              int(bool(inject)), float(ber), int(seed0), _ptr(k_cache), _ptr(v_cache), _ptr(k_scales),
              _ptr(v_scales), _ptr(table), int(num_layers), int(block_size), int(layer), NUM_THREADS)


def shim_read(manager, layer, ctx, codec, interp, out_dtype, stats=None, seq_id=0):
    return shim_read_tensors(manager.k_cache, manager.v_cache, manager.k_scales, manager.v_scales,
                             manager.block_table[seq_id], ctx, manager.num_kv_heads, manager.head_dim,
                             manager.num_layers, manager.block_size, layer, codec, interp, out_dtype, stats)


def shim_read_tensors(k_cache, v_cache, k_scales, v_scales, table, ctx, hkv, d, num_layers, block_size,
                      layer, codec, interp, out_dtype, stats=None):
    shape = (hkv, ctx, d)
    k_out = torch.empty(shape, dtype=out_dtype)
    v_out = torch.empty(shape, dtype=out_dtype)
    _lib.call("kvecc_cpu_shim_read", _ptr(k_cache), _ptr(v_cache), _ptr(k_scales), _ptr(v_scales), _ptr(table),
              int(ctx), int(hkv), int(d), int(num_layers), int(block_size), int(layer), SHIM_CODECS[codec],
              int(bool(interp)), _ptr(k_out), _ptr(v_out), _DT[out_dtype], _ptr(stats), NUM_THREADS)
    return k_out, v_out


def shim_read_batch(k_cache, v_cache, k_scales, v_scales, block_table, ctx, head_dim, layer, codec,
                    out_dtype, stats=None, interp=False, out=None):
    """The shim's fused read (gather -> decode -> dequantize, ecc_shim.py:990-1071)
    for every sequence of a paged cache at once: block_table [B, max_blocks]
    int32 (row b = sequence b), caches [blocks, layers, hkv, block_size * P]
    -> (K, V) [B, hkv, ctx, head_dim] in out_dtype (kvecc_shim_read_batch)."""
    from .ops import _check_shim_read_args  # pure torch, device-agnostic
    if k_cache.device.type != "cpu":
        raise ValueError(f"the cpu backend reads host tensors, k_cache is on {k_cache.device}")
    batch, nl, hkv, bs = _check_shim_read_args(k_cache, v_cache, k_scales, v_scales, block_table, ctx,
                                               head_dim, layer, codec, out_dtype, stats, out)
    shape = (batch, hkv, ctx, head_dim)
    if out is None:
        out = (torch.empty(shape, dtype=out_dtype, device=k_cache.device),
               torch.empty(shape, dtype=out_dtype, device=k_cache.device))
    k_out, v_out = out
    _lib.call("kvecc_cpu_shim_read_batch", _ptr(k_cache), _ptr(v_cache), _ptr(k_scales), _ptr(v_scales),
              _ptr(block_table), block_table.shape[1], batch, int(ctx), hkv, head_dim, nl, bs,
              int(layer), SHIM_CODECS[codec], int(bool(interp)), _ptr(k_out), _ptr(v_out),
              _DT[out_dtype], _ptr(stats), NUM_THREADS)
    return k_out, v_out


# ============================================================================
# Paged decode attention (host twin of ops.paged_attention_ecc)
# ============================================================================

def paged_attention_into(query, k_cache, v_cache, block_table, context_lens, k_scales, v_scales,
                         out, layer_idx, block_size, sm_scale, codec, max_context_len=0):
    batch, heads, head_dim = query.shape
    num_blocks, num_layers, kv_heads, _ = k_cache.shape
    max_blocks = block_table.shape[1]
    _lib.call("kvecc_cpu_paged_attention", _ptr(query), _DT[query.dtype], _ptr(k_cache),
              _ptr(v_cache), _ptr(block_table), _ptr(context_lens), _ptr(k_scales),
              _ptr(v_scales), _ptr(out), batch, heads, kv_heads, head_dim, num_blocks, num_layers,
              int(layer_idx), int(block_size), max_blocks, int(max_context_len or 0),
              float(sm_scale), SHIM_CODECS[codec], NUM_THREADS)
    return out


def paged_attention_ecc(query, k_cache, v_cache, block_table, context_lens, k_scales, layer_idx,
                        block_size, sm_scale=None, codec="hamming84", syndrome_table=None,
                        use_tiled=False, block_m=4, v_scales=None):
    """Host twin of ops.paged_attention_ecc (same arguments and quirks)."""
    _check_cpu(query, "Query")
    if codec not in ("hamming84", "golay"):
        raise ValueError(f"Unknown codec: {codec}")
    if codec == "golay":
        v_scales = k_scales
    if v_scales is None:
        v_scales = k_scales
    if sm_scale is None:
        sm_scale = 1.0 / math.sqrt(query.shape[-1])
    q = query.contiguous()
    out_dtype = torch.float32 if codec == "golay" else q.dtype
    if q.dtype not in _DT:
        raise TypeError(f"unsupported query dtype {q.dtype}")
    if out_dtype != q.dtype:
        q = q.to(out_dtype)
    out = torch.empty(q.shape, dtype=out_dtype)
    paged_attention_into(q, k_cache.contiguous(), v_cache.contiguous(),
                         block_table.to(torch.int32).contiguous(),
                         context_lens.to(torch.int32).contiguous(),
                         k_scales.to(torch.float32).contiguous(),
                         v_scales.to(torch.float32).contiguous(), out, layer_idx, block_size,
                         sm_scale, codec)
    if codec == "hamming84" and use_tiled and block_size >= block_m:
        tiled_empty_to_zero(out, block_table, context_lens, block_size)
    return out


# ============================================================================
# Packed Golay storage (host twins of ops.golay_encode_packed / decode_packed)
# ============================================================================

from .ops import pack_nibbles, tiled_empty_to_zero, unpack_nibbles  # noqa: E402  (pure torch)


def golay_encode_packed(nibbles: torch.Tensor, m: int) -> torch.Tensor:
    _check_cpu(nibbles)
    nib = nibbles.reshape(-1)
    if nib.dtype != torch.uint8 or nib.numel() < (3 * m + 1) // 2:
        raise ValueError(f"need {(3 * m + 1) // 2} packed uint8 nibble bytes for {m} codewords")
    nib = nib.contiguous()
    out = torch.empty(3 * m, dtype=torch.uint8)
    _lib.call("kvecc_cpu_golay_encode_packed", _ptr(nib), _ptr(out), int(m), NUM_THREADS)
    return out


def golay_decode_packed(codewords: torch.Tensor, m: int, return_uncorrectable: bool = False,
                        stats=None):
    _check_cpu(codewords)
    cw = codewords.reshape(-1)
    if cw.dtype != torch.uint8 or cw.numel() < 3 * m:
        raise ValueError(f"need {3 * m} uint8 codeword bytes for {m} codewords")
    cw = cw.contiguous()
    nib = torch.empty((3 * m + 1) // 2, dtype=torch.uint8)
    flags = torch.empty((m + 7) // 8, dtype=torch.uint8) if return_uncorrectable else None
    st = _stats() if stats is None else stats
    _lib.call("kvecc_cpu_golay_decode_packed", _ptr(cw), _ptr(nib), _ptr(flags), int(m), _ptr(st),
              NUM_THREADS)
    if stats is not None:
        return (nib, flags) if return_uncorrectable else nib
    if return_uncorrectable:
        return nib, flags, (int(st[0]), int(st[1]))
    return nib, (int(st[0]), int(st[1]))


from .ops import pack_error_types  # noqa: E402  (pure torch, device-agnostic)


def hamming84_encode_packed(nibbles: torch.Tensor, n: int) -> torch.Tensor:
    _check_cpu(nibbles)
    nib = nibbles.reshape(-1)
    if nib.dtype != torch.uint8 or nib.numel() < (n + 1) // 2:
        raise ValueError(f"need {(n + 1) // 2} packed uint8 nibble bytes for {n} values")
    nib = nib.contiguous()
    out = torch.empty(n, dtype=torch.uint8)
    _lib.call("kvecc_cpu_hamming84_encode_packed", _ptr(nib), _ptr(out), int(n), NUM_THREADS)
    return out


def hamming84_decode_packed(codewords: torch.Tensor, return_error_types: bool = False):
    _check_cpu(codewords)
    cw = codewords.reshape(-1).to(torch.uint8).contiguous()
    n = cw.numel()
    nib = torch.empty((n + 1) // 2, dtype=torch.uint8)
    et = torch.empty((n + 3) // 4, dtype=torch.uint8) if return_error_types else None
    st = _stats()
    _lib.call("kvecc_cpu_hamming84_decode_packed", _ptr(cw), _ptr(nib), _ptr(et), n, _ptr(st),
              NUM_THREADS)
    if return_error_types:
        return nib, et, (int(st[0]), int(st[1]))
    return nib, (int(st[0]), int(st[1]))
