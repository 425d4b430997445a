"""ctypes front-end for the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- as the checker, never as the measured or
shipped path.  The product package (kvecc) never imports this module.

Each function mirrors the reference semantics it restates (see
kvecc_oracle.h for the file:line of every restated kernel) and works on
numpy arrays.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_f32p = ctypes.POINTER(ctypes.c_float)
_i64 = ctypes.c_int64
_int = ctypes.c_int
_f32 = ctypes.c_float


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        sig = {
            "oracle_golay_h_row_masks": [_u32p],
            "oracle_golay_syndrome_table": [_i32p],
            "oracle_h74_encode": [_u8p, _u8p, _i64],
            "oracle_h74_decode": [_u8p, _u8p, _u8p, _i64, _i64p],
            "oracle_h84_encode": [_u8p, _u8p, _i64],
            "oracle_h84_decode": [_u8p, _u8p, _u8p, _i64, _i64p],
            "oracle_golay_encode": [_u8p, _i32p, _i64],
            "oracle_golay_decode": [_i32p, _u8p, _u8p, _i64, _i64p],
            "oracle_philox4x32_10": [ctypes.c_uint32] * 6 + [_u32p],
            "oracle_inject_u8": [_u8p, _u8p, _u8p, _i64, _int, _i64, _f32, _i64, _i64, _i64p],
            "oracle_inject_i32": [_i32p, _i32p, _u8p, _i64, _int, _i64, _f32, _i64, _i64, _i64p],
            "oracle_inject_rows_u8": [_u8p, _u8p, _i64, _i64, _int, _i64, _f32, _i64p],
            "oracle_inject_u8_vectorized": [_u8p, _u8p, _u8p, _i64, _int, _i64, _f32, _i64p],
            "oracle_inject_i32_vectorized": [_i32p, _i32p, _u8p, _i64, _int, _i64, _f32, _i64p],
            "oracle_interpolate": [_u8p, _u8p, _u8p, _i64, _i64, _i64],
            "oracle_quantize_rows": [_f32p, _i64, _i64, _int, _u8p, _f32p],
            "oracle_decode_dequant_h84": [_u8p, _f32p, _i64, _i64, _f32p, _i64p],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = None
        L.oracle_uint_to_uniform.argtypes = [ctypes.c_uint32]
        L.oracle_uint_to_uniform.restype = ctypes.c_float
        _lib = L
        # build the Golay table once, before any multi-threaded use
        dummy = np.zeros(1, np.int32)
        golay_decode(dummy)
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# --------------------------------------------------------------------------
def golay_h_row_masks():
    out = np.zeros(12, np.uint32)
    lib().oracle_golay_h_row_masks(_p(out, _u32p))
    return out


def golay_syndrome_table():
    out = np.zeros(4096, np.int32)
    lib().oracle_golay_syndrome_table(_p(out, _i32p))
    return out


def hamming74_encode(x):
    x = _c(x, np.uint8)
    out = np.empty_like(x)
    lib().oracle_h74_encode(_p(x, _u8p), _p(out, _u8p), x.size)
    return out


def hamming84_encode(x):
    x = _c(x, np.uint8)
    out = np.empty_like(x)
    lib().oracle_h84_encode(_p(x, _u8p), _p(out, _u8p), x.size)
    return out


def hamming74_decode(cw):
    """-> (data, flag, (n_corrected,))  hamming74_triton.py:218-277"""
    cw = _c(cw, np.uint8)
    data = np.empty_like(cw)
    flag = np.empty_like(cw)
    st = np.zeros(2, np.int64)
    lib().oracle_h74_decode(_p(cw, _u8p), _p(data, _u8p), _p(flag, _u8p), cw.size, _p(st, _i64p))
    return data, flag, (int(st[0]),)


def hamming84_decode(cw):
    """-> (data, error_type, (corrected, detected))  hamming84_triton.py:281-351"""
    cw = _c(cw, np.uint8)
    data = np.empty_like(cw)
    et = np.empty_like(cw)
    st = np.zeros(2, np.int64)
    lib().oracle_h84_decode(_p(cw, _u8p), _p(data, _u8p), _p(et, _u8p), cw.size, _p(st, _i64p))
    return data, et, (int(st[0]), int(st[1]))


def golay_encode(trip):
    """triplets [M,3] uint8 -> int32 [M]  golay_triton.py:382-422"""
    t = _c(trip, np.uint8).reshape(-1, 3)
    out = np.empty(t.shape[0], np.int32)
    lib().oracle_golay_encode(_p(t, _u8p), _p(out, _i32p), t.shape[0])
    return out


def golay_decode(cw):
    """-> (triplets [M,3], counts [M], (bits_corrected, uncorrectable))"""
    cw = _c(cw, np.int32).reshape(-1)
    trip = np.empty((cw.size, 3), np.uint8)
    cnt = np.empty(cw.size, np.uint8)
    st = np.zeros(2, np.int64)
    (_lib or lib()).oracle_golay_decode(_p(cw, _i32p), _p(trip, _u8p), _p(cnt, _u8p), cw.size,
                                        _p(st, _i64p))
    return trip, cnt, (int(st[0]), int(st[1]))


def philox(c0, c1, c2, c3, k0, k1):
    out = np.zeros(4, np.uint32)
    lib().oracle_philox4x32_10(c0, c1, c2, c3, k0, k1, _p(out, _u32p))
    return out


def inject(data, ber, n_bits, seed=0, global_n=None, offset0=0):
    """-> (corrupted, counts, (flips, affected)); fault_injection_triton.py:228-334.

    ``global_n``/``offset0`` describe a shard of a larger flat tensor.
    """
    data = np.ascontiguousarray(data)
    flat = data.reshape(-1)
    n = flat.size
    gn = n if global_n is None else int(global_n)
    out = np.empty_like(flat)
    cnt = np.empty(n, np.uint8)
    st = np.zeros(2, np.int64)
    if flat.dtype == np.uint8:
        lib().oracle_inject_u8(_p(flat, _u8p), _p(out, _u8p), _p(cnt, _u8p), n, int(n_bits),
                               int(seed), float(ber), gn, int(offset0), _p(st, _i64p))
    elif flat.dtype == np.int32:
        lib().oracle_inject_i32(_p(flat, _i32p), _p(out, _i32p), _p(cnt, _u8p), n, int(n_bits),
                                int(seed), float(ber), gn, int(offset0), _p(st, _i64p))
    else:
        raise ValueError(f"Unsupported dtype: {flat.dtype}. Use uint8 or int32.")
    return out.reshape(data.shape), cnt, (int(st[0]), int(st[1]))


def inject_rows(data, ber, n_bits, seed0):
    """The shim's per-row injection (kv_cache/ecc_shim.py:594-603, 644-652): uint8
    rows [R, row_len], row r its own tensor with seed seed0 + r.
    -> (corrupted, (flips, affected))"""
    data = _c(data, np.uint8)
    rows, row_len = data.shape
    out = np.empty_like(data)
    st = np.zeros(2, np.int64)
    lib().oracle_inject_rows_u8(_p(data, _u8p), _p(out, _u8p), rows, row_len, int(n_bits), int(seed0),
                                float(ber), _p(st, _i64p))
    return out, (int(st[0]), int(st[1]))


def inject_vectorized(data, ber, n_bits, seed=0):
    data = np.ascontiguousarray(data)
    flat = data.reshape(-1)
    n = flat.size
    out = np.empty_like(flat)
    cnt = np.empty(n, np.uint8)
    st = np.zeros(2, np.int64)
    if flat.dtype == np.uint8:
        lib().oracle_inject_u8_vectorized(_p(flat, _u8p), _p(out, _u8p), _p(cnt, _u8p), n,
                                          int(n_bits), int(seed), float(ber), _p(st, _i64p))
    elif flat.dtype == np.int32:
        lib().oracle_inject_i32_vectorized(_p(flat, _i32p), _p(out, _i32p), _p(cnt, _u8p), n,
                                           int(n_bits), int(seed), float(ber), _p(st, _i64p))
    else:
        raise ValueError(f"Unsupported dtype: {flat.dtype}. Use uint8 or int32.")
    return out.reshape(data.shape), cnt, (int(st[0]), int(st[1]))


def interpolate_kernel(q, err, outer, length, inner):
    """Kernel semantics (every element clamped) on an [outer, length, inner] array."""
    q = _c(q, np.uint8)
    err = _c(err, np.uint8)
    out = np.empty_like(q)
    lib().oracle_interpolate(_p(q, _u8p), _p(err, _u8p), _p(out, _u8p), outer, length, inner)
    return out


def interpolate_double_errors(q, err, seq_dim=-1):
    """interpolation_triton.py:162-265 wrapper semantics on numpy arrays."""
    q = np.asarray(q)
    err = np.asarray(err)
    assert q.shape == err.shape
    if not (err == 2).any():
        return q.copy()
    if q.ndim == 1:
        outer, length, inner, axis = 1, q.shape[0], 1, 0
    elif q.ndim == 2:  # 2-D ignores seq_dim (:210-213)
        outer, length, inner, axis = q.shape[0], q.shape[1], 1, 1
    else:
        axis = seq_dim % q.ndim
        outer = int(np.prod(q.shape[:axis]))
        length = q.shape[axis]
        inner = int(np.prod(q.shape[axis + 1:]))
    out = interpolate_kernel(q.astype(np.uint8), err.astype(np.uint8), outer, length, inner)
    return out.reshape(q.shape)


def quantize_rows(x, rule=0):
    """-> (q uint8 [..., D], scales f32 [...])  ecc_shim.py:572-580
    rule 0: scale by IEEE division (torch on CPU); 1: absmax * RN(1/7) (torch on a GPU)"""
    x = _c(x, np.float32)
    d = x.shape[-1]
    rows = x.size // d if d else 0
    q = np.empty(x.shape, np.uint8)
    s = np.empty(x.shape[:-1], np.float32)
    lib().oracle_quantize_rows(_p(x, _f32p), rows, d, int(rule), _p(q, _u8p), _p(s, _f32p))
    return q, s


def decode_dequant_h84(cw, scales):
    """fused_kernels.py:272-357 data path -> (fp32 out, n_corrected)"""
    cw = _c(cw, np.uint8)
    scales = _c(scales, np.float32)
    d = cw.shape[-1]
    rows = cw.size // d
    out = np.empty(cw.shape, np.float32)
    nc = np.zeros(1, np.int64)
    lib().oracle_decode_dequant_h84(_p(cw, _u8p), _p(scales, _f32p), rows, d, _p(out, _f32p),
                                    _p(nc, _i64p))
    return out, int(nc[0])


def uint_to_uniform(x):
    return lib().oracle_uint_to_uniform(int(x) & 0xFFFFFFFF)
