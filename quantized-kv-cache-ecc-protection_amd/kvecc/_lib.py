"""ctypes binding of libkvecc.so (the C ABI declared in include/kvecc.h).

The library is built in-tree by ``make -C quantized-kv-cache-ecc-protection_amd``
(or ``__graft_entry__.build()``) and lives next to this file.  There is no
fallback: if the library or a GPU is missing, the HIP backend raises.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkvecc.so")

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_f32 = ctypes.c_float
_u8 = ctypes.c_uint8

# name -> argtypes (restype is int status unless listed in _RESTYPE)
SIGNATURES = {
    "kvecc_version": [],
    "kvecc_last_error": [],
    "kvecc_device_count": [],
    "kvecc_time_next_launch": [_vp, _vp],
    "kvecc_init_device": [_int],
    "kvecc_reserve_counter_slots": [_int, _int],
    "kvecc_counter_slots_check": [_int, _vp, _vp],
    "kvecc_debug_fail_graph_retain": [_int],
    "kvecc_golay_syndrome_table_host": [_vp],
    "kvecc_golay_h_row_masks_host": [_vp],
    "kvecc_ber_threshold": [_f32],
    "kvecc_hamming74_encode": [_vp, _vp, _i64, _vp],
    "kvecc_hamming74_decode": [_vp, _vp, _vp, _i64, _vp, _vp],
    "kvecc_hamming84_encode": [_vp, _vp, _i64, _vp],
    "kvecc_hamming84_decode": [_vp, _vp, _vp, _i64, _vp, _vp],
    "kvecc_golay_encode": [_vp, _vp, _i64, _vp],
    "kvecc_golay_decode": [_vp, _vp, _vp, _i64, _vp, _vp],
    "kvecc_golay_encode_rows": [_vp, _vp, _i64, _i64, _vp],
    "kvecc_golay_decode_rows": [_vp, _vp, _i64, _i64, _vp, _vp],
    "kvecc_inject_u8": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _i64, _i64, _vp, _vp],
    "kvecc_inject_i32": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _i64, _i64, _vp, _vp],
    "kvecc_inject_u8_vectorized": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _vp, _vp],
    "kvecc_inject_i32_vectorized": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _vp, _vp],
    "kvecc_inject_rows_u8": [_vp, _vp, _i64, _i64, _int, _i64, _f32, _vp, _vp],
    "kvecc_inject_rows_i32": [_vp, _vp, _i64, _i64, _int, _i64, _f32, _vp, _vp],
    "kvecc_interpolate": [_vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "kvecc_any_equal_u8": [_vp, _i64, _u8, _vp, _vp],
    "kvecc_count_ne_u8": [_vp, _vp, _i64, _vp, _vp],
    "kvecc_mc_trial": [_vp, _i64, _i64, _i64, _i64, _int, _f32, _i64, _i64, _i64, _vp, _vp],
    "kvecc_stats_fold": [_vp, _i64, _int, _vp, _i64, _vp],
    "kvecc_interpolate_auto": [_vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp],
    "kvecc_quantize_encode_rows": [_vp, _int, _int, _int, _vp, _vp, _i64, _i64, _vp],
    "kvecc_decode_dequant_h84_rows": [_vp, _vp, _vp, _int, _i64, _i64, _int, _vp, _vp],
    "kvecc_golay_encode_packed": [_vp, _vp, _i64, _vp],
    "kvecc_golay_decode_packed": [_vp, _vp, _vp, _i64, _vp, _vp],
    "kvecc_hamming84_encode_packed": [_vp, _vp, _i64, _vp],
    "kvecc_hamming84_decode_packed": [_vp, _vp, _vp, _i64, _vp, _vp],
    "kvecc_shim_write": [_vp, _vp, _int, _i64, _i64, _i64, _i64, _int, _int, _int, _int, _f32, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp],
    "kvecc_shim_write_strided": [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _int, _i64, _i64, _i64, _i64, _int, _int, _int, _int, _f32, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp],
    "kvecc_shim_read": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp, _vp, _int, _vp, _vp],
    "kvecc_shim_read_batch": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _int, _int,
                              _vp, _vp, _int, _vp, _vp],
    "kvecc_paged_attention_workspace": [_i64, _i64, _i64, _i64],
    "kvecc_paged_attention": [_vp, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64,
                              _i64, _i64, _i64, _i64, _i64, _i64, _f32, _int, _vp, _i64, _vp],
    # host backend (threads instead of a stream)
    "kvecc_cpu_hamming74_encode": [_vp, _vp, _i64, _int],
    "kvecc_cpu_hamming84_encode": [_vp, _vp, _i64, _int],
    "kvecc_cpu_hamming74_decode": [_vp, _vp, _vp, _i64, _vp, _int],
    "kvecc_cpu_hamming84_decode": [_vp, _vp, _vp, _i64, _vp, _int],
    "kvecc_cpu_golay_encode": [_vp, _vp, _i64, _int],
    "kvecc_cpu_golay_decode": [_vp, _vp, _vp, _i64, _vp, _int],
    "kvecc_cpu_golay_encode_rows": [_vp, _vp, _i64, _i64, _int],
    "kvecc_cpu_golay_decode_rows": [_vp, _vp, _i64, _i64, _vp, _int],
    "kvecc_cpu_golay_encode_packed": [_vp, _vp, _i64, _int],
    "kvecc_cpu_golay_decode_packed": [_vp, _vp, _vp, _i64, _vp, _int],
    "kvecc_cpu_hamming84_encode_packed": [_vp, _vp, _i64, _int],
    "kvecc_cpu_hamming84_decode_packed": [_vp, _vp, _vp, _i64, _vp, _int],
    "kvecc_cpu_inject_u8_vectorized": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _vp, _int],
    "kvecc_cpu_inject_i32_vectorized": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _vp, _int],
    "kvecc_cpu_inject_rows_u8": [_vp, _vp, _i64, _i64, _int, _i64, _f32, _vp, _int],
    "kvecc_cpu_inject_rows_i32": [_vp, _vp, _i64, _i64, _int, _i64, _f32, _vp, _int],
    "kvecc_cpu_inject_u8": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _i64, _i64, _vp, _int],
    "kvecc_cpu_inject_i32": [_vp, _vp, _vp, _i64, _int, _i64, _f32, _i64, _i64, _vp, _int],
    "kvecc_cpu_count_ne_u8": [_vp, _vp, _i64, _vp, _int],
    "kvecc_cpu_interpolate": [_vp, _vp, _vp, _i64, _i64, _i64, _int],
    "kvecc_cpu_quantize_encode_rows": [_vp, _int, _int, _int, _vp, _vp, _i64, _i64, _int],
    "kvecc_cpu_decode_dequant_h84_rows": [_vp, _vp, _vp, _int, _i64, _i64, _int, _vp, _int],
    "kvecc_cpu_shim_write": [_vp, _vp, _int, _i64, _i64, _i64, _i64, _int, _int, _int, _int, _f32, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _int],
    "kvecc_cpu_shim_read": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp, _vp, _int, _vp, _int],
    "kvecc_cpu_shim_read_batch": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _int,
                                  _int, _vp, _vp, _int, _vp, _int],
    "kvecc_cpu_paged_attention": [_vp, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64,
                                  _i64, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _int, _int],
}
_RESTYPE = {
    "kvecc_version": ctypes.c_char_p,
    "kvecc_last_error": ctypes.c_char_p,
    "kvecc_ber_threshold": ctypes.c_uint32,
    "kvecc_paged_attention_workspace": ctypes.c_int64,
}

# dtype / codec codes (include/kvecc.h)
F32, F16, BF16 = 0, 1, 2
CODEC_NONE, CODEC_H74, CODEC_H84, CODEC_GOLAY = 0, 1, 2, 3
CODEC_GOLAY_PACKED = 4  # shim caches only: 3-byte Golay codewords (kvecc.h)
# kvecc_mc_trial codecs (kvecc.h KVECC_MC_*)
MC_CODECS = {"hamming74": 1, "hamming84": 2, "hamming84_interp": 3, "golay": 4}


def golay_packed_row_bytes(g: int) -> int:
    """KVECC_GOLAY_PACKED_ROW: bytes of a packed token row of g Golay codewords."""
    return (3 * g + 3) // 4 * 4
SCALE_DIV7, SCALE_MUL_INV7 = 0, 1
# INT4 row-scale rules (kvecc.h KVECC_SCALE_*): the reference's `abs_max / 7.0`
# (paged_cache_ecc.py:330) as torch computes it on CPU tensors ("div7", IEEE
# division) or on GPU tensors ("mul_inv7", abs_max * RN(1/7))
SCALE_RULES = {"div7": SCALE_DIV7, "mul_inv7": SCALE_MUL_INV7}


def scale_rule_code(rule, default):
    rule = default if rule is None else rule
    if rule not in SCALE_RULES:
        raise ValueError(f"unknown scale rule {rule!r}; expected one of {sorted(SCALE_RULES)}")
    return SCALE_RULES[rule]


class KveccError(RuntimeError):
    """A libkvecc entry point returned a non-zero status."""


_lib = None
_lock = threading.Lock()


def load():
    """Load libkvecc.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} not found: build it with "
                    "`make -C quantized-kv-cache-ecc-protection_amd` or __graft_entry__.build()")
            lib = ctypes.CDLL(LIB_PATH)
            for name, args in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, ctypes.c_int)
            _lib = lib
    return _lib


def call(name, *args):
    """Invoke an int-status entry point; raise KveccError on failure."""
    rc = getattr(load(), name)(*args)
    if rc != 0:
        msg = load().kvecc_last_error().decode(errors="replace")
        raise KveccError(f"{name} failed ({rc}): {msg}")
    return rc


def version() -> str:
    return load().kvecc_version().decode()
