"""Code definitions, result types and metadata of the codec path.

Mirrors the public names of ecc_codecs/triton_kernels/config.py (the
reference's config module, :34-457) so callers can switch imports.  The
numeric tables the kernels use are built natively (csrc/runtime.hip); the
torch tensors here are for callers that inspect or verify the codes.
"""

from __future__ import annotations

import ctypes
from typing import NamedTuple

import torch

# Launch-granularity constants kept for API compatibility (config.py:34-38).
# The HIP kernels choose their own geometry (16-B lanes, 256-thread groups).
HAMMING74_BLOCK_SIZE = 1024
HAMMING84_BLOCK_SIZE = 1024
GOLAY_BLOCK_SIZE = 256
FAULT_INJECTION_BLOCK_SIZE = 1024
INTERPOLATION_BLOCK_SIZE = 1024

_PHYSICAL_DTYPE = {"hamming74": torch.uint8, "hamming84": torch.uint8, "golay": torch.int32,
                   "int4": torch.uint8, "none": torch.float16}
_CODEWORD_BITS = {"hamming74": 7, "hamming84": 8, "golay": 24}
_DATA_BITS = {"hamming74": 4, "hamming84": 4, "golay": 12}


def get_physical_dtype(codec: str) -> torch.dtype:
    """Storage dtype of a codec's codewords (config.py:41-70)."""
    try:
        return _PHYSICAL_DTYPE[codec]
    except KeyError:
        raise ValueError(f"Unknown codec: {codec}") from None


def get_codeword_bits(codec: str) -> int:
    """Bits per codeword (config.py:73-92)."""
    try:
        return _CODEWORD_BITS[codec]
    except KeyError:
        raise ValueError(f"Unknown codec: {codec}") from None


def get_data_bits(codec: str) -> int:
    """Information bits per codeword (config.py:95-114)."""
    try:
        return _DATA_BITS[codec]
    except KeyError:
        raise ValueError(f"Unknown codec: {codec}") from None


# Hamming(7,4): codeword bits [d0 d1 d2 d3 p0 p1 p2]; the syndrome
# s = s0 | s1<<1 | s2<<2 names the flipped bit (-1: none), config.py:131-161.
_H_SYNDROME_TO_BIT = [-1, 4, 5, 0, 6, 1, 2, 3]
SYNDROME_LUT_HAMMING74 = torch.tensor(_H_SYNDROME_TO_BIT, dtype=torch.int8)
SYNDROME_LUT_HAMMING84 = torch.tensor(_H_SYNDROME_TO_BIT, dtype=torch.int8)


def _bits(rows):
    return torch.tensor(rows, dtype=torch.uint8)


# parity p0 = d0^d1^d3, p1 = d0^d2^d3, p2 = d1^d2^d3 (systematic G = [I | P])
HAMMING74_G = _bits([[1, 0, 0, 0, 1, 1, 0], [0, 1, 0, 0, 1, 0, 1],
                     [0, 0, 1, 0, 0, 1, 1], [0, 0, 0, 1, 1, 1, 1]])
HAMMING74_H = _bits([[1, 1, 0, 1, 1, 0, 0], [1, 0, 1, 1, 0, 1, 0], [0, 1, 1, 1, 0, 0, 1]])
HAMMING84_G = HAMMING74_G
HAMMING84_H = HAMMING74_H

# Golay(24,12): rows of the symmetric 12x12 matrix B as 12-bit masks
# (bit i of row j = B[j][i]); G = [I | B], H = [B^T | I].
_GOLAY_ROW_MASKS = (0xA3B, 0xD1D, 0xE8E, 0xB47, 0xDA3, 0xED1, 0xF68, 0xBB4, 0x9DA, 0x8ED,
                    0xC76, 0x7FF)
GOLAY_B_MATRIX = torch.tensor([[(m >> i) & 1 for i in range(12)] for m in _GOLAY_ROW_MASKS],
                              dtype=torch.uint8)
GOLAY_H_ROW_MASKS = tuple(m | (1 << (12 + i)) for i, m in enumerate(_GOLAY_ROW_MASKS))
GOLAY_UNCORRECTABLE = 0xFFFFFFFF


class ErrorType:
    """SECDED classification written by Hamming(8,4) decode (config.py:197-213)."""

    NO_ERROR = 0
    SINGLE_CORRECTED = 1
    DOUBLE_DETECTED = 2   # data kept uncorrected; interpolation may repair it
    PARITY_ONLY = 3       # only the overall-parity bit flipped; data intact


class DecodeResult(NamedTuple):
    """Hamming(8,4) decode result (config.py:222-242)."""

    data: torch.Tensor
    error_type: torch.Tensor
    corrected_count: int
    detected_count: int


class GolayDecodeResult(NamedTuple):
    """Golay(24,12) decode result (config.py:245-267)."""

    data: torch.Tensor
    errors_corrected: int
    uncorrectable_count: int


def build_golay_syndrome_table() -> torch.Tensor:
    """Syndrome -> error pattern (int32[4096], -1 = uncorrectable).

    Same ordering as config.py:403-457 (weights 1, 2, 3, lexicographic, first
    pattern wins); produced by the native library's table builder.
    """
    from . import _lib
    out = torch.empty(4096, dtype=torch.int32)
    _lib.call("kvecc_golay_syndrome_table_host", ctypes.c_void_p(out.data_ptr()))
    return out
