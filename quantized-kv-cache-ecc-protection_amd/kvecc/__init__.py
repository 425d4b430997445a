"""kvecc -- MI355X-native ECC protection for INT4 KV caches.

Drop-in for the reference's ``ecc_codecs.triton_kernels`` package (same public
names, see its ``__init__.py:58-99``), implemented as hand-written HIP kernels
for gfx950 behind the C ABI of include/kvecc.h.
"""

from .backends import (CODEC_BACKENDS, available_backends, get_codec_backend,
                       register_codec_backend, require_hip)
from .codecs import Golay2412, Hamming74, Hamming84
from .config import (DecodeResult, ErrorType, FAULT_INJECTION_BLOCK_SIZE, GOLAY_B_MATRIX,
                     GOLAY_BLOCK_SIZE, GOLAY_H_ROW_MASKS, GolayDecodeResult, HAMMING74_BLOCK_SIZE,
                     HAMMING74_G, HAMMING74_H, HAMMING84_BLOCK_SIZE, HAMMING84_G, HAMMING84_H,
                     INTERPOLATION_BLOCK_SIZE, SYNDROME_LUT_HAMMING74, SYNDROME_LUT_HAMMING84,
                     build_golay_syndrome_table, get_codeword_bits, get_data_bits,
                     get_physical_dtype)
from .ops import (fused_decode_dequantize_hamming84, fused_quantize_encode_hamming74,
                  fused_quantize_encode_hamming84, golay_decode, golay_encode, hamming74_decode,
                  hamming74_encode, hamming84_decode, hamming84_encode, inject_bit_errors,
                  inject_bit_errors_triton, inject_bit_errors_triton_batched,
                  inject_bit_errors_triton_vectorized, interpolate_double_errors,
                  interpolate_double_errors_1d, interpolate_double_errors_autotuned,
                  paged_attention_ecc)
from . import torch_ops  # noqa: F401  -- registers torch.ops.kvecc.* (CPU + HIP kernels, fake kernels)

__version__ = "0.1.0"

__all__ = [
    "paged_attention_ecc",
    "get_physical_dtype", "get_codeword_bits", "get_data_bits",
    "HAMMING74_BLOCK_SIZE", "HAMMING84_BLOCK_SIZE", "GOLAY_BLOCK_SIZE",
    "FAULT_INJECTION_BLOCK_SIZE", "INTERPOLATION_BLOCK_SIZE",
    "SYNDROME_LUT_HAMMING74", "SYNDROME_LUT_HAMMING84", "ErrorType", "DecodeResult",
    "GolayDecodeResult", "HAMMING74_G", "HAMMING74_H", "HAMMING84_G", "HAMMING84_H",
    "GOLAY_B_MATRIX", "GOLAY_H_ROW_MASKS", "build_golay_syndrome_table",
    "Hamming74", "Hamming84", "Golay2412",
    "hamming74_encode", "hamming74_decode", "hamming84_encode", "hamming84_decode",
    "golay_encode", "golay_decode", "inject_bit_errors_triton", "inject_bit_errors",
    "inject_bit_errors_triton_batched", "inject_bit_errors_triton_vectorized",
    "interpolate_double_errors", "interpolate_double_errors_1d",
    "interpolate_double_errors_autotuned",
    "fused_quantize_encode_hamming84", "fused_quantize_encode_hamming74",
    "fused_decode_dequantize_hamming84",
    "CODEC_BACKENDS", "get_codec_backend", "register_codec_backend", "available_backends",
    "require_hip",
]
