"""Object-style codec API: Hamming74, Hamming84, Golay2412.

Same constructor arguments, attributes and return types as the reference's
classes (hamming74_triton.py:285-363, hamming84_triton.py:359-451,
golay_triton.py:506-619).  They run on the codec backend named by `backend`:
"hip" (kvecc.ops) by default, or "cpu" (kvecc.cpu_ops) when `device` is
"cpu" -- the reference's classes accept device="cpu" but then fail inside
their CUDA-only wrappers.  An explicit `backend=` always wins; a "hip" backend
on a CPU device raises, as the reference does.
"""

from __future__ import annotations

import torch

from .backends import get_codec_backend
from .config import (DecodeResult, GOLAY_B_MATRIX, GOLAY_H_ROW_MASKS, GOLAY_UNCORRECTABLE,
                     GolayDecodeResult, HAMMING74_G, HAMMING74_H, HAMMING84_G, HAMMING84_H,
                     SYNDROME_LUT_HAMMING74, SYNDROME_LUT_HAMMING84, build_golay_syndrome_table)


def _backend(device, backend):
    if backend is None:
        backend = "cpu" if torch.device(device).type == "cpu" else "hip"
    return get_codec_backend(backend)


class Hamming74:
    """Hamming(7,4) single-error-correcting codec."""

    G = HAMMING74_G
    H = HAMMING74_H
    SYNDROME_TO_POSITION = SYNDROME_LUT_HAMMING74

    def __init__(self, device: str = "cuda", backend: str | None = None):
        self.device = device
        self.ops = _backend(device, backend)
        self._G = self.G.to(device)
        self._H = self.H.to(device)
        self._syndrome_lut = self.SYNDROME_TO_POSITION.to(device)

    def encode(self, int4_values: torch.Tensor) -> torch.Tensor:
        return self.ops.hamming74_encode(int4_values.to(self.device))

    def decode(self, codewords: torch.Tensor):
        """-> (decoded, error_detected as bool)"""
        decoded, flag, _ = self.ops.hamming74_decode(codewords.to(self.device),
                                                return_error_detected=True)
        return decoded, flag.bool()

    def encode_batch(self, int4_tensor):
        return self.encode(int4_tensor)

    def decode_batch(self, codeword_tensor):
        return self.decode(codeword_tensor)


class Hamming84:
    """Hamming(8,4) SECDED codec (double errors detected, data kept)."""

    G_74 = HAMMING84_G
    H_74 = HAMMING84_H
    SYNDROME_TO_POSITION = SYNDROME_LUT_HAMMING84

    def __init__(self, device: str = "cuda", on_double_error: str = "zero",
                 backend: str | None = None):
        self.device = device
        self.ops = _backend(device, backend)
        self.on_double_error = on_double_error  # accepted for compatibility; unused
        self._G = self.G_74.to(device)
        self._H = self.H_74.to(device)
        self._syndrome_lut = self.SYNDROME_TO_POSITION.to(device)

    def encode(self, int4_values: torch.Tensor) -> torch.Tensor:
        return self.ops.hamming84_encode(int4_values.to(self.device))

    def decode(self, codewords: torch.Tensor) -> DecodeResult:
        data, etype, (corrected, detected) = self.ops.hamming84_decode(
            codewords.to(self.device), return_error_types=True)
        return DecodeResult(data=data, error_type=etype, corrected_count=corrected,
                            detected_count=detected)


class Golay2412:
    """Extended Golay(24,12) codec over INT4 triplets (corrects 3 bit errors)."""

    UNCORRECTABLE = GOLAY_UNCORRECTABLE

    def __init__(self, device: str = "cuda", backend: str | None = None):
        self.device = device
        self.ops = _backend(device, backend)
        self.G, self.H, self.P = self._build_matrices()
        self.syndrome_table = build_golay_syndrome_table().to(device)
        self.h_row_masks = torch.tensor(GOLAY_H_ROW_MASKS, dtype=torch.int64, device=device)

    def _build_matrices(self):
        b = GOLAY_B_MATRIX.to(self.device)
        eye = torch.eye(12, dtype=torch.uint8, device=self.device)
        return torch.cat([eye, b], dim=1), torch.cat([b.T, eye], dim=1), b

    def encode(self, triplets: torch.Tensor) -> torch.Tensor:
        """[N,3] -> int64 [N] (the reference returns int64 here, :577)."""
        return self.ops.golay_encode(triplets.to(self.device)).to(torch.int64)

    def decode(self, codewords: torch.Tensor) -> GolayDecodeResult:
        data, (bits, unc) = self.ops.golay_decode(codewords.to(torch.int32).to(self.device))
        return GolayDecodeResult(data=data, errors_corrected=bits, uncorrectable_count=unc)

    def verify_properties(self) -> bool:
        """G @ H^T == 0 over GF(2)."""
        prod = (self.G.float() @ self.H.T.float()) % 2
        return bool(prod.sum() == 0)
