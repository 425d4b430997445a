"""Codec backend registry.

The reference has no codec-backend selector (its ECCShimConfig has no
`backend`, ecc_shim.py:165-186); its only registry is the quantizer one,
QUANTIZER_BACKENDS / get_quantizer (ecc_codecs/quantization_backends.py:672-706).
This module introduces the codec selector in that idiom: a name -> backend
table and a factory that raises ValueError on unknown names.

A backend is any object exposing the reference's codec function set
(`FUNCTIONS`).  "hip" is the MI355X implementation and the default; it never
falls back to anything else.  "cpu" is the host twin built from the same
codec algebra (kvecc.cpu_ops); it is used only when asked for by name.
"""

from __future__ import annotations

import importlib
import types

import torch

FUNCTIONS = (
    "hamming74_encode", "hamming74_decode", "hamming84_encode", "hamming84_decode",
    "golay_encode", "golay_decode", "inject_bit_errors_triton", "interpolate_double_errors",
    "fused_quantize_encode_hamming84", "fused_quantize_encode_hamming74",
    "fused_decode_dequantize_hamming84",
)

# backend name -> module implementing FUNCTIONS
CODEC_BACKENDS = {
    "hip": "kvecc.ops",
    "cpu": "kvecc.cpu_ops",  # host twin (BASELINE config 1); explicit, never a fallback
}

DEFAULT_BACKEND = "hip"


def available_backends():
    return tuple(CODEC_BACKENDS)


def register_codec_backend(name: str, module_path: str) -> None:
    """Register an additional backend module under `name`."""
    CODEC_BACKENDS[name.lower().replace("-", "_")] = module_path


def get_codec_backend(backend: str = DEFAULT_BACKEND) -> types.ModuleType:
    """Return the backend module for `backend` (case/dash-insensitive).

    Raises ValueError for unknown names, like get_quantizer.
    """
    key = str(backend).lower().replace("-", "_")
    if key not in CODEC_BACKENDS:
        raise ValueError(f"Unknown codec backend '{backend}'. "
                         f"Available backends: {', '.join(CODEC_BACKENDS)}")
    mod = importlib.import_module(CODEC_BACKENDS[key])
    missing = [f for f in FUNCTIONS if not hasattr(mod, f)]
    if missing:
        raise ValueError(f"codec backend '{backend}' lacks {missing}")
    if key == "hip":
        require_hip()
    elif key == "cpu":
        from . import _lib
        _lib.load()
    return mod


def require_hip() -> None:
    """Fail loudly unless libkvecc.so is built and a GPU is visible."""
    from . import _lib
    _lib.load()
    if not torch.cuda.is_available():
        raise RuntimeError("the 'hip' codec backend needs a visible AMD GPU (none found)")
