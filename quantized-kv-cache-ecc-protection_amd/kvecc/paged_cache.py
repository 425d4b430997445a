"""Non-paged quantize+encode helpers of kv_cache/paged_cache_ecc.py.

compute_quantization_scales (:302-334) and write_kv_to_cache_simple
(:337-397) with the reference's arithmetic: absmax/7 in the input dtype
(0 -> 1), torch.round (half-even) of kv/scale in the input dtype, clamp
[-8, 7] + 8, then the codec's encoder -- the HIP backend for GPU tensors, the
host backend for CPU tensors (the reference moves CPU input to CUDA first).
The scalar paged write kernel (:201-299) is unused by the reference product
and hard-codes 32 layers; the shim's fused write (kvecc_shim_write) replaces it.
"""

from __future__ import annotations

import torch

from .backends import get_codec_backend


def compute_quantization_scales(tensor, dim=-1):
    scales = tensor.abs().max(dim=dim, keepdim=False).values / 7.0
    return torch.where(scales == 0, torch.ones_like(scales), scales)


def _backend_for(t):
    return get_codec_backend("cpu" if t.device.type == "cpu" else "hip")


def write_kv_to_cache_simple(kv, codec="hamming84", scale=None):
    """-> (encoded, scales): uint8 codewords of kv's shape for "hamming84",
    int32 Golay codewords of the zero-padded flat triplets for "golay", raw
    INT4 otherwise."""
    if scale is None:
        scale = compute_quantization_scales(kv, dim=-1)
    quantized = torch.round(kv / scale.unsqueeze(-1)).clamp(-8, 7) + 8
    int4_vals = quantized.to(torch.uint8)
    be = _backend_for(int4_vals)
    if codec == "hamming84":
        encoded = be.hamming84_encode(int4_vals.flatten()).view(int4_vals.shape)
    elif codec == "golay":
        flat = int4_vals.flatten()
        pad = (3 - flat.numel() % 3) % 3
        if pad:
            flat = torch.cat([flat, flat.new_zeros(pad)])
        encoded = be.golay_encode(flat.view(-1, 3))
    else:
        encoded = int4_vals
    return encoded, scale
