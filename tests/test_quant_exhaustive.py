"""Exhaustive check of the fused quantizer's division for 16-bit inputs.

For fp16/bf16 rows the quantize kernels compute x / scale as a reciprocal
multiply with one FMA correction (codec_math.h div_recip) instead of IEEE
division.  The shim's torch path (ecc_shim.py:572-580) divides in IEEE fp32,
so this test runs EVERY finite 16-bit value x against EVERY finite positive
16-bit row max through kvecc_quantize_encode_rows, under both scale rules, and
compares nibbles and scales with torch bit for bit.  Rows are [x0..x6, amax];
a row whose |x| exceeds amax simply tests another (x, max) pair.

The references: "div7" divides tensor by tensor (IEEE on either device);
"mul_inv7" is the reference's own `abs_max / 7.0` (paged_cache_ecc.py:330) on
the GPU.  torch's device division is pinned against host division on the
first chunk.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

INV7 = torch.tensor([1.0]) / torch.tensor([7.0])  # RN(1/7)


def _finite_codes(dtype):
    codes = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16)
    vals = codes.view(dtype)
    return codes[torch.isfinite(vals.float())]


def _reference(rows, rule):
    xf = rows.float()
    amax = xf.abs().amax(-1)
    if rule == "div7":
        scale = amax / torch.full_like(amax, 7.0)
    else:
        scale = amax * INV7.to(amax.device)
    scale = torch.where(scale == 0, torch.ones_like(scale), scale)
    q = torch.round(xf / scale.unsqueeze(-1)).clamp(-8, 7) + 8
    return q.to(torch.uint8), scale


@pytest.mark.parametrize("rule", ["div7", "mul_inv7"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_quantize_every_value_against_every_row_max(gpu, dtype, rule):
    from kvecc import ops
    xs = _finite_codes(dtype)
    pad = (-xs.numel()) % 7
    xs = torch.cat([xs, xs.new_zeros(pad)]).view(-1, 7).to(gpu)         # [nx, 7]
    amaxes = _finite_codes(dtype)
    amaxes = amaxes[amaxes > 0].to(gpu)                                  # positive finite
    nx, chunk = xs.shape[0], 384
    rows = torch.empty(chunk, nx, 8, dtype=torch.int16, device=gpu)
    rows[:, :, :7] = xs
    checked = 0
    for c0 in range(0, amaxes.numel(), chunk):
        a = amaxes[c0:c0 + chunk]
        r = rows[:a.numel()]
        r[:, :, 7] = a.unsqueeze(1)
        x = r.view(-1, 8).view(dtype)
        nib, scales = ops.quantize_rows(x, scale_rule=rule)
        ref_nib, ref_scale = _reference(x, rule)
        if c0 == 0:
            cn, cs = _reference(x[:200000].cpu(), rule)  # torch device vs host arithmetic
            assert torch.equal(cn, ref_nib[:200000].cpu()) and torch.equal(cs, ref_scale[:200000].cpu())
        if rule == "mul_inv7":  # the reference's expression on the GPU
            amax = x.float().abs().amax(-1)
            assert torch.equal(torch.where(amax == 0, torch.ones_like(amax), amax / 7.0), ref_scale)
        bad = (nib != ref_nib).any(-1)
        if bad.any():
            i = int(bad.nonzero()[0, 0])
            raise AssertionError(f"row {x[i].tolist()}: kernel {nib[i].tolist()} "
                                 f"torch {ref_nib[i].tolist()}")
        assert torch.equal(scales.view(torch.int32), ref_scale.view(torch.int32))
        checked += x.shape[0] * 7
    assert checked >= 7 * nx * amaxes.numel()
