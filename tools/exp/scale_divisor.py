"""How torch divides a tensor by a Python scalar on the GPU vs the CPU.

compute_quantization_scales (kv_cache/paged_cache_ecc.py:330) computes
`abs_max / 7.0`.  On a GPU, PyTorch multiplies by the reciprocal of a CPU-scalar
divisor; on the CPU it divides.  This script counts, for every positive finite
fp16/bf16 row max (and a fp32 sample), how often the two results differ.
usage: python tools/exp/scale_divisor.py   (needs a GPU)
"""
import json

import torch

d = torch.device("cuda:0")
res = {}
inv = torch.tensor([1.0]) / torch.tensor([7.0])  # RN(1/7) in fp32
for dt, top in ((torch.float16, 0x7C00), (torch.bfloat16, 0x7F80)):
    a = torch.arange(1, top, dtype=torch.int32).to(torch.int16).view(dt).float()
    cpu = a / 7.0
    gpu = (a.to(d) / 7.0).cpu()
    res[str(dt)] = {"n": a.numel(), "gpu_ne_cpu": int((gpu != cpu).sum()),
                    "gpu_equals_mul_by_rn_inverse": bool(torch.equal(gpu, a * inv)),
                    "gpu_tensor_div_equals_cpu": bool(torch.equal(
                        (a.to(d) / torch.full_like(a.to(d), 7.0)).cpu(), cpu))}
x = torch.randn(1 << 22, generator=torch.Generator().manual_seed(0)).abs() * 3
res["randn_f32"] = {"n": x.numel(), "gpu_ne_cpu": int(((x.to(d) / 7.0).cpu() != x / 7.0).sum())}
print(json.dumps(res))
