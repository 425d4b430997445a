"""The bench's injection launches, alone, for rocprofv3 counter passes
(tools/gpu_r05.sh): Golay int32 codewords M = 45,088,768 x 24 bits at BER 1e-2
(bench.py's inject section), then Hamming(8,4) bytes V = 134,217,728 x 8 bits at
BER 1e-3 (config 2), each REPS times.  Summarised by tools/inject_summary.py."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402
from kvecc import ops  # noqa: E402

REPS = int(os.environ.get("REPS", "3"))
dev = torch.device("cuda:0")
m = 8 * 4096 * 32 * 43
cw = torch.randint(0, 1 << 24, (m,), dtype=torch.int32, device=dev)
out = torch.empty_like(cw)
st = ops.new_stats(dev)
for _ in range(REPS):
    ops.inject_into(cw, out, 1e-2, 24, seed=42, stats=st)
torch.cuda.synchronize()
del cw, out
v = 8 * 4096 * 32 * 128
x = torch.randint(0, 256, (v,), dtype=torch.uint8, device=dev)
y = torch.empty_like(x)
for _ in range(REPS):
    ops.inject_into(x, y, 1e-3, 8, seed=42, stats=st)
torch.cuda.synchronize()
print("inject_pmc done", ops.read_stats(st))
