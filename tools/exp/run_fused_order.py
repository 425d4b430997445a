"""bench.py's fused H(8,4) read section (plain, then interpolating) three times in a
row, and once in the other order: is the interpolating read's gap to the plain
read in the bench a property of the kernels or of the measuring order?"""
import json
import os
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda:0")
from kvecc import ops  # noqa: E402,F401
for rep in range(3):
    r = bench.fused_h84_bench(dev, 50, 100)
    print(json.dumps({"rep": rep, "plain_us": r["plain"]["kernel_ms"] * 1e3, "interp_us": r["interp"]["kernel_ms"] * 1e3}),
          flush=True)
