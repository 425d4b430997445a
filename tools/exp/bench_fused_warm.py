"""bench.py's fused-read sections run standalone in a fresh process with W
warm-up calls (argv: W values, e.g. 5 100 5), to separate the warm-up count
from the sections' order inside bench.py."""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
for w in [int(x) for x in sys.argv[1:]] or [5, 100]:
    h = bench.fused_h84_bench(dev, 50, w)
    g = bench.fused_decode_bench(dev, 50, w)
    print(json.dumps({"warmup": w, "h84_plain_us": round(h["plain"]["kernel_ms"] * 1e3, 1),
                      "h84_interp_us": round(h["interp"]["kernel_ms"] * 1e3, 1),
                      "golay_us": round(g["kernel_ms"] * 1e3, 1)}), flush=True)
