"""Per-head Golay rows encode/decode throughput vs head_dim: is the encode's
output tile alignment (16 rows x 4g bytes: 2752 B at d=128, not a multiple of
128 B; 2048 B at d=96; 4096 B at d=192) what keeps it below the flat encode?
Same total values (2^27) per case; back-to-back launches, median of 30."""
import statistics, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "quantized-kv-cache-ecc-protection_amd"))
import torch
from kvecc import ops
dev = torch.device("cuda:0")
gen = torch.Generator().manual_seed(0)
for d in (96, 128, 192, 64, 256):
    g = (d + 2) // 3
    rows = (1 << 27) // d
    x = torch.randint(0, 16, (rows, d), generator=gen, dtype=torch.uint8).to(dev)
    cw = torch.empty(rows, g, dtype=torch.int32, device=dev)
    y = torch.empty_like(x)
    st = ops.new_stats(dev)
    res = {}
    for name, fn in (("encode", lambda: ops.golay_encode_rows_into(x, cw)),
                     ("decode", lambda: ops.golay_decode_rows_into(cw, y, st))):
        for _ in range(5):
            fn()
        ts = []
        for _ in range(30):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); fn(); b.record(); torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res[name] = statistics.median(ts)
    assert torch.equal(y, x)
    nb = rows * (d + 4 * g)
    print(f"d={d:3d} g={g:2d} tile_out={16 * 4 * g:5d} B  encode {res['encode']:6.1f} us "
          f"{nb / res['encode'] / 1e3:5.0f} GB/s  decode {res['decode']:6.1f} us {nb / res['decode'] / 1e3:5.0f} GB/s",
          flush=True)
