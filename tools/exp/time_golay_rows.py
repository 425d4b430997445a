import sys, torch, statistics
sys.path.insert(0, "quantized-kv-cache-ecc-protection_amd")
from kvecc import ops
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
x = torch.randint(0, 16, (8, 4096, 32, 128), generator=g, dtype=torch.uint8).to(dev)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
def timed(fn, n=7):
    ts = []
    for _ in range(n):
        junk.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)
cw = ops.golay_encode_rows(x)
st = ops.new_stats(dev)
m = cw.numel()
te = timed(lambda: ops.golay_encode_rows(x))
td = timed(lambda: ops.golay_decode_rows(cw, 128, st))
print(f"encode_rows {te:.1f} us ({(x.numel() + 4 * m) / te / 1e3:.0f} GB/s)  decode_rows {td:.1f} us ({(x.numel() + 4 * m) / td / 1e3:.0f} GB/s)")
