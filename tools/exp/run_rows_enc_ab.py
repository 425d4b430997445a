"""A/B of kvecc_golay_encode_rows across library builds (product first),
interleaved in one process, on [8,4096,32,128] (43 codewords per head row) and
a few ragged row counts; outputs must equal the first library's bit for bit.
usage: python tools/exp/run_rows_enc_ab.py lib.so [lib.so ...]"""
import ctypes, os, statistics, sys
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402
from kvecc import _lib  # noqa: E402

dev = torch.device("cuda:0")
libs = []
for p in sys.argv[1:]:
    h = ctypes.CDLL(os.path.abspath(p))
    fn = h.kvecc_golay_encode_rows
    fn.argtypes = _lib.SIGNATURES["kvecc_golay_encode_rows"]
    fn.restype = ctypes.c_int
    libs.append((os.path.basename(p), fn))
s = torch.cuda.current_stream().cuda_stream
gen = torch.Generator().manual_seed(3)
for rows, d in ((8 * 4096 * 32, 128), (1000003, 128), (4099, 64), (77777, 96), (5, 256)):
    g = (d + 2) // 3
    x = torch.randint(0, 16, (rows, d), generator=gen, dtype=torch.uint8).to(dev)
    outs = [torch.full((rows, g), -1, dtype=torch.int32, device=dev) for _ in libs]
    call = lambda i: libs[i][1](x.data_ptr(), outs[i].data_ptr(), rows, d, s)  # noqa: E731
    for i in range(len(libs)):
        assert call(i) == 0
    torch.cuda.synchronize()
    same = [torch.equal(o, outs[0]) for o in outs]
    ts = [[] for _ in libs]
    for _ in range(40):
        for i in range(len(libs)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); call(i); b.record()
            ts[i].append((a, b))
    torch.cuda.synchronize()
    nb = rows * (d + 4 * g)
    for i, (name, _) in enumerate(libs):
        us = statistics.median(a.elapsed_time(b) * 1e3 for a, b in ts[i])
        print(f"rows={rows:8d} d={d:3d} {name:18s} equal={same[i]} median {us:7.1f} us "
              f"{nb / us / 1e3:5.0f} GB/s ({nb / us / 8e4:.1f}% of 8 TB/s)", flush=True)
