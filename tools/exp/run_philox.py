import ctypes, os, statistics, torch
HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libphilox.so"))
lib.philox_bench.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
out = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
blocks, iters = 8192, 8
res = {0: [], 1: []}
chk = {}
for rnd in range(6):
    for f in (0, 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); assert lib.philox_bench(f, ctypes.c_void_p(out.data_ptr()), blocks, iters, s) == 0; b.record()
        torch.cuda.synchronize()
        res[f].append(a.elapsed_time(b) * 1e-3)
        chk[f] = int(out[: blocks * 256].sum())
n = blocks * 256 * iters * 24
for f in (0, 1):
    t = statistics.median(res[f])
    print(f"form {f}: {t*1e3:.3f} ms  {n / t:.3e} philox/s  checksum {chk[f]}")
