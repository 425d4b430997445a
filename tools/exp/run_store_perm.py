"""The fused-read byte mix (2816 B read + 4096 B written per 16-row tile) with
the reads gathered through a random block table like the shim cache's
(store_ceiling.hip probe_perm), against the same with sequential reads: one
unit per wave, full grid, 8 / 12 / 16 waves per CU.  How much of the gap
between the fused Golay read and the sequential probe is the gather."""
import ctypes, os, statistics, torch
HERE = os.path.dirname(os.path.abspath(__file__))
VP, U32, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
lib = ctypes.CDLL(os.path.join(HERE, "libstore.so"))
lib.store_probe_perm.argtypes = [VP, VP, U32, VP, I, VP]
dev = torch.device("cuda:0")
sp = VP(torch.cuda.current_stream().cuda_stream)
UNITS = 131072
src = torch.empty(UNITS * 2816, dtype=torch.uint8, device=dev).random_(0, 256)
dst = torch.empty(UNITS * 4096, dtype=torch.uint8, device=dev)
perm = torch.randperm(2048, generator=torch.Generator().manual_seed(7)).to(torch.int32).to(dev)
for wpc in (8, 12, 16):
    lds = (160 * 1024 // (wpc // 4)) & ~1023
    for name, pp in (("sequential", None), ("block table", perm)):
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(8):
                assert lib.store_probe_perm(VP(src.data_ptr()), VP(dst.data_ptr()), UNITS,
                                            VP(pp.data_ptr()) if pp is not None else None, lds, sp) == 0
            b.record(); torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / 8)
        us = statistics.median(ts)
        print(f"{wpc:2d} w/CU {name:12s}: {us:6.1f} us {UNITS * 6912 / us / 1e3:5.0f} GB/s", flush=True)
