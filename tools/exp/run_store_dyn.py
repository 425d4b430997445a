"""Fused-read byte mix with dynamically scheduled persistent workgroups
(store_ceiling.hip probe_dyn) against the one-unit-per-wave full grid (probe,
chunk 1) at the same waves per CU.  Kernel times from dispatch stamps
(hipExtLaunchKernelGGL events), the counters zeroed before each launch."""
import ctypes, os, statistics, torch
HERE = os.path.dirname(os.path.abspath(__file__))
VP, U32, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
lib = ctypes.CDLL(os.path.join(HERE, "libstore.so"))
lib.store_probe_dyn.argtypes = [VP, VP, U32, VP, I, I, VP, VP, VP]
lib.store_probe.argtypes = [VP, VP, U32, U32, U32, I, I, I, I, I, I, VP]
lib.store_probe_mode.argtypes = [U32, U32, VP]
dev = torch.device("cuda:0")
sp = VP(torch.cuda.current_stream().cuda_stream)
NCU = torch.cuda.get_device_properties(0).multi_processor_count
UNITS, RCH, WCH = 131072, 2816, 4096
src = torch.empty(UNITS * RCH, dtype=torch.uint8, device=dev).random_(0, 256)
dst = torch.empty(UNITS * WCH, dtype=torch.uint8, device=dev)
ctr = torch.zeros(8 * 32, dtype=torch.int32, device=dev)
for wpc in (8, 12, 16, 24, 32):
    wg = wpc // 4
    lds = (160 * 1024 // wg) & ~1023
    grid = NCU * wg
    ts = []
    for rep in range(25):
        ctr.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); b.record()
        assert lib.store_probe_dyn(VP(src.data_ptr()), VP(dst.data_ptr()), UNITS, VP(ctr.data_ptr()), grid, lds,
                                   VP(a.cuda_event), VP(b.cuda_event), sp) == 0
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    us = statistics.median(ts[5:])
    print(f"DYN  {wpc:2d}w/CU grid={grid:5d}: {us:7.1f} us {UNITS * (RCH + WCH) / us / 1e3:6.0f} GB/s", flush=True)
    lib.store_probe_mode(1, 0, None)
    ts = []
    for rep in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(8):
            lib.store_probe(VP(src.data_ptr()), VP(dst.data_ptr()), RCH, WCH, UNITS, 16, 1, 0, 256, UNITS // 4, lds, sp)
        b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / 8)
    us = statistics.median(ts)
    print(f"FULL {wpc:2d}w/CU grid={UNITS // 4:5d}: {us:7.1f} us {UNITS * (RCH + WCH) / us / 1e3:6.0f} GB/s", flush=True)
    lib.store_probe_mode(0, 0, None)
