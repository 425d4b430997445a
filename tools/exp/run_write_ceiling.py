"""Write-only HBM rate by store cache policy (tools/exp/golay_exp.hip
write_only_pol): plain / nt / sc1 / sc0 sc1 / nt sc1 / sc0, 512 MB, cold."""
import ctypes, os, statistics, torch
HERE = os.path.dirname(os.path.abspath(__file__))
VP = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "libexp.so"))
lib.exp_ceiling.argtypes = [VP, VP, ctypes.c_int64, ctypes.c_int, ctypes.c_int, VP]
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
names = {7: "global nt", 8: "global plain", 9: "buffer aux0", 10: "buffer nt", 11: "buffer sc1",
         12: "buffer sc0sc1", 13: "buffer nt sc1", 14: "buffer sc0"}
for mb in (256, 512):
    dst = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    for v, nm in names.items():
        for grid in (2048, 8192):
            ts = []
            for _ in range(7):
                junk.fill_(1)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                assert lib.exp_ceiling(VP(dst.data_ptr()), VP(dst.data_ptr()), dst.numel(), v, grid, s) == 0
                b.record(); torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            med = statistics.median(ts)
            print(f"{mb:4d} MB {nm:14s} grid {grid:5d}: {dst.numel() / med / 1e3:6.0f} GB/s", flush=True)
    del dst
