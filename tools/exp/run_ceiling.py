"""HBM ceiling study on the GPU box: copy / read-only / write-only kernels."""
import ctypes, json, os, statistics, sys
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
VP = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "libexp.so"))
lib.exp_ceiling.argtypes = [VP, VP, ctypes.c_int64, ctypes.c_int, ctypes.c_int, VP]
dev = torch.device("cuda:0")
s = VP(torch.cuda.current_stream().cuda_stream)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
names = ["copy_nt_u4_b256", "copy_nt_u2_b256", "copy_nt_u1_b256", "copy_nt_u4_b512", "copy_nt_u2_b1024",
         "read_nt", "read_plain", "write_nt", "write_plain"]
res = {}
for mb in (180, 512, 1024):
    src = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    for v, nm in enumerate(names):
        for grid in (1024, 2048, 4096, 8192):
            ts = []
            for _ in range(6):
                junk.fill_(1)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                assert lib.exp_ceiling(VP(src.data_ptr()), VP(dst.data_ptr()), src.numel(), v, grid, s) == 0
                b.record(); torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            byts = src.numel() * (2 if nm.startswith("copy") else 1)
            med = statistics.median(ts)
            res[f"{nm}_{mb}MB_g{grid}"] = round(byts / med / 1e3)
    del src, dst
best = sorted(res.items(), key=lambda kv: -kv[1])
print(json.dumps(dict(best[:25]), indent=0))
print(json.dumps({k: v for k, v in res.items() if "g2048" in k}, indent=0))
