"""A/B of the interpolating Hamming(8,4) fused read (kvecc_shim_read_batch ->
shim_read_bytes_tiles_kernel<H84, INTERP>) across library builds, interleaved
in one process: [B=8, L=4096, Hkv=32, D=128] K+V, block_size 16, BER 1e-3,
fp16 out, random block table.

usage: python tools/exp/run_shim_read_interp.py [lib.so ...]   (product lib first)
Prints per-lib median / min kernel time and whether outputs + statistics equal
the first lib's (the NOHALO / NOVALU ceiling builds are expected to differ).
"""
import ctypes
import os
import statistics
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import _lib, ops  # noqa: E402

B, L, H, D, BS = 8, 4096, 32, 128, 16
BER = float(os.environ.get("BER", "1e-3"))
ROUNDS = int(os.environ.get("ROUNDS", "30"))
INTERP = int(os.environ.get("INTERP", "1"))


def main():
    dev = torch.device("cuda:0")
    libs = sys.argv[1:] or [_lib.LIB_PATH]
    handles = []
    for p in libs:
        h = ctypes.CDLL(os.path.abspath(p))
        fn = h.kvecc_shim_read_batch
        fn.argtypes = _lib.SIGNATURES["kvecc_shim_read_batch"]
        fn.restype = ctypes.c_int
        handles.append((os.path.basename(p), fn))
    nlb = L // BS
    nb = B * nlb
    gen = torch.Generator().manual_seed(7)
    caches, scales = [], []
    for side in range(2):
        x = torch.randint(0, 16, (nb * H * BS * D,), generator=gen, dtype=torch.uint8).to(dev)
        cw = ops.hamming84_encode(x)
        ops.inject_into(cw, cw, BER, 8, seed=42 + side)
        caches.append(cw.view(nb, 1, H, BS * D).contiguous())
        scales.append((torch.rand(nb, 1, H, BS, generator=gen) * 0.1 + 0.01).to(dev))
    table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
    if os.environ.get("TABLE") == "seq":
        table = torch.arange(nb, dtype=torch.int32).view(B, nlb).to(dev)
    table[1, 5] = -1
    table[6, 200] = -1
    outs = [(torch.empty(B, H, L, D, dtype=torch.float16, device=dev),
             torch.empty(B, H, L, D, dtype=torch.float16, device=dev)) for _ in handles]
    stats = [ops.new_stats(dev) for _ in handles]
    times = [[] for _ in handles]
    stream = torch.cuda.current_stream(dev).cuda_stream

    def call(i):
        name, fn = handles[i]
        rc = fn(caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
                table.data_ptr(), table.shape[1], B, L, H, D, 1, BS, 0, ops.SHIM_CODECS["hamming84"], INTERP,
                outs[i][0].data_ptr(), outs[i][1].data_ptr(), ops._DT[torch.float16], stats[i].data_ptr(), stream)
        assert rc == 0, (name, rc)

    for i in range(len(handles)):
        for _ in range(3):
            call(i)
    for s in stats:
        s.zero_()
    for i in range(len(handles)):
        call(i)
    torch.cuda.synchronize()
    for i, (name, _) in enumerate(handles):
        same = torch.equal(outs[i][0], outs[0][0]) and torch.equal(outs[i][1], outs[0][1])
        print(f"{name}: outputs equal first={same} stats={ops.read_stats(stats[i])}", flush=True)
    for _ in range(ROUNDS):
        for i in range(len(handles)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call(i)
            e1.record()
            times[i].append((e0, e1))
    torch.cuda.synchronize()
    nbytes = 2 * B * L * H * (D + 4 + 2 * D)
    for i, (name, _) in enumerate(handles):
        us = [a.elapsed_time(b) * 1e3 for a, b in times[i]]
        med = statistics.median(us)
        print(f"interp={INTERP} {name}: median {med:.1f} us min {min(us):.1f} "
              f"({nbytes / med / 1e3:.0f} GB/s, {nbytes / med / 1e3 / 8000 * 100:.1f}% of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
