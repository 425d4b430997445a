"""A/B of kvecc_paged_attention across library builds, interleaved in one
process: [B=8, ctx=4096, H=32, D=128] fp16 queries, block 16, Hkv 32 (MHA) and
8 (GQA), encoded caches at BER 1e-3 (H84) / 1e-2 (Golay) -- bench_attention's
workloads.

usage: python tools/exp/run_attn_ab.py lib.so [lib.so ...]   (first = reference)
env: CODECS=hamming84,golay_packed,golay  PASSES=9  ITERS=100

Per pass every library runs ITERS back-to-back calls bracketed by events (the
split + combine kernels, as bench_attention times them), libraries in turn;
the median pass is reported.  Outputs are compared with the first library's.
"""
import ctypes
import math
import os
import statistics
import sys
import time

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import _lib, ops  # noqa: E402

B, CTX, H, D, BS = 8, 4096, 32, 128, 16
PASSES = int(os.environ.get("PASSES", "9"))
ITERS = int(os.environ.get("ITERS", "100"))
CODECS = os.environ.get("CODECS", "hamming84,golay_packed,golay").split(",")


def caches(codec, kvh, dev, g):
    nb = B * CTX // BS
    per = D if codec == "hamming84" else (D + 2) // 3
    if codec == "golay_packed":
        per = (3 * per + 3) // 4 * 4
    dt = torch.int32 if codec == "golay" else torch.uint8
    out = []
    for side in range(2):
        x = torch.randint(0, 16, (nb, 1, kvh, BS, D), device=dev, generator=g, dtype=torch.uint8)
        if codec == "hamming84":
            cw = ops.hamming84_encode(x.view(-1))
            ops.inject_into(cw, cw, 1e-3, 8, seed=42 + side)
            c = cw.view(nb, 1, kvh, BS * per)
        else:
            gg = (D + 2) // 3
            cw = ops.golay_encode_rows(x).view(-1)
            ops.inject_into(cw, cw, 1e-2, 24, seed=42 + side)
            if codec == "golay":
                c = cw.view(nb, 1, kvh, BS * per)
            else:
                c = torch.zeros(nb, 1, kvh, BS, per, dtype=dt, device=dev)
                b3 = torch.stack([(cw >> (8 * k)) & 0xFF for k in range(3)], -1).to(torch.uint8)
                c[..., :3 * gg] = b3.view(nb, 1, kvh, BS, 3 * gg)
                c = c.view(nb, 1, kvh, BS * per)
        out.append(c.contiguous())
    return out, nb


def main():
    dev = torch.device("cuda:0")
    libs = sys.argv[1:] or [_lib.LIB_PATH]
    fns = []
    for p in libs:
        h = ctypes.CDLL(os.path.abspath(p))
        fn = h.kvecc_paged_attention
        fn.argtypes = _lib.SIGNATURES["kvecc_paged_attention"]
        fn.restype = ctypes.c_int
        ws = h.kvecc_paged_attention_workspace
        ws.argtypes = _lib.SIGNATURES["kvecc_paged_attention_workspace"]
        ws.restype = ctypes.c_int64
        fns.append((os.path.basename(p), fn, ws))
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    for codec in CODECS:
        for kvh in (32, 8):
            (kc, vc), nb = caches(codec, kvh, dev, g)
            ks = torch.rand(nb, 1, kvh, BS, device=dev, generator=g)
            vs = torch.rand_like(ks)
            table = torch.randperm(nb, device=dev, generator=g).to(torch.int32).view(B, CTX // BS)
            lens = torch.full((B,), CTX, dtype=torch.int32, device=dev)
            q = torch.randn(B, H, D, device=dev, generator=g).half()
            outs = [torch.empty_like(q) for _ in fns]
            wss = [torch.empty(int(w(B, H, D, CTX)), dtype=torch.float32, device=dev) for _, _, w in fns]

            def call(i):
                rc = fns[i][1](q.data_ptr(), ops._DT[q.dtype], kc.data_ptr(), vc.data_ptr(), table.data_ptr(),
                               lens.data_ptr(), ks.data_ptr(), vs.data_ptr(), outs[i].data_ptr(), B, H, kvh, D,
                               nb, 1, 0, BS, table.shape[1], CTX, 1 / math.sqrt(D), ops.SHIM_CODECS[codec],
                               wss[i].data_ptr(), wss[i].numel(), stream)
                assert rc == 0, (fns[i][0], rc)

            for i in range(len(fns)):
                call(i)
            torch.cuda.synchronize()
            same = [torch.equal(o, outs[0]) for o in outs]
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.5:
                for i in range(len(fns)):
                    for _ in range(50):
                        call(i)
                torch.cuda.synchronize()
            passes = [[] for _ in fns]
            for _ in range(PASSES):
                for i in range(len(fns)):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(ITERS):
                        call(i)
                    e1.record()
                    passes[i].append((e0, e1))
            torch.cuda.synchronize()
            for i, (name, _, _) in enumerate(fns):
                us = [a.elapsed_time(b) * 1e3 / ITERS for a, b in passes[i]]
                print(f"{codec:13s} Hkv {kvh:2d} {name:24s} median {statistics.median(us):6.2f} us  "
                      f"min {min(us):6.2f}  same={same[i]}", flush=True)
            del kc, vc, outs, wss


if __name__ == "__main__":
    main()
