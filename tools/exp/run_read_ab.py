"""A/B of the fused shim reads (kvecc_shim_read_batch) across library builds,
interleaved in one process: Golay int32 / packed and Hamming(8,4) plain /
interpolating, [B=8, L=4096, Hkv=32, D=128] K+V, block 16, fp16 out (the
bench's fused-read workloads; Golay at BER 1e-2, H84 at 1e-3).

usage: python tools/exp/run_read_ab.py lib.so [lib.so ...]  (first = reference)

Times are the kernels' own dispatch stamps (kvecc_time_next_launch), median
over ROUNDS interleaved rounds (BLOCK=n: n consecutive launches per library in
turn, as bench.py times them); outputs and statistics are compared with the
first library's.
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
ROUNDS = int(os.environ.get("ROUNDS", "40"))
ODT = torch.float32 if os.environ.get("OUT") == "fp32" else torch.float16
CASES = os.environ.get("CASES", "golay,golay_packed,hamming84,hamming84+interp").split(",")


def golay_caches(dev, packed, gen, nb):
    g = (D + 2) // 3
    out = []
    for side in range(2):
        x = torch.randint(0, 16, (nb, 1, H, BS, D), generator=gen, dtype=torch.uint8).to(dev)
        cw = ops.golay_encode_rows(x).view(-1)
        ops.inject_into(cw, cw, 1e-2, 24, seed=42 + side)
        cw = cw.view(nb, 1, H, BS * g)
        if packed:
            cw = torch.stack([(cw >> (8 * k)) & 0xFF for k in range(3)], -1).to(torch.uint8)
            cw = cw.view(nb, 1, H, BS, 3 * g)
            row = (3 * g + 3) // 4 * 4
            pad = torch.zeros(nb, 1, H, BS, row, dtype=torch.uint8, device=dev)
            pad[..., :3 * g] = cw
            cw = pad.view(nb, 1, H, BS * row)
        out.append(cw.contiguous())
    return out


def h84_caches(dev, gen, nb):
    out = []
    for side in range(2):
        x = torch.randint(0, 16, (nb * H * BS * D,), generator=gen, dtype=torch.uint8).to(dev)
        c = ops.hamming84_encode(x)
        ops.inject_into(c, c, 1e-3, 8, seed=42 + side)
        out.append(c.view(nb, 1, H, BS * D))
    return out


def main():
    dev = torch.device("cuda:0")
    libs = sys.argv[1:] or [_lib.LIB_PATH]
    handles = []
    for p in libs:
        h = ctypes.CDLL(os.path.abspath(p))
        fn = h.kvecc_shim_read_batch
        fn.argtypes = _lib.SIGNATURES["kvecc_shim_read_batch"]
        fn.restype = ctypes.c_int
        tn = h.kvecc_time_next_launch
        tn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        handles.append((os.path.basename(p), fn, tn))
    nlb = L // BS
    nb = B * nlb
    gen = torch.Generator().manual_seed(7)
    table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
    scales = [(torch.rand(nb, 1, H, BS, generator=gen) * 0.1 + 0.01).to(dev) for _ in range(2)]
    stream = torch.cuda.current_stream(dev).cuda_stream
    summary = {}
    for case in CASES:
        codec, interp = case.split("+")[0], case.endswith("+interp")
        if codec.startswith("golay"):
            caches = golay_caches(dev, codec == "golay_packed", gen, nb)
            g = (D + 2) // 3
            per = ((3 * g + 3) // 4 * 4) if codec == "golay_packed" else g
            inb = 3 * g if codec == "golay_packed" else 4 * g
        else:
            caches = h84_caches(dev, gen, nb)
            per, inb = D, D
        bs = caches[0].shape[-1] // per
        cid = ops.SHIM_CODECS[codec]
        # one output pair for every library: where the outputs sit in HBM
        # relative to the caches moved a library's time by up to 6 %
        shared = (torch.empty(B, H, L, D, dtype=ODT, device=dev), torch.empty(B, H, L, D, dtype=ODT, device=dev))
        outs = [shared for _ in handles]
        stats = [ops.new_stats(dev) for _ in handles]

        def call(i, ev=None):
            name, fn, tn = handles[i]
            if ev is not None:
                tn(ctypes.c_void_p(ev[0].cuda_event), ctypes.c_void_p(ev[1].cuda_event))
            rc = fn(caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
                    table.data_ptr(), table.shape[1], B, L, H, D, 1, bs, 0, cid, int(interp),
                    outs[i][0].data_ptr(), outs[i][1].data_ptr(), ops._DT[ODT], stats[i].data_ptr(), stream)
            assert rc == 0, (name, rc)

        for i in range(len(handles)):
            call(i)
        for s in stats:
            s.zero_()
        ok, ref = [], None
        for i in range(len(handles)):
            shared[0].fill_(float("nan"))
            shared[1].fill_(float("nan"))
            call(i)
            torch.cuda.synchronize()
            if ref is None:
                ref = (shared[0].clone(), shared[1].clone())
            ok.append(torch.equal(shared[0], ref[0]) and torch.equal(shared[1], ref[1])
                      and ops.read_stats(stats[i]) == ops.read_stats(stats[0]))
        del ref
        # WARMUP back-to-back calls each right before the timed rounds: after any
        # idle the clocks take ~40 launches (~6 ms) to settle for the full-grid
        # H(8,4) reads (tools/exp/run_sustained.py, profiles/r04/fused/sustained.log)
        for i in range(len(handles)):
            for _ in range(int(os.environ.get("WARMUP", "100"))):
                call(i)
        times = [[] for _ in handles]
        blk = int(os.environ.get("BLOCK", "1"))  # consecutive launches of one library before the next
        for r in range(0, ROUNDS, blk):
            for i in range(len(handles)):
                for _ in range(blk):
                    ev = ops.kernel_timer(dev)
                    call(i, ev)
                    times[i].append(ev)
        torch.cuda.synchronize()
        nbytes = 2 * B * L * H * (inb + 4 + ODT.itemsize * D)
        for i, (name, _, _) in enumerate(handles):
            us = [a.elapsed_time(b) * 1e3 for a, b in times[i]]
            med = statistics.median(us)
            summary.setdefault(name, {})[case] = med
            print(f"{case:17s} {name:24s} median {med:6.1f} us  min {min(us):6.1f}  "
                  f"{nbytes / med / 1e3:5.0f} GB/s  {nbytes / med / 1e3 / 80:5.1f}%  same={ok[i]}", flush=True)
        del caches, outs
    print("summary (median us):")
    for name, row in summary.items():
        print(f"  {name:24s} " + "  ".join(f"{c}={v:.1f}" for c, v in row.items()))


if __name__ == "__main__":
    main()
