"""Sustained back-to-back launches of the fused shim reads: per-launch kernel
time (dispatch-stamped events, created before the loop) over N consecutive
launches with nothing between them, for the product's Golay read (persistent
grid) and Hamming(8,4) plain / interpolating reads (full grids), same workload
as bench.py.  Then the same with a short idle gap (GAP_US of host sleep after
every launch's enqueue is not possible without a sync, so: a sync every K
launches).  Shows whether per-launch time drifts under sustained load.

usage: python tools/exp/run_sustained.py [N]
"""
import os
import statistics
import sys
import time

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import ops  # noqa: E402

B, L, H, D, BS = 8, 4096, 32, 128, 16


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    nlb = L // BS
    nb = B * nlb
    gen = torch.Generator().manual_seed(7)
    table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, nlb).to(dev)
    scales = [(torch.rand(nb, 1, H, BS, generator=gen) * 0.1 + 0.01).to(dev) for _ in range(2)]
    h84 = []
    for side in range(2):
        x = torch.randint(0, 16, (nb * H * BS * D,), generator=gen, dtype=torch.uint8).to(dev)
        c = ops.hamming84_encode(x)
        ops.inject_into(c, c, 1e-3, 8, seed=42 + side)
        h84.append(c.view(nb, 1, H, BS * D))
        del x
    g = (D + 2) // 3
    gol = []
    for side in range(2):
        x = torch.randint(0, 16, (nb, 1, H, BS, D), generator=gen, dtype=torch.uint8).to(dev)
        cw = ops.golay_encode_rows(x).view(-1)
        ops.inject_into(cw, cw, 1e-2, 24, seed=42 + side)
        gol.append(cw.view(nb, 1, H, BS * g))
        del x
    outs = (torch.empty(B, H, L, D, dtype=torch.float16, device=dev),
            torch.empty(B, H, L, D, dtype=torch.float16, device=dev))
    st = ops.new_stats(dev)
    runs = {
        "golay": lambda: ops.shim_read_batch(gol[0], gol[1], scales[0], scales[1], table, L, D, 0, "golay",
                                             torch.float16, stats=st, out=outs),
        "h84": lambda: ops.shim_read_batch(h84[0], h84[1], scales[0], scales[1], table, L, D, 0, "hamming84",
                                           torch.float16, stats=st, out=outs),
        "h84_interp": lambda: ops.shim_read_batch(h84[0], h84[1], scales[0], scales[1], table, L, D, 0,
                                                  "hamming84", torch.float16, stats=st, interp=True, out=outs),
    }
    for name, call in runs.items():
        for sync_every in (0, 4):
            for _ in range(20):
                call()
            torch.cuda.synchronize()
            time.sleep(0.2)  # idle: the clocks and power budget settle
            evs = [ops.kernel_timer(dev) for _ in range(n)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(n):
                ops.time_next_launch(*evs[k])
                call()
                if sync_every and (k + 1) % sync_every == 0:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            us = [a.elapsed_time(b) * 1e3 for a, b in evs]
            q = [statistics.mean(us[i:i + n // 10]) for i in range(0, n, n // 10)]
            print(f"{name:10s} sync_every={sync_every}: per-launch mean by tenths " +
                  " ".join(f"{x:5.0f}" for x in q) +
                  f" | min {min(us):.0f} max {max(us):.0f} | wall {wall / n * 1e6:.0f} us/launch", flush=True)


if __name__ == "__main__":
    main()
