"""Child process of tests/test_montecarlo.py's multi-process GPU tests.

Started as a fresh interpreter (subprocess), so its first GPU call happens
after the process group exists.  Reads RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT from the environment (torchrun's contract), runs the config-5
sweep driver kvecc.montecarlo.run_sweep on a HipShard of cuda:0 under the
given backend, and rank 0 writes the reduced rows as JSON.

    python tests/mp_sweep_worker.py BACKEND OUT_JSON B L H D
"""

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd")]


def main():
    backend, out = sys.argv[1], sys.argv[2]
    shape = tuple(int(v) for v in sys.argv[3:7])
    import torch
    import torch.distributed as dist

    from kvecc import montecarlo as mc
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)  # every rank on the one GPU of the box
    if backend == "nccl":
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    cfg = mc.MonteCarloConfig(shape=shape, bers=(1e-3, 0.03), seeds=(42, 7))
    rows, _ = mc.run_sweep(cfg, mc.HipShard(cfg, rank, world, dev), dist, rank)
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"rows": rows, "backend": dist.get_backend(), "world": world}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
