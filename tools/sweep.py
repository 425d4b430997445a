"""Launcher for the sharded Monte-Carlo sweep (kvecc.montecarlo).

    python tools/sweep.py --gpus 8 --output sweep.jsonl      # spawns its 8 ranks

or under torchrun (WORLD_SIZE set, nothing spawned):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29501 tools/sweep.py --output sweep.jsonl
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "quantized-kv-cache-ecc-protection_amd"))

from kvecc.montecarlo import main  # noqa: E402

if __name__ == "__main__":
    main()
