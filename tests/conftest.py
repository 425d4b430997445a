"""Shared pytest configuration.

Markers: ``gpu`` = needs an MI355X (runs on the GPU box via gpurun).
The product package lives in ``quantized-kv-cache-ecc-protection_amd/`` (a
directory name that is not a Python identifier), so it is put on sys.path
here, as bench.py and __graft_entry__.py do.
"""

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct GPU (gfx950)")


@pytest.fixture(scope="session")
def golden():
    """Load a golden fixture by name -> dict of numpy arrays."""
    cache = {}

    def load(name):
        if name not in cache:
            with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
                cache[name] = {k: z[k] for k in z.files}
        return cache[name]

    return load


@pytest.fixture(scope="session")
def manifest():
    import json
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def gpu():
    """The HIP product backend on cuda:0 (skips when no GPU is visible)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import kvecc
    kvecc.require_hip()
    return torch.device("cuda:0")
