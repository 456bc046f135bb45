import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


def pytest_collection_modifyitems(config, items):
    # torch ships its own HIP runtime; once the engine's (/opt/rocm) has initialised the device in
    # this process, torch.cuda.is_available() came back False on the MI355X box (a run that began
    # with tests/test_gpu_half.py). So when GPU tests are selected, torch initialises first.
    if any(item.get_closest_marker("gpu") for item in items):
        import torch
        torch.cuda.is_available()


def load_p256_vectors():
    """Golden P-256 vectors: (fields (n,160) uint8, expected (n,), category (n,), names)."""
    import json
    raw = np.fromfile(os.path.join(GOLDEN, "p256_vectors.bin"), dtype=np.uint8).reshape(-1, 162)
    cats = json.load(open(os.path.join(GOLDEN, "p256_categories.json")))["categories"]
    return raw[:, :160].copy(), raw[:, 160].copy(), raw[:, 161].copy(), cats


def split_fields(f):
    return f[:, 0:32], f[:, 32:64], f[:, 64:96], f[:, 96:128], f[:, 128:160]


@pytest.fixture(scope="session")
def p256_vectors():
    return load_p256_vectors()


@pytest.fixture(scope="session")
def gpu():
    """The product path. Fails (does not skip) if the HIP library or GPU is missing."""
    import torch
    from smartbft_amd import GpuVerifier
    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X"
    v = GpuVerifier()
    yield v
    v.close()
