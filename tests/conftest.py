import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the HIP device library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    # GPU tests run only when a GPU is visible; selecting them with -m gpu on a CPU-only host
    # fails loudly instead of skipping (the driver runs -m gpu on a real MI355X).
    import torch

    if torch.cuda.is_available():
        return
    expr = config.getoption("-m") or ""
    if "gpu" in expr and "not gpu" not in expr:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def small_mnist():
    from svm355.utils.data import synthetic_mnist

    tr = synthetic_mnist(1200, seed=7)
    te = synthetic_mnist(400, seed=7, offset=1200)
    return tr, te
