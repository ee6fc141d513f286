import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def golden(name: str):
    return np.load(GOLDEN / f"{name}.npz", allow_pickle=False)


def unflat(vals, lens):
    out, s = [], 0
    for n in lens:
        out.append(vals[s:s + n])
        s += n
    return out


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
