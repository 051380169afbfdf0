import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIXTURES = os.path.join(ROOT, "tests", "fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm MI355X device (runs on the GPU box)")
    config.addinivalue_line("markers", "dist: multi-process torch.distributed test")
    config.addinivalue_line("markers", "slow: slow test")


@pytest.fixture(scope="session")
def fixtures_dir():
    return FIXTURES


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)
