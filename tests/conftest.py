import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "lab: kernel-lab case (dead / slower kernels); ALPHAGO_AMD_LAB_TESTS=1 runs it")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("ALPHAGO_AMD_LAB_TESTS", "0") == "1":
        return
    skip = pytest.mark.skip(reason="kernel-lab case: ALPHAGO_AMD_LAB_TESTS=1 runs it")
    for item in items:
        if item.get_closest_marker("lab") is not None:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def cuda_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
