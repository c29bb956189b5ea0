import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs through librs_hip.so")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test but torch.cuda.is_available() is False")
    from recommender_system_amd import _lib
    _lib.lib()  # fail loudly if the extension is missing
    return torch.device("cuda")
