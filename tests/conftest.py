import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def _torch_first():
    """Initialise torch's HIP runtime before the engine's: tests that move
    tensors to the GPU then find the device whatever test ran first."""
    import torch

    if torch.cuda.is_available():
        torch.cuda.set_device(0)
        torch.zeros(1, device="cuda")


@pytest.fixture(scope="session")
def engine():
    from handel_amd.engine import Engine
    _torch_first()
    e = Engine(device=0, flavor="go")
    yield e
    e.close()


@pytest.fixture(scope="session")
def engine_cf():
    from handel_amd.engine import Engine
    _torch_first()
    e = Engine(device=0, flavor="cf")
    yield e
    e.close()
