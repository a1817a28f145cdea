import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Aggregate requests in the GPU suite run on the headline path (GT fold over
# 16-key windows) whatever their volume; tests of the other table levels and
# of the volume policy run in child processes with their own HG_GT_LEVEL.
os.environ.setdefault("HG_GT_LEVEL", "2")


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
