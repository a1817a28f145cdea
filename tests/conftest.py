import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The session engines pin aggregate requests to the headline path (GT fold
# over 16-key windows, hg_set_aggregate_level) whatever their volume; the
# parity tests that matter at every level take the `agg_level` fixture (the
# G2 fold + two-pairing check that serves a message's first requests by
# default, and the GT path), and the volume policy itself is tested on
# contexts left at the policy (level -1).
AGG_LEVEL_DEFAULT = 2


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
    e.set_aggregate_level(AGG_LEVEL_DEFAULT)
    yield e
    e.close()


@pytest.fixture(scope="session")
def engine_cf():
    from handel_amd.engine import Engine
    _torch_first()
    e = Engine(device=0, flavor="cf")
    e.set_aggregate_level(AGG_LEVEL_DEFAULT)
    yield e
    e.close()


@pytest.fixture(params=[0, 2], ids=["g2fold", "gt16"])
def agg_level(request):
    """Runs an aggregate parity test at table level 0 (G2 point fold +
    two-pairing k_verify: a message's first 16384 requests by default) and at
    level 2 (GT fold over 16-key windows + k_verify_sig: the serving path); the
    session engines are pinned for the test and restored afterwards."""
    engines = [request.getfixturevalue(n) for n in ("engine", "engine_cf")]
    for e in engines:
        e.set_aggregate_level(request.param)
    yield request.param
    for e in engines:
        e.set_aggregate_level(AGG_LEVEL_DEFAULT)
