import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 device (run on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running (exhaustive) checks")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first():
    """torch carries its own HIP runtime beside /opt/rocm's (which
    libipt_hip.so links); when both are in one process torch's must
    initialise first, or it finds no GPU. Tests that put torch tensors
    next to an ipt context rely on this order (bench.py has it too)."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


@pytest.fixture(scope="session")
def oracle():
    import oracle_binding

    oracle_binding.build()
    return oracle_binding.load()


@pytest.fixture(scope="session")
def gpu_ctx():
    from ipt_amd import capi

    ctx = capi.Context(0)
    yield ctx
    ctx.close()
