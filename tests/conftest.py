import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_runtime_first(request):
    """torch bundles its own HIP runtime; libmjgpu uses /opt/rocm's.  When libmjgpu's
    initialises first in a process, torch then finds no device ("No HIP GPUs are
    available", reproduced with both the r01 and r02 libraries), so a GPU session brings
    torch's up first (the order bench.py uses)."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
