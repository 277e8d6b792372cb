import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _gpu_strict(request, monkeypatch):
    """GPU tests run the executor in strict mode: a device fault raises
    instead of being answered from the host fragments, and no test may end
    with a recorded device fault (pilosa_amd/executor.py DEVICE_FAULTS)."""
    if "gpu" not in request.keywords:
        yield
        return
    from pilosa_amd import executor as ex
    monkeypatch.setenv("PILOSA_GPU_STRICT", "1")
    before = ex.DEVICE_FAULTS[0]
    yield
    assert ex.DEVICE_FAULTS[0] == before, "a device fault was answered from the host"
