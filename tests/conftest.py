import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


_SHM_TMP = None


def _shm_tmp():
    """Test data dirs on /dev/shm when it exists: the tests' many small
    files, fsyncs and sqlite commits cost ~30 ms each on an overlay /tmp.
    Stale dirs of dead test processes are removed first."""
    import shutil
    import tempfile
    base = "/dev/shm"
    if os.environ.get("PILOSA_TEST_TMP") == "keep" or not os.path.isdir(base) or not os.access(base, os.W_OK):
        return None
    for name in os.listdir(base):
        if name.startswith("pilosa_amd_tests_"):
            try:
                pid = int(name.rsplit("_", 1)[1])
                os.kill(pid, 0)
            except (ValueError, ProcessLookupError):
                shutil.rmtree(os.path.join(base, name), ignore_errors=True)
            except PermissionError:
                pass
    d = os.path.join(base, f"pilosa_amd_tests_{os.getpid()}")
    os.makedirs(d, exist_ok=True)
    tempfile.tempdir = d
    os.environ["TMPDIR"] = d
    return d


def pytest_configure(config):
    global _SHM_TMP
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    _SHM_TMP = _shm_tmp()
    # servers opened by tests do not freeze the collector (utils/gctune.py)
    os.environ.setdefault("PILOSA_GC_FREEZE", "0")


def pytest_unconfigure(config):
    if _SHM_TMP:
        import shutil
        shutil.rmtree(_SHM_TMP, ignore_errors=True)


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
