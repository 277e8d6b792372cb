"""Device-fault failover and the paranoia cross-check,
exercised on CPU with stand-in GPU executors."""
import numpy as np
import pytest

from tests.helpers import SW, Env


class _FaultyGpu:
    """Every device call fails like a lost HIP device."""

    def __init__(self):
        self.calls = 0

    def count(self, index, child, shards):
        self.calls += 1
        raise RuntimeError("hipErrorLaunchFailure: unspecified launch failure")

    def try_count_batch(self, index, calls, shards):
        self.calls += 1
        raise RuntimeError("hipErrorLaunchFailure: unspecified launch failure")


class _WrongGpu:
    def count(self, index, child, shards):
        return 12345


@pytest.fixture
def env():
    e = Env()
    e.create_index("i")
    e.field("i", "f")
    rng = np.random.default_rng(2)
    f = e.holder.index("i").field("f")
    c = rng.choice(2 * SW, size=5000, replace=False).astype(np.uint64)
    f.import_bits(np.full(len(c), 1, np.uint64), c)
    yield e
    e.close()


def test_device_faults_fall_back_to_host_then_detach(env, monkeypatch):
    monkeypatch.setenv("PILOSA_COALESCE", "0")
    want = env.q1("i", "Count(Row(f=1))")
    gpu = _FaultyGpu()
    env.executor.gpu = gpu
    env.executor.coalesce = False
    import pilosa_amd.executor as ex
    for k in range(ex.GPU_FAULT_LIMIT):
        assert env.executor.gpu is gpu
        assert env.q1("i", "Count(Row(f=1))") == want
    assert env.executor.gpu is None and env.executor.gpu_faults == ex.GPU_FAULT_LIMIT
    assert env.q("i", "Count(Row(f=1)) Count(Row(f=2))") == [want, 0]


def test_batch_path_fault_falls_back(env):
    want = env.q("i", "Count(Row(f=1)) Count(Row(f=2))")
    env.executor.gpu = _FaultyGpu()
    env.executor.coalesce = False
    assert env.q("i", "Count(Row(f=1)) Count(Row(f=2))") == want
    assert env.executor.gpu_faults >= 1


def test_paranoia_catches_wrong_device_results(env):
    env.executor.gpu = _WrongGpu()
    env.executor.coalesce = False
    env.executor.paranoia = True
    with pytest.raises(AssertionError, match="paranoia"):
        env.q1("i", "Count(Row(f=1))")
    env.executor.paranoia = False
    assert env.q1("i", "Count(Row(f=1))") == 12345


def test_strict_mode_raises_device_faults(env):
    env.executor.gpu = _FaultyGpu()
    env.executor.coalesce = False
    env.executor.strict_gpu = True
    with pytest.raises(RuntimeError, match="hipErrorLaunchFailure"):
        env.q1("i", "Count(Row(f=1))")
    with pytest.raises(RuntimeError, match="hipErrorLaunchFailure"):
        env.q("i", "Count(Row(f=1)) Count(Row(f=2))")
