"""The shard-width knob (reference shardwidth/*.go build tags): the host
data model, executor and fragment expectations hold at other widths.  Each
width runs in a fresh interpreter because, like the reference's build tag,
the width is fixed for the life of a process."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("exp", [16, 18, 22, 24])
def test_reference_expectations_at_other_widths(exp):
    env = dict(os.environ, PILOSA_SHARD_WIDTH=str(exp))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "tests/test_executor_ref.py", "tests/test_fragment_ref.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


def test_width_is_validated_and_gpu_refused():
    code = ("from pilosa_amd import shardwidth as s; print(s.EXPONENT, s.SHARD_WIDTH, s.CONTAINERS_PER_ROW, "
            "s.device_supported())")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                         env=dict(os.environ, PILOSA_SHARD_WIDTH="22"), timeout=120)
    assert out.stdout.split() == ["22", str(1 << 22), "64", "False"]
    bad = subprocess.run([sys.executable, "-c", "import pilosa_amd.shardwidth"], cwd=ROOT, capture_output=True,
                         text=True, env=dict(os.environ, PILOSA_SHARD_WIDTH="40"), timeout=120)
    assert bad.returncode != 0 and "PILOSA_SHARD_WIDTH" in bad.stderr
    refused = subprocess.run([sys.executable, "-c", "from pilosa_amd.ops.gpu_executor import GpuExecutor\n"
                              "try:\n    GpuExecutor(None, 'cpu')\nexcept NotImplementedError as e:\n    print('refused')"],
                             cwd=ROOT, capture_output=True, text=True,
                             env=dict(os.environ, PILOSA_SHARD_WIDTH="18"), timeout=120)
    assert "refused" in refused.stdout, refused.stderr[-2000:]
