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
                             env=dict(os.environ, PILOSA_SHARD_WIDTH="22"), timeout=120)
    assert "refused" in refused.stdout, refused.stderr[-2000:]
    narrow = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                            env=dict(os.environ, PILOSA_SHARD_WIDTH="18"), timeout=120)
    assert narrow.stdout.split() == ["18", str(1 << 18), "4", "True"]


_ARENA_CODE = r"""
import os, tempfile
import numpy as np
from pilosa_amd import _roaring, shardwidth as sw
from pilosa_amd.ops.loader import load_view
from pilosa_amd.ops.device import DeviceView
rng = np.random.default_rng(3)
d = tempfile.mkdtemp()
paths, bms = [], []
for s in range(3):
    rows = rng.integers(0, 40, 20000).astype(np.uint64)
    cols = rng.integers(0, sw.SHARD_WIDTH, 20000).astype(np.uint64)
    bm = _roaring.Bitmap(rows * np.uint64(sw.SHARD_WIDTH) + cols)
    p = os.path.join(d, str(s))
    open(p, "wb").write(bm.to_bytes())
    paths.append(p)
    bms.append(bm)
v = load_view(paths, [0, 1, 2], "cpu", patchable=False)
w = DeviceView.from_bitmaps(bms, "cpu", shards=[0, 1, 2])
assert np.array_equal(v.rows, w.rows)
for a, b in ((v.t_rowptr, w.t_rowptr), (v.t_shard_base, w.t_shard_base)):
    assert np.array_equal(a.numpy(), b.numpy())
m1, m2 = v.t_meta.numpy()[:int(v.t_shard_base[-1])], w.t_meta.numpy()[:int(w.t_shard_base[-1])]
assert np.array_equal(m1 & ((1 << 23) - 1), m2 & ((1 << 23) - 1))
assert int((m1 & 15).max()) < sw.CONTAINERS_PER_ROW
k = np.arange(0, 200, dtype=np.uint64)
assert np.array_equal(sw.host_key(sw.device_key(k)), k)
print("ok", sw.CONTAINERS_PER_ROW, len(m1))
"""


@pytest.mark.parametrize("exp", [16, 18, 20])
def test_device_arena_keys_at_narrow_widths(exp):
    """Device arenas at shard widths 2^16..2^20: the fragment-file loader
    (key_shift) and build_arena (containers per row) place every container in
    slot j = key % (ShardWidth/2^16) of its row, identically."""
    r = subprocess.run([sys.executable, "-c", _ARENA_CODE], cwd=ROOT, capture_output=True, text=True,
                       env=dict(os.environ, PILOSA_SHARD_WIDTH=str(exp)), timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]
