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


def test_width_is_validated_and_device_shards_mapped():
    code = ("from pilosa_amd import shardwidth as s; print(s.EXPONENT, s.SHARD_WIDTH, s.CONTAINERS_PER_ROW, "
            "s.device_supported(), s.DEVICE_SUBSHARDS, s.device_shards([0, 3])[-1], s.sub_of_key(16 * 64 + 33), "
            "s.host_key(s.device_key(5 * 64 + 33), 2))")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                         env=dict(os.environ, PILOSA_SHARD_WIDTH="22"), timeout=120)
    # 2^22 columns: 4 device sub-shards per shard; key 16*64+33 = row 16, container 33 -> sub 2, slot 1
    assert out.stdout.split() == ["22", str(1 << 22), "64", "True", "4", "15", "2", str(5 * 64 + 33)], out.stderr
    bad = subprocess.run([sys.executable, "-c", "import pilosa_amd.shardwidth"], cwd=ROOT, capture_output=True,
                         text=True, env=dict(os.environ, PILOSA_SHARD_WIDTH="40"), timeout=120)
    assert bad.returncode != 0 and "PILOSA_SHARD_WIDTH" in bad.stderr
    narrow = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                            env=dict(os.environ, PILOSA_SHARD_WIDTH="18"), timeout=120)
    assert narrow.stdout.split()[:5] == ["18", str(1 << 18), "4", "True", "1"]


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


_WIDE_ARENA_CODE = r"""
import os, tempfile
import numpy as np
from pilosa_amd import _roaring, shardwidth as sw
from pilosa_amd.ops.loader import load_view
from pilosa_amd.ops.device import DeviceView
M = sw.DEVICE_SUBSHARDS
rng = np.random.default_rng(5)
d = tempfile.mkdtemp()
paths, bms = [], []
for s in range(2):
    rows = rng.integers(0, 30, 40000).astype(np.uint64)
    cols = rng.integers(0, sw.SHARD_WIDTH, 40000).astype(np.uint64)
    bm = _roaring.Bitmap(rows * np.uint64(sw.SHARD_WIDTH) + cols)
    p = os.path.join(d, str(s))
    open(p, "wb").write(bm.to_bytes())
    paths.append(p)
    bms.append(bm)
mapped = _roaring.MappedBitmap(paths[1])
# sub-shard i of a shard = its columns [i * 2^20, (i + 1) * 2^20), row by row
for s, bm in enumerate(bms):
    for i in range(M):
        sub = bm.sub_shard(sw.KEY_SHIFT, i)
        want = _roaring.Bitmap()
        want.union_in_place([bm.offset_range(r << 20, r * sw.SHARD_WIDTH + (i << 20), r * sw.SHARD_WIDTH + ((i + 1) << 20))
                             for r in range(30)])
        assert sub.equals(want), (s, i)
        if s == 1:
            assert mapped.sub_shard(sw.KEY_SHIFT, i).equals(want)
dsh = sw.device_shards([0, 1])
v = load_view([p for p in paths for _ in range(M)], dsh, "cpu", patchable=False, subs=[i for _ in paths for i in range(M)])
w = DeviceView.from_bitmaps([bm.sub_shard(sw.KEY_SHIFT, i) for bm in bms for i in range(M)], "cpu", shards=dsh)
assert v.S == w.S == 2 * M and v.shards == dsh
assert np.array_equal(v.rows, w.rows)
for a, b in ((v.t_rowptr, w.t_rowptr), (v.t_shard_base, w.t_shard_base)):
    assert np.array_equal(a.numpy(), b.numpy())
m1, m2 = v.t_meta.numpy()[:int(v.t_shard_base[-1])], w.t_meta.numpy()[:int(w.t_shard_base[-1])]
assert np.array_equal(m1 & ((1 << 23) - 1), m2 & ((1 << 23) - 1))
assert np.array_equal(v.t_payload.numpy()[:v.payload_used], w.t_payload.numpy()[:w.payload_used])
print("ok", M, len(m1))
"""


@pytest.mark.parametrize("exp", [21, 22, 24])
def test_device_arena_sub_shards_at_wide_widths(exp):
    """Shards wider than 2^20 columns become 2^(e-20) device sub-shards: the
    native sub_shard split (Bitmap and MappedBitmap) equals the row-by-row
    column ranges, and the fragment-file loader reading one sub-shard of a
    file per arena shard builds the same arena as build_arena over the
    split bitmaps."""
    r = subprocess.run([sys.executable, "-c", _WIDE_ARENA_CODE], cwd=ROOT, capture_output=True, text=True,
                       env=dict(os.environ, PILOSA_SHARD_WIDTH=str(exp)), timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("exp", [16, 18, 20])
def test_device_arena_keys_at_narrow_widths(exp):
    """Device arenas at shard widths 2^16..2^20: the fragment-file loader
    (key_shift) and build_arena (containers per row) place every container in
    slot j = key % (ShardWidth/2^16) of its row, identically."""
    r = subprocess.run([sys.executable, "-c", _ARENA_CODE], cwd=ROOT, capture_output=True, text=True,
                       env=dict(os.environ, PILOSA_SHARD_WIDTH=str(exp)), timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]
