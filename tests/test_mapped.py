"""MappedBitmap (native/mapped.cpp): the copy-on-write mmap view of a
fragment file a cold fragment serves host reads and single-bit writes from
(reference roaring/container_stash.go:262-346 frozen/mapped containers,
roaring.go:1616-1622, fragment.go:311-456).  Differential against the owned
Bitmap decoded from the same bytes, with op logs and every container type."""
import os
import tempfile

import numpy as np
import pytest

from pilosa_amd import _roaring
from pilosa_amd.models.fragment import OP_ADD, OP_ADD_BATCH, OP_ADD_ROARING, OP_REMOVE, OP_REMOVE_BATCH

SW = 1 << 20


def _random_bitmap(rng):
    vals = []
    for _ in range(rng.integers(1, 40)):
        base = int(rng.integers(0, 64)) * 65536
        kind = rng.integers(0, 3)
        if kind == 0:    # array
            vals.append(base + rng.choice(65536, size=int(rng.integers(1, 300)), replace=False))
        elif kind == 1:  # bitmap
            vals.append(base + rng.choice(65536, size=int(rng.integers(5000, 20000)), replace=False))
        else:            # runs
            s = int(rng.integers(0, 60000))
            vals.append(base + np.arange(s, s + int(rng.integers(1, 5000))))
    bm = _roaring.Bitmap(np.unique(np.concatenate(vals)).astype(np.uint64))
    bm.optimize()
    return bm


def _with_ops(rng, bm, path):
    data = bytearray(bm.to_bytes())
    ref = _roaring.Bitmap.from_bytes(bytes(data))
    for _ in range(int(rng.integers(0, 25))):
        t = int(rng.integers(0, 5))
        if t in (0, 1):
            v = int(rng.integers(0, 70 * 65536))
            data += _roaring.encode_op(OP_ADD if t == 0 else OP_REMOVE, v, np.zeros(0, np.uint64), b"", 0)
        elif t in (2, 3):
            vs = np.unique(rng.integers(0, 70 * 65536, size=int(rng.integers(1, 50)))).astype(np.uint64)
            data += _roaring.encode_op(OP_ADD_BATCH if t == 2 else OP_REMOVE_BATCH, len(vs), vs, b"", 0)
        else:
            blob = _roaring.Bitmap(np.unique(rng.integers(0, 70 * 65536, size=200)).astype(np.uint64))
            data += _roaring.encode_op(OP_ADD_ROARING, len(blob.to_bytes()), np.zeros(0, np.uint64),
                                       blob.to_bytes(), 200)
    with open(path, "wb") as fh:
        fh.write(bytes(data))
    return _roaring.Bitmap.from_bytes(bytes(data))


@pytest.mark.parametrize("seed", range(12))
def test_mapped_matches_decoded_bitmap(seed):
    rng = np.random.default_rng(seed)
    d = tempfile.mkdtemp()
    path = os.path.join(d, "0")
    want = _with_ops(rng, _random_bitmap(rng), path)
    m = _roaring.MappedBitmap(path)
    assert m.ops == want.ops and m.opn == want.opn
    for step in range(300):
        op = int(rng.integers(0, 6))
        v = int(rng.integers(0, 70 * 65536))
        if op == 0:
            assert m.add(v) == want.add(v)
        elif op == 1:
            assert m.remove(v) == want.remove(v)
        elif op == 2:
            assert m.contains(v) == want.contains(v)
        elif op == 3:
            a = int(rng.integers(0, 70 * 65536))
            b = a + int(rng.integers(0, 4 * 65536))
            assert m.count_range(a, b) == want.count_range(a, b), (a, b)
        elif op == 4:
            k = int(rng.integers(0, 70))
            got = m.offset_range(SW, k * 65536, (k + 3) * 65536)
            assert got.equals(want.offset_range(SW, k * 65536, (k + 3) * 65536))
        else:
            col = int(rng.integers(0, SW))
            assert m.rows_with_column(col, 16).tolist() == want.rows_with_column(col, 16).tolist()
    assert m.count() == want.count()
    assert m.any() == want.any()
    if want.any():
        assert m.max() == want.max()
    rows = np.arange(0, 6, dtype=np.uint64)
    assert m.count_rows(rows, 16).tolist() == want.count_rows(rows, 16).tolist()
    # only the containers written to were copied
    assert m.overlay_containers() if callable(m.overlay_containers) else m.overlay_containers <= 300 + 70


def test_mapped_rejects_corrupt_files():
    d = tempfile.mkdtemp()
    bm = _roaring.Bitmap(np.arange(0, 100000, 3, dtype=np.uint64))
    data = bm.to_bytes()
    for k, bad in enumerate([data[:6], data[:20], b"\x00" * 64, data[:len(data) - 7]]):
        p = os.path.join(d, str(k))
        with open(p, "wb") as fh:
            fh.write(bad)
        with pytest.raises(Exception):
            _roaring.MappedBitmap(p)
    p = os.path.join(d, "torn")
    with open(p, "wb") as fh:   # a torn op at the tail is an error, as Bitmap.from_bytes reports
        fh.write(data + _roaring.encode_op(OP_ADD, 5, np.zeros(0, np.uint64), b"", 0)[:9])
    with pytest.raises(Exception):
        _roaring.MappedBitmap(p)
    p = os.path.join(d, "empty")
    open(p, "wb").close()
    m = _roaring.MappedBitmap(p)
    assert not m.any() and m.count() == 0 and m.add(7) and m.contains(7)


@pytest.mark.parametrize("seed", range(8))
def test_mapped_bulk_ops_and_streamed_snapshot(seed):
    rng = np.random.default_rng(100 + seed)
    d = tempfile.mkdtemp()
    path = os.path.join(d, "0")
    want = _with_ops(rng, _random_bitmap(rng), path)
    m = _roaring.MappedBitmap(path)
    for _ in range(6):
        vals = np.unique(rng.integers(0, 70 * 65536, size=int(rng.integers(1, 5000)))).astype(np.uint64)
        k = int(rng.integers(0, 3))
        if k == 0:
            assert m.add_many(vals, True) == want.add_many(vals, True)
        elif k == 1:
            assert m.remove_many(vals) == want.remove_many(vals)
        else:
            blob = _roaring.Bitmap(vals).to_bytes()
            clear = bool(rng.integers(0, 2))
            got, gd = m.import_roaring(blob, clear, 16)
            exp, ed = want.import_roaring(blob, clear, 16)
            assert got == exp and {k_: v for k_, v in gd.items() if v} == {k_: v for k_, v in ed.items() if v}
    snap = os.path.join(d, "snap")
    n = m.write_snapshot(snap)
    data = open(snap, "rb").read()
    assert n == len(data)
    back = _roaring.Bitmap.from_bytes(data)
    assert back.equals(want) and back.flags == want.flags
    assert back.check() == ""
    m2 = _roaring.MappedBitmap(snap)
    assert m2.count() == want.count() and m2.overlay_containers == 0
