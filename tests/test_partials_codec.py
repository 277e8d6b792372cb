"""Typed int64 encoding of per-rank partial results (parallel/collectives.py
encode_partial / decode_partial): what the intra-node mesh all-gathers as
tensors instead of msgpack byte blobs."""
import numpy as np

from pilosa_amd.executor import FieldRow, GroupCount, RowIdentifiers, ValCount
from pilosa_amd.models.cache import Pair
from pilosa_amd.models.row import Row
from pilosa_amd.parallel.collectives import (TAG_GROUPS, TAG_MSGPACK, TAG_PAIRS, TAG_ROW, TAG_ROWIDS,
                                             TAG_VALCOUNT, RemoteError, decode_partial, encode_partial)


def rt(x):
    w = encode_partial(x)
    assert w.dtype == np.int64 and w.ndim == 1
    return w, decode_partial(w)


def test_scalars_and_none():
    for v in (None, True, False, 0, -5, (1 << 63) - 1):
        assert rt(v)[1] == v
    w, v = rt(ValCount(-12, 7))
    assert w[0] == TAG_VALCOUNT and (v.val, v.count) == (-12, 7)
    _, p = rt(Pair((1 << 64) - 2, 9))
    assert (p.id, p.count) == ((1 << 64) - 2, 9)


def test_lists():
    pairs = [Pair(3, 10), Pair(1 << 40, 2), Pair(7, 1)]
    w, got = rt(pairs)
    assert w[0] == TAG_PAIRS and [(p.id, p.count) for p in got] == [(3, 10), (1 << 40, 2), (7, 1)]
    w, got = rt([5, 1 << 63, 9])
    assert w[0] == TAG_ROWIDS and got == [5, 1 << 63, 9]
    assert rt([])[1] == []
    w, got = rt(RowIdentifiers([4, 8]))
    assert isinstance(got, RowIdentifiers) and got.rows == [4, 8]


def test_groups_typed_and_keyed_fallback():
    g = [GroupCount([FieldRow("a", 1), FieldRow("b", 2)], 10), GroupCount([FieldRow("a", 3), FieldRow("b", 0)], 4)]
    w, got = rt(g)
    assert w[0] == TAG_GROUPS and got == g
    keyed = [GroupCount([FieldRow("a", 1, "k1")], 3)]
    w, got = rt(keyed)
    assert w[0] == TAG_MSGPACK and got == keyed


def test_row_segments_and_errors():
    cols = np.array([1, 5, (1 << 20) + 3, (7 << 20) + 65537], np.uint64)
    w, got = rt(Row(cols))
    assert w[0] == TAG_ROW and sorted(got.columns().tolist()) == sorted(cols.tolist())
    r = Row(cols)
    r.keys = ["x"]
    assert rt(r)[0][0] == TAG_MSGPACK
    w, got = rt(ValueError("boom"))
    assert w[0] == TAG_MSGPACK and isinstance(got, RemoteError) and "boom" in str(got)
    assert rt({"i": [1, 2]})[1] == {"i": [1, 2]}
