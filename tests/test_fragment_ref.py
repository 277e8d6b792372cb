"""Expectations ported from the reference fragment tests
(/root/reference/fragment_internal_test.go), one test per reference function
(line ranges cited); run against models/fragment.py on the CPU."""
import io
import os
import random
import shutil
import tempfile

import numpy as np
import pytest

from pilosa_amd.models.cache import CACHE_TYPE_LRU, CACHE_TYPE_NONE, CACHE_TYPE_RANKED
from pilosa_amd.models.fragment import Fragment, TopOptions
from pilosa_amd.models.row import Row

from pilosa_amd.shardwidth import SHARD_WIDTH as SW  # noqa: E402


class _Frags:
    def __init__(self):
        self.dirs = []
        self.frags = []

    def open(self, shard=0, cache_type=CACHE_TYPE_RANKED, cache_size=50000, **kw):
        """mustOpenFragment (fragment_internal_test.go:1985-2010)."""
        d = tempfile.mkdtemp(prefix="frag_")
        self.dirs.append(d)
        f = Fragment(os.path.join(d, str(shard)), "i", "f", "standard", shard, cache_type=cache_type,
                     cache_size=cache_size, **kw)
        f.open()
        self.frags.append(f)
        return f

    def reopen(self, f):
        f.close()
        g = Fragment(f.path, f.index, f.field, f.view, f.shard, cache_type=f.cache_type, cache_size=f.cache_size,
                     max_opn=f.max_opn, mutex=f.mutex, bool_field=f.bool_field)
        g.open()
        self.frags.append(g)
        return g

    def close(self):
        for f in self.frags:
            try:
                f.close()
            except Exception:  # noqa: BLE001 - already closed
                pass
        for d in self.dirs:
            shutil.rmtree(d, ignore_errors=True)


@pytest.fixture
def frags():
    fs = _Frags()
    yield fs
    fs.close()


def cols(row):
    return [int(c) for c in row.columns()]


# ---------------------------------------------------------------- bits (:51-220)
def test_set_bit(frags):
    f = frags.open()
    f.set_bit(120, 1)
    f.set_bit(120, 6)
    f.set_bit(121, 0)
    assert f.row(120).count() == 2 and f.row(121).count() == 1
    f = frags.reopen(f)
    assert f.row(120).count() == 2 and f.row(121).count() == 1


def test_clear_bit(frags):
    f = frags.open()
    f.set_bit(1000, 1)
    f.set_bit(1000, 2)
    f.clear_bit(1000, 1)
    assert f.row(1000).count() == 1
    f = frags.reopen(f)
    assert f.row(1000).count() == 1


def test_rowcache_map(frags):
    """:109-145 -- a row read before snapshots keeps its bits while the
    fragment is rewritten underneath it."""
    f = frags.open()
    f.max_opn = 200
    for i in range(f.max_opn):
        f.set_bit(0, i * 32)
    f.snapshot()
    row = f.row(0)
    for j in range(5):
        for i in range(f.max_opn):
            f.set_bit(0, i * 32 + j + 1)
    assert all(row.includes(i * 32) for i in range(200))
    assert row.count() == 200


def test_clear_row(frags):
    if SW <= 1 << 16:
        pytest.skip("uses a second container per row (columns >= 65536 in shard 0)")
    f = frags.open()
    f.set_bit(1000, 1)
    f.set_bit(1000, 65536)
    f.clear_row(1000)
    assert f.row(1000).count() == 0
    f = frags.reopen(f)
    assert f.row(1000).count() == 0


def test_set_row(frags):
    if SW <= 1 << 16:
        pytest.skip("uses a second container per row (columns >= 65536 in shard 0)")
    f = frags.open(shard=7)
    f.set_bit(1000, 7 * SW + 1)
    f.set_bit(1000, 7 * SW + 65536)
    assert cols(f.row(1000)) == [7 * SW + 1, 7 * SW + 65536]
    assert f.set_row(Row([7 * SW + 1, 7 * SW + 65537, 7 * SW + 140000]), 1000) is True
    assert cols(f.row(1000)) == [7 * SW + 1, 7 * SW + 65537, 7 * SW + 140000]
    f = frags.reopen(f)
    assert f.row(1000).count() == 3


# ---------------------------------------------------------------- BSI (:222-900)
def test_set_value(frags):
    f = frags.open()
    assert f.set_value(100, 16, 3829) is True
    assert f.value(100, 16) == (3829, True)
    assert f.set_value(100, 16, 3829) is False
    f = frags.open()
    assert f.set_value(100, 16, 3829) is True
    assert f.set_value(100, 16, 2028) is True
    assert f.value(100, 16) == (2028, True)
    f = frags.open()
    f.set_value(100, 16, 3829)
    assert f.clear_value(100, 16, 2028) is True
    assert f.value(100, 16) == (0, False)
    f = frags.open()
    assert f.set_value(100, 10, 20) is True
    assert f.value(101, 11) == (0, False)
    # QuickCheck analogue: random depths / columns / values
    rng = random.Random(7)
    for _ in range(20):
        depth = rng.randint(1, 62)
        n = rng.randint(1, 99)
        f = frags.open()
        m = {}
        for _ in range(rng.randint(0, 30)):
            v = rng.getrandbits(depth)
            m[v % n] = v
            f.set_value(v % n, depth, v)
        for c, v in m.items():
            assert f.value(c, depth) == (v, True)


def _bsi(frags, vals):
    f = frags.open()
    for c, v in vals:
        f.set_value(c, 16, v)
    return f


def test_sum(frags):
    f = _bsi(frags, [(1000, 382), (2000, 300), (3000, 2818), (4000, 300)])
    assert f.sum(None, 16) == (3800, 4)
    assert f.sum(Row([2000, 4000, 5000]), 16) == (600, 2)
    f.clear_value(1000, 16, 23)
    assert f.sum(None, 16) == (3800 - 382, 3)


def test_min_max(frags):
    f = _bsi(frags, [(1000, 382), (2000, 300), (3000, 2818), (4000, 300), (5000, 2818), (6000, 2817), (7000, 0)])
    for filt, exp, cnt in ((None, 0, 1), ([2000, 4000, 5000], 300, 2), ([2000, 4000], 300, 2), ([1], 0, 0),
                           ([1000], 382, 1), ([7000], 0, 1)):
        assert f.min(Row(filt) if filt is not None else None, 16) == (exp, cnt), filt
    for filt, exp, cnt in ((None, 2818, 2), ([2000, 4000, 5000], 2818, 1), ([2000, 4000], 300, 2), ([1], 0, 0),
                           ([1000], 382, 1), ([7000], 0, 1)):
        assert f.max(Row(filt) if filt is not None else None, 16) == (exp, cnt), filt


def test_range(frags):
    f = _bsi(frags, [(1000, 382), (2000, 300), (3000, 2818), (4000, 300)])
    assert cols(f.range_op("==", 16, 300)) == [2000, 4000]
    assert cols(f.range_op("!=", 16, 300)) == [1000, 3000]
    vals = [(1000, 382), (2000, 300), (3000, 2817), (4000, 301), (5000, 1), (6000, 0)]
    f = _bsi(frags, vals)
    assert cols(f.range_op("<", 16, 301)) == [2000, 5000, 6000]
    assert cols(f.range_op("<", 16, 300)) == [5000, 6000]
    assert cols(f.range_op("<=", 16, 301)) == [2000, 4000, 5000, 6000]
    assert cols(f.range_op("<=", 16, 300)) == [2000, 5000, 6000]
    assert cols(f.range_op(">", 16, 300)) == [1000, 3000, 4000]
    assert cols(f.range_op(">", 16, 301)) == [1000, 3000]
    assert cols(f.range_op(">=", 16, 300)) == [1000, 2000, 3000, 4000]
    assert cols(f.range_op(">=", 16, 301)) == [1000, 3000, 4000]
    assert cols(f.range_between(16, 300, 2817)) == [1000, 2000, 3000, 4000]
    assert cols(f.range_between(16, 301, 2817)) == [1000, 3000, 4000]
    assert cols(f.range_between(16, 301, 2816)) == [1000, 4000]
    assert cols(f.range_between(16, 300, 2816)) == [1000, 2000, 4000]


# ---------------------------------------------------------------- snapshot / iteration (:901-957)
def test_snapshot(frags):
    f = frags.open()
    f.set_bit(1000, 1)
    f.set_bit(1000, 2)
    f.clear_bit(1000, 1)
    f.snapshot()
    assert f.row(1000).count() == 1
    f = frags.reopen(f)
    assert f.row(1000).count() == 1


def test_for_each_bit(frags):
    f = frags.open()
    f.set_bit(100, 20)
    f.set_bit(2, 38)
    f.set_bit(2, 37)
    assert list(f.for_each_bit()) == [(2, 37), (2, 38), (100, 20)]


# ---------------------------------------------------------------- TopN (:959-1196)
def _set_bits(f, row, *cs):
    for c in cs:
        f.set_bit(row, c)


def _pairs(ps):
    return [(p.id, p.count) for p in ps]


def _top3(frags, cache_type=CACHE_TYPE_RANKED):
    f = frags.open(cache_type=cache_type)
    _set_bits(f, 100, 1, 3, 200)
    _set_bits(f, 101, 1)
    _set_bits(f, 102, 1, 2)
    f.recalculate_cache()
    return f


def test_top(frags):
    f = _top3(frags)
    assert _pairs(f.top(TopOptions(n=2))) == [(100, 3), (102, 2)]


def test_top_filter(frags):
    from pilosa_amd.models.attrs import MemAttrStore
    f = _top3(frags)
    store = MemAttrStore()
    store.set_attrs(101, {"x": 10})
    store.set_attrs(102, {"x": 20})
    got = f.top(TopOptions(n=2, filter_name="x", filter_values=[10, 15, 20], attr_store=store))
    assert _pairs(got) == [(102, 2), (101, 1)]


def test_topn_intersect(frags):
    f = frags.open()
    _set_bits(f, 100, 1, 10, 11, 12)
    _set_bits(f, 101, 1, 2, 3, 4)
    _set_bits(f, 102, 1, 2, 4, 5, 6)
    _set_bits(f, 103, 1000, 1001, 1002)
    f.recalculate_cache()
    assert _pairs(f.top(TopOptions(n=3, src=Row([1, 2, 3])))) == [(101, 3), (102, 2), (100, 1)]


def test_topn_intersect_large(frags):
    """:1044-1094 -- rows 0..999, row i has columns 0..i-1, imported as one
    roaring bitmap."""
    from pilosa_amd import _roaring
    f = frags.open()
    i = np.arange(1000, dtype=np.uint64)
    rows = np.repeat(i, i.astype(np.int64))
    colsv = np.concatenate([np.arange(k, dtype=np.uint64) for k in range(1000)])
    bm = _roaring.Bitmap(np.sort(rows * np.uint64(SW) + colsv))
    f.import_roaring(bm.to_bytes())
    f.recalculate_cache()
    src = Row(list(range(980, 1000)))
    assert _pairs(f.top(TopOptions(n=10, src=src))) == [(999 - k, 19 - k) for k in range(10)]


def test_topn_ids(frags):
    f = frags.open()
    _set_bits(f, 100, 1, 2, 3)
    _set_bits(f, 101, 4, 5, 6, 7)
    _set_bits(f, 102, 8, 9, 10, 11, 12)
    assert _pairs(f.top(TopOptions(row_ids=[100, 101, 200]))) == [(101, 4), (100, 3)]


def test_topn_nop_cache(frags):
    f = frags.open(cache_type=CACHE_TYPE_NONE, cache_size=0)
    _set_bits(f, 100, 1, 2, 3)
    _set_bits(f, 101, 4, 5, 6, 7)
    _set_bits(f, 102, 8, 9, 10, 11, 12)
    assert f.top(TopOptions(row_ids=[100, 101, 200])) == []


def test_topn_cache_size(frags):
    f = frags.open(cache_size=3)
    _set_bits(f, 100, 1, 2, 3)
    _set_bits(f, 101, 4, 5, 6, 7)
    _set_bits(f, 102, 8, 9, 10, 11, 12)
    _set_bits(f, 103, 8, 9, 10, 11, 12, 13)
    _set_bits(f, 104, 8, 9, 10, 11, 12, 13, 14)
    _set_bits(f, 105, 10, 11)
    f.recalculate_cache()
    got = _pairs(f.top(TopOptions(n=5)))
    assert len(got) <= 3 and got == [(104, 7), (103, 6), (102, 5)]


# ---------------------------------------------------------------- blocks (:1198-1271)
def test_checksum(frags):
    from pilosa_amd.models.fragment import HASH_BLOCK_SIZE
    f = frags.open()
    orig = f.checksum()
    f.set_bit(1, 200)
    f.set_bit(HASH_BLOCK_SIZE * 2, 200)
    assert f.checksum() != orig


def test_blocks(frags):
    f = frags.open()
    f.set_bit(0, 0)
    prev = f.blocks()
    assert prev[0][1]
    f.set_bit(20, 0)
    blocks = f.blocks()
    assert blocks[0][1] != prev[0][1]
    prev = blocks
    f.set_bit(20, 100)
    assert f.blocks()[0][1] != prev[0][1]


def test_blocks_empty(frags):
    f = frags.open()
    f.set_bit(100, 1)
    blocks = f.blocks()
    assert len(blocks) == 1 and blocks[0][0] == 1


# ---------------------------------------------------------------- cache persistence (:1273-1356)
def test_lru_cache_persistence(frags):
    from pilosa_amd.models.cache import LRUCache
    f = frags.open(cache_type=CACHE_TYPE_LRU)
    for i in range(1000):
        f.set_bit(i, 0)
    assert isinstance(f.cache, LRUCache) and len(f.cache) == 1000
    f = frags.reopen(f)
    assert isinstance(f.cache, LRUCache) and len(f.cache) == 1000


def test_rank_cache_persistence():
    """:1305-1356 -- through Index -> Field -> View like the reference."""
    from pilosa_amd.models.cache import RankCache
    from tests.helpers import Env
    env = Env()
    try:
        env.create_index("i")
        env.field("i", "f", type="set", cache_type="ranked", cache_size=50000)
        f = env.holder.field("i", "f")
        for i in range(1000):
            f.set_bit(i, 0)
        frag = env.holder.fragment("i", "f", "standard", 0)
        assert isinstance(frag.cache, RankCache) and len(frag.cache) == 1000
        env.reopen()
        frag = env.holder.fragment("i", "f", "standard", 0)
        assert isinstance(frag.cache, RankCache) and len(frag.cache) == 1000
    finally:
        env.close()


# ---------------------------------------------------------------- tar (:1358-1410)
def test_write_to_read_from(frags):
    f0 = frags.open()
    f0.set_bit(1000, 1)
    f0.set_bit(1000, 2)
    f0.clear_bit(1000, 1)
    assert len(f0.cache) == 1
    buf = io.BytesIO()
    f0.write_to(buf)
    wn = buf.tell()
    buf.seek(0)
    f1 = frags.open()
    f1.read_from(buf)
    assert buf.tell() == wn
    assert len(f1.cache) == 1
    assert cols(f1.row(1000)) == [2]
    f1 = frags.reopen(f1)
    assert len(f1.cache) == 1 and cols(f1.row(1000)) == [2]


# ---------------------------------------------------------------- Tanimoto (:1463-1509)
def _tani(frags):
    f = frags.open()
    _set_bits(f, 100, 1, 3, 2, 200)
    _set_bits(f, 101, 1, 3)
    _set_bits(f, 102, 1, 2, 10, 12)
    f.recalculate_cache()
    return f


def test_tanimoto(frags):
    f = _tani(frags)
    assert _pairs(f.top(TopOptions(tanimoto_threshold=50, src=Row([1, 2, 3])))) == [(100, 3), (101, 2)]


def test_zero_tanimoto(frags):
    f = _tani(frags)
    assert _pairs(f.top(TopOptions(tanimoto_threshold=0, src=Row([1, 2, 3])))) == [(100, 3), (101, 2), (102, 2)]


def test_snapshot_run(frags):
    f = frags.open()
    for i in range(1, 3):
        f.set_bit(1000, i)
    f.snapshot()
    assert f.row(1000).count() == 2
    f = frags.reopen(f)
    assert f.row(1000).count() == 2


# ---------------------------------------------------------------- mutex / imports (:1538-2000)
def test_set_mutex(frags):
    f = frags.open(mutex=True)
    f.set_bit(1, 100)
    assert cols(f.row(1)) == [100]
    f.set_bit(2, 100)
    assert cols(f.row(1)) == [] and cols(f.row(2)) == [100]


IMPORT_CASES = {
    # (set rows, set cols, set expectation, clear rows, clear cols, clear expectation) per kind
    "set": [
        ([1, 1, 1, 1], [0, 1, 2, 3], {1: [0, 1, 2, 3]}, [], [], {1: [0, 1, 2, 3]}),
        ([1, 1, 1, 1, 2, 2, 2, 2], [0, 1, 2, 3, 0, 1, 2, 3], {1: [0, 1, 2, 3], 2: [0, 1, 2, 3]},
         [1, 1, 2], [1, 2, 3], {1: [0, 3], 2: [0, 1, 2]}),
        ([1, 1, 1, 1, 2], [0, 1, 2, 3, 1], {1: [0, 1, 2, 3], 2: [1]}, [1, 1, 1, 1], [0, 1, 2, 3], {1: [], 2: [1]}),
        ([1, 1, 1, 1, 2, 2, 1], [0, 1, 2, 3, 1, 8, 1], {1: [0, 1, 2, 3], 2: [1, 8]}, [1, 1], [0, 0],
         {1: [1, 2, 3], 2: [1, 8]}),
        ([1, 2, 3], [8, 8, 8], {1: [8], 2: [8], 3: [8]}, [1, 2, 3], [9, 9, 9], {1: [8], 2: [8], 3: [8]}),
    ],
    "mutex": [
        ([1, 1, 1, 1], [0, 1, 2, 3], {1: [0, 1, 2, 3]}, [], [], {1: [0, 1, 2, 3]}),
        ([1, 1, 1, 1, 2, 2, 2, 2], [0, 1, 2, 3, 0, 1, 2, 3], {1: [], 2: [0, 1, 2, 3]}, [1, 1, 2], [1, 2, 3],
         {1: [], 2: [0, 1, 2]}),
        ([1, 1, 1, 1, 2], [0, 1, 2, 3, 1], {1: [0, 2, 3], 2: [1]}, [1, 1, 1, 1], [0, 1, 2, 3], {1: [], 2: [1]}),
        ([1, 1, 1, 1, 2, 2, 1], [0, 1, 2, 3, 1, 8, 1], {1: [0, 1, 2, 3], 2: [8]}, [1, 1], [0, 0],
         {1: [1, 2, 3], 2: [8]}),
        ([1, 2, 3], [8, 8, 8], {1: [], 2: [], 3: [8]}, [1, 2, 3], [9, 9, 9], {1: [], 2: [], 3: [8]}),
    ],
    "bool": [
        ([1, 1, 1, 1], [0, 1, 2, 3], {1: [0, 1, 2, 3]}, [], [], {1: [0, 1, 2, 3]}),
        ([0, 0, 0, 0, 1, 1, 1, 1], [0, 1, 2, 3, 0, 1, 2, 3], {0: [], 1: [0, 1, 2, 3]}, [1, 1, 2], [1, 2, 3],
         {0: [], 1: [0, 3], 2: []}),
        ([0, 0, 0, 0, 1], [0, 1, 2, 3, 1], {0: [0, 2, 3], 1: [1]}, [1, 1, 1, 1], [0, 1, 2, 3],
         {0: [0, 2, 3], 1: []}),
        ([1, 1, 1, 1, 0, 0, 1], [0, 1, 2, 3, 1, 8, 1], {0: [8], 1: [0, 1, 2, 3]}, [1, 1], [0, 0],
         {0: [8], 1: [1, 2, 3]}),
        ([0, 1, 2], [8, 8, 8], {0: [], 1: [], 2: [8]}, [1, 2, 3], [9, 9, 9], {0: [], 1: [], 2: [8]}),
    ],
}


@pytest.mark.parametrize("kind", ["set", "mutex", "bool"])
def test_import(frags, kind):
    """:1570-1700 (ImportSet), :1703-1819 (ImportMutex), :1821-1940 (ImportBool)."""
    for i, (sr, sc, sexp, cr, cc, cexp) in enumerate(IMPORT_CASES[kind]):
        f = frags.open(mutex=kind == "mutex", bool_field=kind == "bool")
        f.bulk_import(sr, sc)
        for k, v in sexp.items():
            assert cols(f.row(k)) == v, (kind, i, "set", k)
        f.bulk_import(cr, cc, clear=True)
        for k, v in cexp.items():
            assert cols(f.row(k)) == v, (kind, i, "clear", k)


def test_concurrent_import(frags):
    """:1687-1700"""
    import threading
    f = frags.open()
    errs = []

    def imp(r, c):
        try:
            f.bulk_import(r, c)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=imp, args=([1, 2], [1, 2])), threading.Thread(target=imp, args=([3, 4], [3, 4]))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs
    assert [cols(f.row(r)) for r in (1, 2, 3, 4)] == [[1], [2], [3], [4]]


# ---------------------------------------------------------------- rows / roaring import (:2634-2915)
def test_rows_iteration(frags):
    if SW <= 1 << 16:
        pytest.skip("uses a second container per row (columns >= 65536 in shard 0)")
    f = frags.open()
    for i in range(100, 200):
        f.set_bit(i, i % 2)
    assert f.rows(0) == list(range(100, 200))
    assert f.rows(0, column=1) == [i for i in range(100, 200) if i % 2]
    f = frags.open()
    f.set_bit(1, 66000)
    f.set_bit(2, 66000)
    f.set_bit(2, 166000)
    assert f.rows(0) == [1, 2] and f.rows(0, column=66000) == [1, 2]
    f = frags.open()
    expected = []
    for r in range(1, 10000, 100):
        expected.append(r)
        for c in range(1, SW - 1, 10000 * 7):  # the reference's grid, every 7th column step
            f.set_bit(r, c)
            assert f.rows(0, column=c) == expected
        assert f.rows(0) == expected


def _calc_expected(*inputs):
    rows = {}
    for inp in inputs:
        for v in inp:
            rows.setdefault(v // SW, set()).add(v % SW)
    return {r: sorted(c) for r, c in rows.items()}


def test_roaring_import(frags):
    from pilosa_amd import _roaring
    cases = [[[0], [1]],
             [[0, 65535, 65536, 65537, 65538, 65539, 130000], [1000, 67000, 130000]],
             [[0, 65535, 65536, 65537, 65538, 65539, 130000], [0, 65535, 65536, 65537, 65538, 65539, 130000]],
             [[0, 65535, 65536, SW + 1, SW * 2 + 1], [1, SW + 2, SW * 2 + 2]]]
    for case in cases:
        f = frags.open()
        for num, inp in enumerate(case):
            f.import_roaring(_roaring.Bitmap(np.array(sorted(inp), dtype=np.uint64)).to_bytes())
            for row, want in _calc_expected(*case[:num + 1]).items():
                assert cols(f.row(row)) == want


def _calc_top(rows, colsv):
    d = {}
    for r, c in zip(rows, colsv):
        d.setdefault(r, set()).add(c)
    return sorted(((r, len(c)) for r, c in d.items()), key=lambda p: -p[1])


def test_roaring_import_topn(frags):
    from pilosa_amd import _roaring
    f = frags.open()
    rows, cs = [4, 4, 4, 4], [0, 1, 2, 3]
    f.bulk_import(rows, cs)
    assert _pairs(f.top(TopOptions())) == _calc_top(rows, cs)
    r2, c2 = [5, 5, 5, 5, 5], [0, 1, 2, 3, 4]
    f.bulk_import(r2, c2)
    rows, cs = rows + r2, cs + c2
    assert _pairs(f.top(TopOptions())) == _calc_top(rows, cs)
    bits = [0, 65535, 65536, SW + 1, SW + 2, SW * 2 + 1]
    f.import_roaring(_roaring.Bitmap(np.array(bits, dtype=np.uint64)).to_bytes())
    assert _pairs(f.top(TopOptions())) == _calc_top(rows + [b // SW for b in bits], cs + [b % SW for b in bits])


def test_fragment_row_iterator(frags):
    """:2915-3031"""
    for wrap in (False, True):
        for ids in ([0, 1, 2, 3], [1, 3, 5, 7]):
            f = frags.open()
            for r in ids:
                f.set_bit(r, 0)
            it = f.row_iterator(wrap)
            for k in range(len(ids) + (1 if wrap else 0)):
                row, rid, wrapped = it.next()
                assert rid == ids[k % len(ids)]
                assert wrapped == (k >= len(ids))
                assert cols(row) == [0]
            if not wrap:
                row, rid, wrapped = it.next()
                assert row is None and rid == 0 and wrapped


def test_union_in_place_mapped(frags):
    """:3033-3097 -- a bitmap written into the fragment, then unioned in
    place with another: the count is between the larger input and the sum."""
    from pilosa_amd import _roaring
    rng0, rng1 = np.random.default_rng(2), np.random.default_rng(1)
    d0 = np.unique(rng0.integers(0, 1 << 28, 1_000_000, dtype=np.uint64))
    d1 = np.unique(rng1.integers(0, 1 << 28, 1_000_000, dtype=np.uint64))
    f = frags.open(cache_type=CACHE_TYPE_NONE, cache_size=0)
    f.import_roaring(_roaring.Bitmap(d0).to_bytes())
    assert f.storage.count() == len(d0)
    f.import_roaring(_roaring.Bitmap(d1).to_bytes())
    n = f.storage.count()
    assert max(len(d0), len(d1)) <= n <= len(d0) + len(d1)
    assert n == len(np.union1d(d0, d1))
    f = frags.reopen(f)
    assert f.storage.count() == n


# ---------------------------------------------------------------- BSI positions / restart (:3099-3433)
def test_positions_for_value(frags):
    f = frags.open(cache_type=CACHE_TYPE_NONE, cache_size=0)
    for col, depth, val, to_set, to_clear in (
            (0, 1, 0, [0], [SW, SW * 2]),
            (0, 3, 0, [0], [SW, SW * 2, SW * 3, SW * 4]),
            (1, 3, 0, [1], [SW + 1, SW * 2 + 1, SW * 3 + 1, SW * 4 + 1]),
            (0, 1, 1, [0, SW * 2], [SW]),
            (0, 4, 10, [0, SW * 3, SW * 5], [SW, SW * 2, SW * 4]),
            (0, 5, 10, [0, SW * 3, SW * 5], [SW, SW * 2, SW * 4, SW * 6])):
        s, c = f._positions_for_values(np.array([col]), np.array([val]), depth, False)
        assert sorted(int(x) for x in s) == to_set and sorted(int(x) for x in c) == to_clear, (col, depth, val)


@pytest.mark.parametrize("max_opn", [0, 10000])
def test_import_clear_restart(frags, max_opn):
    """:3181-3290 -- import, reopen, reopen on a second fragment object,
    clear import, reopen: the rows are exactly as expected every time, and
    the op count survives restarts while it fits under max_opn."""
    cases = [([1], [1]), ([1, 2, 3, 4, 5, 6, 7, 8, 9, 1], [1, 2, 3, 4, 5, 6, 7, 8, 9, 500000]),
             ([0] * 10, [0, 65535, 65536, 131071, 131072, 196607, 196608, 262143, 262144, 1000000]),
             ([1, 2, 20, 200, 2000, 200000], [1] * 6)]
    for rows, cs in cases:
        cs = [c % SW for c in cs]   # shard 0 under any PILOSA_SHARD_WIDTH
        exp = {}
        for r, c in zip(rows, cs):
            exp.setdefault(r, set()).add(c)
        exp_opn = sum(len(v) for v in exp.values())

        def check(fr, want):
            for r, cset in want.items():
                assert set(cols(fr.row(r))) == cset, (r, max_opn)
        f = frags.open(max_opn=max_opn)
        f.bulk_import(rows, cs)
        if exp_opn <= max_opn:
            assert f.opn == exp_opn
        check(f, exp)
        f = frags.reopen(f)
        if exp_opn <= max_opn:
            assert f.opn == exp_opn
        check(f, exp)
        f2 = frags.reopen(f)
        check(f2, exp)
        f2.bulk_import(rows, cs, clear=True)
        cleared = {r: set() for r in exp}
        check(f2, cleared)
        f3 = frags.reopen(f2)
        check(f3, cleared)


def test_import_value_concurrent(frags):
    import threading
    f = frags.open()
    errs = []

    def work(i):
        rng = random.Random(i)
        try:
            for j in range(10):
                f.import_value([j], [rng.randrange(1000)], 10, clear=i % 2 == 0)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs


@pytest.mark.parametrize("max_opn", [0, 10000])
def test_import_multiple_values(frags, max_opn):
    """:3361-3406 -- the last value of a column in one import wins."""
    f = frags.open(max_opn=max_opn)
    f.import_value([0, 0], [97, 100], 7)
    assert f.value(0, 7) == (100, True)


def test_fragment_concurrent_read_write(frags):
    import threading
    f = frags.open()
    errs = []

    def writer():
        try:
            for i in range(1000):
                f.set_bit(i % 4, i)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    t = threading.Thread(target=writer)
    t.start()
    acc = 0
    for i in range(100):
        acc += f.row(i % 4).count()
    t.join()
    assert not errs
    assert sum(f.row(r).count() for r in range(4)) == 1000


# ---------------------------------------------------------------- anti-entropy merge (fragment.go:1873-1991)
def test_merge_block_majority_vote(frags):
    """mergeBlock: a pair is set when at least (n+1)/2 of the n block copies
    (local + replicas) have it; each copy's diff brings it to the consensus.
    (The reference appends a clear to its *sets* slice -- a bug at
    fragment.go:1969-1970; the cases below never mix sets and clears for
    one copy, so both agree.)"""
    f = frags.open()
    f.set_bit(1, 10)   # local + r1 -> stays
    f.set_bit(2, 20)   # local only -> cleared locally
    f.set_bit(150, 5)  # other block: untouched
    r1 = ([1, 3], [10, 30])          # has (1,10), (3,30)
    r2 = ([3, 4, 250], [30, 40, 1])  # (3,30) with r1 -> set everywhere; (250, 1) is outside block 0
    sets, clears = f.merge_block(0, [r1, r2])
    assert cols(f.row(1)) == [10] and cols(f.row(2)) == [] and cols(f.row(3)) == [30]
    assert cols(f.row(150)) == [5]
    assert [list(map(list, s)) for s in sets] == [[[], []], [[1], [10]]]
    assert [list(map(list, c)) for c in clears] == [[[], []], [[4], [40]]]
    # even split of 2 copies: set wins
    f = frags.open()
    f.set_bit(7, 70)
    sets, clears = f.merge_block(0, [([], [])])
    assert cols(f.row(7)) == [70]
    assert [list(map(list, s)) for s in sets] == [[[7], [70]]]
    with pytest.raises(Exception):
        f.merge_block(0, [([1, 2], [1])])


# ---------------------------------------------------------------- snapshot concurrency
def test_snapshot_does_not_stall_writers_and_keeps_their_ops(frags, monkeypatch):
    """The snapshot's write + fsync run outside the fragment lock; writes
    landing meanwhile go to the old op log and are carried onto the new file."""
    import threading
    import pilosa_amd.models.fragment as fm
    f = frags.open()
    for c in range(100):
        f.set_bit(1, c)
    entered, release = threading.Event(), threading.Event()
    real_fsync = os.fsync

    def slow_fsync(fd):
        if not entered.is_set():
            entered.set()
            assert release.wait(10)
        real_fsync(fd)
    monkeypatch.setattr(fm.os, "fsync", slow_fsync)
    t = threading.Thread(target=f.snapshot)
    t.start()
    assert entered.wait(10)
    done = threading.Event()

    def writer():   # must not block on the in-flight snapshot
        for c in range(100, 150):
            f.set_bit(2, c)
        f.clear_bit(1, 0)
        done.set()
    w = threading.Thread(target=writer)
    w.start()
    assert done.wait(5), "writer stalled behind the snapshot"
    release.set()
    t.join(10)
    w.join(5)
    assert f.opn >= 0
    g = frags.reopen(f)
    assert cols(g.row(1)) == list(range(1, 100)) and cols(g.row(2)) == list(range(100, 150))


def test_background_and_inline_snapshots_do_not_deadlock(frags, monkeypatch):
    """A queued snapshot in its write+fsync phase and a ClearRow (which
    snapshots while holding the fragment lock) must both finish; the newer
    inline snapshot wins and the background one discards its file."""
    import threading
    import pilosa_amd.models.fragment as fm
    f = frags.open()
    for c in range(50):
        f.set_bit(1, c)
        f.set_bit(2, c)
    entered, release = threading.Event(), threading.Event()
    real_fsync = os.fsync

    def slow_fsync(fd):
        if threading.current_thread().name == "bg-snap" and not entered.is_set():
            entered.set()
            assert release.wait(10)
        real_fsync(fd)
    monkeypatch.setattr(fm.os, "fsync", slow_fsync)
    bg = threading.Thread(target=f.snapshot, name="bg-snap")
    bg.start()
    assert entered.wait(10)
    done = threading.Event()
    t = threading.Thread(target=lambda: (f.clear_row(1), done.set()))
    t.start()
    assert done.wait(10), "ClearRow deadlocked against the background snapshot"
    release.set()
    bg.join(10)
    t.join(10)
    assert not bg.is_alive()
    g = frags.reopen(f)
    assert cols(g.row(1)) == [] and cols(g.row(2)) == list(range(50))
    assert not [n for n in os.listdir(os.path.dirname(f.path)) if n.endswith(".snapshotting")]


def test_view_open_drops_stale_snapshot_files(tmp_path):
    """Snapshot temp files of a process that died mid-snapshot are removed
    when the view opens; other files are kept (ADVICE r02 fragment.py:310)."""
    import os as _os

    from pilosa_amd.models.fragment import remove_stale_snapshots
    d = tmp_path / "fragments"
    d.mkdir()
    names = ["3", "3.cache", "3.99999999.12.snapshotting", "3.snapshotting",
             f"3.{_os.getpid()}.7.snapshotting", "notes.snapshotting"]
    for nm in names:
        (d / nm).write_bytes(b"x")
    assert remove_stale_snapshots(str(d), _os.listdir(d)) == 2
    assert sorted(_os.listdir(d)) == sorted(["3", "3.cache", f"3.{_os.getpid()}.7.snapshotting",
                                             "notes.snapshotting"])
