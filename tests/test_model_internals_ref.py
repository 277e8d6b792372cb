"""Ported expectations of small reference unit tests: iterator_internal_test.go
(slice / buffered iterators), cache_test.go (rank cache size after
Recalculate), pilosa_internal_test.go (validateName), view_internal_test.go
(fragment delete / concurrent create), server_internal_test.go (open-file
count, anti-entropy with a zero interval)."""
import os
import tempfile
import threading
import time

import pytest

from pilosa_amd.errors import PilosaError, validate_name
from pilosa_amd.models.cache import RankCache
from pilosa_amd.models.iterator import BufIterator, LimitIterator, RoaringIterator, SliceIterator


# ---------------------------------------------------------------- iterator_internal_test.go
def _all(itr):
    out = []
    while True:
        r, c, eof = itr.next()
        if eof:
            return out
        out.append((r, c))


def test_slice_iterator():  # TestSliceIterator
    itr = SliceIterator([0, 0, 2, 4], [0, 1, 0, 10])
    assert _all(itr) == [(0, 0), (0, 1), (2, 0), (4, 10)]


def test_buf_iterator_seek_and_unread():  # TestBufIterator
    itr = BufIterator(SliceIterator([0, 0, 1, 2], [1, 3, 0, 100]))
    itr.seek(0, 2)
    assert itr.next() == (0, 3, False)
    assert itr.next() == (1, 0, False)
    itr.unread()
    assert itr.next() == (1, 0, False)
    assert itr.next() == (2, 100, False)
    assert itr.next()[2] is True


def test_buf_iterator_double_fill():  # TestBufIterator_DoubleFillPanic
    itr = BufIterator(SliceIterator(None, None))
    itr.unread()
    with pytest.raises(PilosaError, match="^pilosa.BufIterator: buffer full$"):
        itr.unread()


def test_slice_iterator_length_mismatch():
    with pytest.raises(PilosaError, match="pair length mismatch: 2 != 1"):
        SliceIterator([1, 2], [1])


def test_limit_and_roaring_iterators():
    from pilosa_amd.shardwidth import SHARD_WIDTH as W
    pos = [0 * W + 5, 1 * W + 7, 1 * W + 9, 3 * W + 1]
    assert _all(RoaringIterator(pos)) == [(0, 5), (1, 7), (1, 9), (3, 1)]
    assert _all(LimitIterator(RoaringIterator(pos), 1, 8)) == [(0, 5), (1, 7)]
    it = RoaringIterator(pos)
    it.seek(1, 8)
    assert it.next() == (1, 9, False)


# ---------------------------------------------------------------- cache_test.go
def test_rank_cache_size_after_recalculate():  # TestCache_Rank
    c = RankCache(3)
    for i in range(1, 6):
        c.add(i, 3)
    c.recalculate()
    assert len(c) == 3


# ---------------------------------------------------------------- pilosa_internal_test.go
@pytest.mark.parametrize("name", ["a", "ab", "ab1", "b-c", "d_e", "exists", "a" * 64])
def test_validate_name(name):  # TestValidateName
    validate_name(name)


@pytest.mark.parametrize("name", ["", "'", "^", "/", "\\", "A", "*", "a:b", "valid?no", "yüce", "1", "_", "-",
                                  "a" * 64 + "1", "_exists"])
def test_validate_name_invalid(name):  # TestValidateNameInvalid
    with pytest.raises(PilosaError):
        validate_name(name)


# ---------------------------------------------------------------- view_internal_test.go
def _view():
    from pilosa_amd.models.view import View
    v = View(tempfile.mkdtemp(prefix="pilosa-view-"), "i", "f", "v")
    v.open()
    return v


def test_view_delete_fragment():  # TestView_DeleteFragment
    v = _view()
    try:
        f1 = v.create_fragment_if_not_exists(9)
        assert f1 is not None
        v.delete_fragment(9)
        assert v.fragment(9) is None
        f2 = v.create_fragment_if_not_exists(9)
        assert f2 is not f1
    finally:
        v.close()


def test_view_create_fragment_race():  # TestView_CreateFragmentRace
    v = _view()
    # a slow create-shard broadcast (the reference's delayBroadcaster)
    v.on_create_shard = lambda shard: time.sleep(0.01)
    got, errs = [], []

    def create():
        try:
            got.append(v.create_fragment_if_not_exists(0))
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    try:
        ts = [threading.Thread(target=create) for _ in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs and len(got) == 2 and got[0] is got[1]
    finally:
        v.close()


# ---------------------------------------------------------------- server_internal_test.go
def test_count_open_files():  # TestCountOpenFiles
    assert len(os.listdir("/proc/self/fd")) > 0


def test_anti_entropy_zero_interval_returns():  # TestMonitorAntiEntropyZero
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger
    s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger(), replica_n=2,
               anti_entropy_interval=0).open()
    try:
        assert not any(t.name == "anti-entropy" and t.is_alive() for t in threading.enumerate())
    finally:
        s.close()


def test_rank_cache_rerank_moves_the_mutation_epoch():
    """A re-rank with no write (explicit recalculate, or the 10 s throttle
    expiring on a read) changes top(): device rank-cache memos keyed on the
    mutation epoch must see it (GpuExecutor._rank_caches fast path)."""
    from pilosa_amd.models.fragment import mutation_epoch
    c = RankCache(2)
    for rid, n in ((1, 5), (2, 4), (3, 4)):
        c.bulk_add(rid, n)
    e0 = mutation_epoch()
    c.recalculate()
    assert mutation_epoch() > e0
    assert c.top() == [(1, 5), (2, 4)]   # tie at the cut: row id ascending
    e1 = mutation_epoch()
    c.invalidate()                       # inside the throttle window: no re-rank
    assert mutation_epoch() == e1
