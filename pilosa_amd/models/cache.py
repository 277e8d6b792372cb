"""TopN count caches (reference: cache.go).

* ``RankCache`` – id -> count map with a sorted ``rankings`` list; new entries
  below the threshold (count of the first trimmed item) are ignored, rankings
  are recomputed at most every 10 s on ``invalidate`` (cache.go:235-243), and
  entries are trimmed once they exceed 1.1 x max (cache.go:245-281).
* ``LRUCache`` – bounded LRU of counts (cache.go:58-133).
* ``NopCache``.
* ``Pair``/``Pairs`` helpers incl. ``pairs_add`` (cache.go:356-375).

Ordering is (count desc, id asc) so results are deterministic (Go's sort.Sort
is unstable; the reference leaves tie order unspecified).
"""
from __future__ import annotations

import collections
import threading
import time
from typing import Dict, Iterable, List, Tuple

import numpy as np

THRESHOLD_FACTOR = 1.1
CACHE_TYPE_RANKED = "ranked"
CACHE_TYPE_LRU = "lru"
CACHE_TYPE_NONE = "none"
DEFAULT_CACHE_SIZE = 50000
INVALIDATE_INTERVAL_S = 10.0


class Pair:
    __slots__ = ("id", "key", "count")

    def __init__(self, id: int, count: int, key: str = ""):
        self.id = int(id)
        self.count = int(count)
        self.key = key

    def to_json(self):
        d = {"id": self.id, "count": self.count}
        if self.key:
            d["key"] = self.key
        return d

    def __eq__(self, other):
        return isinstance(other, Pair) and (self.id, self.count, self.key) == (other.id, other.count, other.key)

    def __repr__(self):
        return f"Pair({self.id}, {self.count}{', ' + repr(self.key) if self.key else ''})"


def pairs_from_arrays(ids, counts) -> List[Pair]:
    """``[Pair(id, count), ...]`` from parallel id / count sequences, built in
    bulk by the native core when it is loaded (pyroaring ``make_pairs``: the
    same objects, ~0.1 us each instead of ~0.5 us through ``__init__``; a
    16-call TopN request returns thousands of pairs)."""
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    fast = _make_pairs()
    if fast is not None:
        got = fast(Pair, ids, counts)
        if got is not None:
            return got
    return [Pair(i, c) for i, c in zip(ids.tolist(), counts.tolist())]


class PairArray:
    """A TopN result kept columnar: ``ids`` (uint64) and ``counts`` (int64)
    in result order.  It behaves like the ``[Pair, ...]`` list the reference
    returns (len, indexing, slicing, iteration, equality with a list of
    Pairs) but builds Pair objects only when someone iterates or indexes it:
    a 16-call cache-only TopN request returns ~3k pairs, and creating them
    was 40 % of its host time (profiles/r05_topn/).  The HTTP / protobuf /
    collective encoders read the arrays directly."""

    __slots__ = ("ids", "counts", "_items")

    def __init__(self, ids, counts):
        self.ids = np.ascontiguousarray(ids, dtype=np.uint64)
        self.counts = np.ascontiguousarray(counts, dtype=np.int64)
        if len(self.ids) != len(self.counts):
            raise ValueError("PairArray: ids and counts differ in length")
        self._items = None

    def to_list(self) -> List["Pair"]:
        if self._items is None:
            fast = _make_pairs()
            got = fast(Pair, self.ids, self.counts) if fast is not None else None
            if got is None:
                got = [Pair(i, c) for i, c in zip(self.ids.tolist(), self.counts.tolist())]
            self._items = got
        return self._items

    def __len__(self):
        return len(self.ids)

    def __bool__(self):
        return len(self.ids) > 0

    def __iter__(self):
        return iter(self.to_list())

    def __getitem__(self, i):
        if isinstance(i, slice):
            return PairArray(self.ids[i], self.counts[i])
        return self.to_list()[i]

    def __eq__(self, other):
        if isinstance(other, PairArray):
            return np.array_equal(self.ids, other.ids) and np.array_equal(self.counts, other.counts)
        if isinstance(other, (list, tuple)):
            return len(other) == len(self) and all(a == b for a, b in zip(self.to_list(), other))
        return NotImplemented

    def __repr__(self):
        return f"PairArray({self.to_list()!r})"

    def to_json(self):
        return [{"id": i, "count": c} for i, c in zip(self.ids.tolist(), self.counts.tolist())]

    def json_bytes(self) -> bytes:
        """The JSON array text (Go's layout), natively when the core is loaded."""
        try:
            from pilosa_amd import _roaring
            return _roaring.pairs_json(self.ids, self.counts)
        except (ImportError, AttributeError):
            import json
            return json.dumps(self.to_json(), separators=(",", ":")).encode()


def pair_array(ids, counts) -> "PairArray":
    """A final TopN result from parallel id / count arrays (see PairArray)."""
    return PairArray(ids, counts)


_new_pa = object.__new__


def pair_arrays_split(ids: np.ndarray, counts: np.ndarray, offs) -> List["PairArray"]:
    """PairArrays over consecutive slices ``offs[i]:offs[i+1]`` of contiguous
    uint64 ids and int64 counts (a native batch's answers): views, no
    conversion or per-result checks."""
    out = []
    for a, b in zip(offs, offs[1:]):
        p = _new_pa(PairArray)
        p.ids = ids[a:b]
        p.counts = counts[a:b]
        p._items = None
        out.append(p)
    return out


_MAKE_PAIRS = []


def _make_pairs():
    if not _MAKE_PAIRS:
        try:
            from pilosa_amd import _roaring
            _MAKE_PAIRS.append(getattr(_roaring, "make_pairs", None))
        except ImportError:
            _MAKE_PAIRS.append(None)
    return _MAKE_PAIRS[0]


def sort_pairs(pairs: List[Pair]) -> List[Pair]:
    return sorted(pairs, key=lambda p: (-p.count, p.id))


def pairs_add(a: Iterable[Pair], b: Iterable[Pair]) -> List[Pair]:
    m: Dict[int, int] = collections.OrderedDict()
    for p in a:
        m[p.id] = p.count
    for p in b:
        m[p.id] = m.get(p.id, 0) + p.count
    return [Pair(k, v) for k, v in m.items()]


class NopCache:
    version = 0

    def add(self, id, n):
        pass

    def bulk_add(self, id, n):
        pass

    def get(self, id):
        return 0

    def __len__(self):
        return 0

    def ids(self):
        return []

    def invalidate(self):
        pass

    def recalculate(self):
        pass

    def top(self) -> List[Tuple[int, int]]:
        return []


class LRUCache:
    def __init__(self, max_entries: int):
        self.max_entries = int(max_entries)
        self._d: "collections.OrderedDict[int, int]" = collections.OrderedDict()
        self._lock = threading.Lock()
        self.version = 0

    def add(self, id, n):
        with self._lock:
            self.version += 1
            self._d[id] = n
            self._d.move_to_end(id)
            while self.max_entries > 0 and len(self._d) > self.max_entries:
                self._d.popitem(last=False)

    bulk_add = add

    def get(self, id):
        with self._lock:
            n = self._d.get(id)
            if n is None:
                return 0
            self._d.move_to_end(id)
            return n

    def __len__(self):
        return len(self._d)

    def ids(self):
        return sorted(self._d)

    def invalidate(self):
        pass

    def recalculate(self):
        pass

    def top(self):
        return sorted(self._d.items(), key=lambda kv: (-kv[1], kv[0]))


class RankCache:
    def __init__(self, max_entries: int):
        self.max_entries = int(max_entries)
        self.threshold_buffer = int(THRESHOLD_FACTOR * self.max_entries)
        self.entries: Dict[int, int] = {}
        self._ranked = (np.zeros(0, np.uint64), np.zeros(0, np.int64))
        self._rankings: List[Tuple[int, int]] = []
        self.version = 0  # bumped whenever top() can change (device TopN index validity)
        self.threshold_value = 0
        self.update_time = 0.0
        self._lock = threading.Lock()

    def add(self, id, n):
        with self._lock:
            if n < self.threshold_value and n > 0:
                return
            self.entries[id] = n
            self._invalidate()

    def bulk_add(self, id, n):
        with self._lock:
            if n < self.threshold_value:
                return
            self.entries[id] = n

    def bulk_add_many(self, ids, counts):
        """bulk_add for arrays of (row id, count) at once (bulk imports,
        cache open): one dict update instead of a call per row."""
        ids = np.asarray(ids, dtype=np.uint64)
        counts = np.asarray(counts, dtype=np.int64)
        with self._lock:
            keep = counts >= self.threshold_value
            self.entries.update(zip(ids[keep].tolist(), counts[keep].tolist()))

    def get(self, id):
        with self._lock:
            return self.entries.get(id, 0)

    def __len__(self):
        return len(self.entries)

    def ids(self):
        with self._lock:
            return sorted(self.entries)

    def invalidate(self):
        with self._lock:
            self._invalidate()

    def recalculate(self):
        with self._lock:
            self._recalculate()

    def _invalidate(self):
        if time.monotonic() - self.update_time < INVALIDATE_INTERVAL_S:
            return
        self._recalculate()

    def _recalculate(self):
        # count desc, then id asc (cache.go:245-281), sorted with numpy
        n = len(self.entries)
        ids = np.fromiter(self.entries.keys(), dtype=np.uint64, count=n)
        cnt = np.fromiter(self.entries.values(), dtype=np.int64, count=n)
        order = np.lexsort((ids, -cnt))
        ids, cnt = ids[order], cnt[order]
        if n > self.max_entries:
            self.threshold_value = int(cnt[self.max_entries])
            if n > self.threshold_buffer:
                for id in ids[self.max_entries:].tolist():
                    self.entries.pop(id, None)
            ids, cnt = ids[:self.max_entries], cnt[:self.max_entries]
        else:
            self.threshold_value = 1
        # the (id, count) list is built when someone reads it (top()): a bulk
        # import re-ranks after every batch, TopN reads far less often
        self._ranked = (ids, cnt)
        self._rankings = None
        self.version += 1
        self.update_time = time.monotonic()
        # a re-rank with no write (the 10 s throttle expiring on a read, an
        # explicit recalculate) changes top() too: device rank-cache memos
        # skip their per-fragment version check only while the process-wide
        # mutation epoch stands still
        from pilosa_amd.models.fragment import _bump_epoch
        _bump_epoch()

    @property
    def rankings(self) -> List[Tuple[int, int]]:
        r = self._rankings
        if r is None:
            ids, cnt = self._ranked
            r = self._rankings = list(zip(ids.tolist(), cnt.tolist()))
        return r

    def top(self):
        return self.rankings


def new_cache(cache_type: str, size: int):
    if cache_type == CACHE_TYPE_RANKED:
        return RankCache(size)
    if cache_type == CACHE_TYPE_LRU:
        return LRUCache(size)
    return NopCache()
