"""Fragment: one (index, field, view, shard) bitmap (reference: fragment.go).

Storage is a host roaring ``Bitmap`` (C++ core) whose bit ``row*ShardWidth +
col%ShardWidth`` is set for every (row, column) pair.  Durability follows the
reference exactly: the file holds a Pilosa-format snapshot followed by an
append-only op log (13-byte ops with fnv32a checksums); opening replays the
log, a snapshot (write ``.snapshotting`` -> fsync -> rename) runs once more
than ``max_opn`` bits were logged (fragment.go:2284-2381).  A ``.cache`` file
(protobuf ``Cache{IDs}``) persists the TopN rank-cache membership.

Every mutation bumps ``version`` so the GPU arena (pilosa_amd/ops/) knows when
its HBM replica of this fragment is stale.
"""
from __future__ import annotations

import fcntl
import heapq
import io
import math
import os
import tarfile
import threading
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import xxhash

from pilosa_amd import _roaring
from pilosa_amd.errors import PilosaError
from pilosa_amd.models.cache import (CACHE_TYPE_NONE, CACHE_TYPE_RANKED, DEFAULT_CACHE_SIZE, Pair, new_cache,
                                     sort_pairs)
from pilosa_amd.models.row import Row

Bitmap = _roaring.Bitmap

from pilosa_amd.shardwidth import CONTAINERS_PER_ROW, SHARD_WIDTH  # noqa: E402
from pilosa_amd.shardwidth import EXPONENT as SHARD_WIDTH_EXP  # noqa: E402
HASH_BLOCK_SIZE = 100
DEFAULT_MAX_OPN = 10000
FALSE_ROW_ID, TRUE_ROW_ID = 0, 1
BSI_EXISTS_BIT, BSI_SIGN_BIT, BSI_OFFSET_BIT = 0, 1, 2
ROARING_FLAG_BSI_V2 = 0x01

OP_ADD, OP_REMOVE, OP_ADD_BATCH, OP_REMOVE_BATCH, OP_ADD_ROARING, OP_REMOVE_ROARING = range(6)


def pos(row: int, col: int) -> int:
    return row * SHARD_WIDTH + (col % SHARD_WIDTH)


class TopOptions:
    __slots__ = ("n", "src", "row_ids", "min_threshold", "filter_name", "filter_values", "tanimoto_threshold",
                 "attr_store")

    def __init__(self, n=0, src: Optional[Row] = None, row_ids: Optional[Sequence[int]] = None, min_threshold=0,
                 filter_name="", filter_values=None, tanimoto_threshold=0, attr_store=None):
        self.n = n
        self.src = src
        self.row_ids = list(row_ids or [])
        self.min_threshold = min_threshold
        self.filter_name = filter_name
        self.filter_values = filter_values or []
        self.tanimoto_threshold = tanimoto_threshold
        self.attr_store = attr_store



# Process-wide mutation epoch: bumped with every fragment version (and when a
# fragment is created), so device-side caches keyed on many fragments can
# skip re-reading each fragment's version while nothing changed.
_EPOCH = [0]


def _bump_epoch():
    _EPOCH[0] += 1


def mutation_epoch() -> int:
    return _EPOCH[0]


# bumped whenever the set of fragments, views or fields (or a field's remote
# available shards) changes: Index.available_shards is memoised on it
_SHARD_EPOCH = [0]


def bump_shard_epoch():
    _SHARD_EPOCH[0] += 1


def shard_epoch() -> int:
    return _SHARD_EPOCH[0]


def remove_stale_snapshots(dirpath: str, names: Iterable[str]) -> int:
    """Snapshot temp files (``<shard>.<pid>.<tid>.snapshotting``, or the old
    fixed ``<shard>.snapshotting``) left by a process that died mid-snapshot
    are never renamed: View.open drops them.  Files of this process may
    belong to a snapshot still running and are kept."""
    me = str(os.getpid())
    n = 0
    for nm in names:
        if not nm.endswith(".snapshotting"):
            continue
        parts = nm[:-len(".snapshotting")].split(".")
        if not parts[0].isdigit() or not all(p.isdigit() for p in parts) or len(parts) not in (1, 3):
            continue
        if len(parts) == 3 and parts[1] == me:
            continue
        try:
            os.unlink(os.path.join(dirpath, nm))
            n += 1
        except OSError:
            pass
    return n


class Fragment:
    def __init__(self, path: str, index: str, field: str, view: str, shard: int,
                 cache_type: str = CACHE_TYPE_RANKED, cache_size: int = DEFAULT_CACHE_SIZE,
                 max_opn: int = DEFAULT_MAX_OPN, mutex: bool = False, bool_field: bool = False, stats=None):
        self.path = path
        self.index, self.field, self.view, self.shard = index, field, view, int(shard)
        self.cache_type = cache_type
        self.cache_size = cache_size
        self.max_opn = max_opn
        self.mutex = mutex
        self.bool_field = bool_field
        self._storage = Bitmap()
        self._cache = new_cache(cache_type, cache_size)
        self.checksums: Dict[int, bytes] = {}
        self.opn = 0
        self.ops = 0
        self._file_gen = 0                 # bumped whenever the data file is replaced
        self._max_row_id = 0
        # lazy open: the file is only validated by its header; the storage (and
        # the rank cache that needs its counts) is read on first host access.
        # A GPU node reads cold fragments straight into HBM instead
        # (native/arena_io.cpp), so the host never holds their containers.
        self.lazy = False
        # cold host access: a copy-on-write mmap view of the file
        # (_roaring.MappedBitmap) serves membership, counts, row reads, the
        # rank cache and single-bit writes without reading the file into heap
        self._mapped = None
        self._flags_hint = 0
        self._cache_pending = False
        self.version = 0
        _bump_epoch()
        # per-consumer dirty-row sets (device arenas patch only changed rows);
        # None = unknown / too many -> the consumer refreshes the whole shard
        self._dirty_subs: Dict[object, Optional[set]] = {}
        self.mu = threading.RLock()
        self._fh = None
        self._lockfd = None
        self.stats = stats
        self.row_attr_store = None

    # ------------------------------------------------------------ lifecycle
    def open(self):
        with self.mu:
            self._open_storage()
            if self._storage is None:
                self._cache_pending = self.cache_type != CACHE_TYPE_NONE
            else:
                self._open_cache()
        return self

    # ------------------------------------------------------------ lazy storage
    @property
    def storage(self):
        s = self._storage
        if s is None:
            s = self._load_cold()
        return s

    @storage.setter
    def storage(self, bm):
        self._storage = bm
        self._cache_pending = False

    @property
    def cache(self):
        if self._cache_pending:
            with self.mu:
                if self._cache_pending:
                    self._open_cache()   # counts from the mapped file (fragment.go openCache)
        return self._cache

    @cache.setter
    def cache(self, c):
        self._cache = c

    @property
    def max_row_id(self) -> int:
        if self._storage is None and self._mapped is None:
            self._cold()
        return self._max_row_id

    @max_row_id.setter
    def max_row_id(self, v: int):
        self._max_row_id = v

    def cache_is_live(self) -> bool:
        """True once the rank cache has been opened in memory (a write opens
        it, mapped fragments included): from then on it, not the persisted
        ``.cache`` file, is the fragment's ranking."""
        return self.cache_type != CACHE_TYPE_NONE and not self._cache_pending

    def is_cold(self) -> bool:
        """True while the storage has not been read into heap.  The file is
        exactly the fragment's state: writes to a cold fragment go to the
        mapped view's overlay and to the op log appended to the file."""
        return self._storage is None

    def _cold(self):
        """The mapped view of a cold fragment (created on first use).  Past
        the process's map-count cap (utils/syswrap.py) the file is read into
        heap instead, as the reference falls back when mmap is refused."""
        with self.mu:
            m = self._mapped
            if m is None:
                from pilosa_amd.utils import syswrap
                if not syswrap.try_acquire():
                    return self._load_cold()
                try:
                    m = _roaring.MappedBitmap(self.path)
                except Exception as e:  # noqa: BLE001
                    syswrap.release()
                    raise PilosaError(f"unmarshal storage: file={self.path}, err={e}")
                self._mapped = m
                self.opn, self.ops = int(m.opn), int(m.ops)
                self._max_row_id = int(m.max()) // SHARD_WIDTH if m.any() else 0
            return m

    def _drop_mapped(self):
        if self._mapped is not None:
            from pilosa_amd.utils import syswrap
            self._mapped = None
            syswrap.release()

    def _rw(self):
        """Storage for the operations the mapped view offers: the heap
        Bitmap once materialised, else the mapped view."""
        s = self._storage
        return s if s is not None else self._cold()

    def mapped_stats(self) -> Optional[dict]:
        m = self._mapped
        if m is None or self._storage is not None:
            return None
        return {"mapped_bytes": int(m.mapped_bytes), "containers": int(m.mapped_containers),
                "overlay_containers": int(m.overlay_containers)}

    def _read_storage(self) -> Bitmap:
        with open(self.path, "rb") as fh:
            data = fh.read()
        try:
            return Bitmap.from_bytes(data)
        except Exception as e:  # noqa: BLE001
            raise PilosaError(f"unmarshal storage: file={self.path}, err={e}")

    def _load_cold(self) -> Bitmap:
        with self.mu:
            if self._storage is None:
                bm = self._read_storage()
                self.opn = int(bm.opn)
                self.ops = int(bm.ops)
                self._storage = bm
                self._drop_mapped()   # the file holds every write the mapped view took
                self._max_row_id = int(bm.max()) // SHARD_WIDTH if bm.any() else 0
            if self._cache_pending:
                self._cache_pending = False
                self._open_cache()
            return self._storage

    def _open_storage(self):
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        if os.path.exists(self.path) and os.path.getsize(self.path) > 0:
            if self.lazy:
                with open(self.path, "rb") as fh:
                    head = fh.read(8)
                if len(head) < 8:
                    raise PilosaError(f"unmarshal storage: file={self.path}, err=data too small")
                self._flags_hint = head[3] if int.from_bytes(head[:2], "little") == _roaring.MAGIC else 0
                self._storage = None
            else:
                bm = self._read_storage()
                self._storage = bm
                self.opn = int(bm.opn)
                self.ops = int(bm.ops)
        else:
            self.storage = Bitmap()
            # new fragments start with a valid empty snapshot (BSI v2 flag)
            self.storage.flags = ROARING_FLAG_BSI_V2
            with open(self.path, "wb") as fh:
                fh.write(self.storage.to_bytes())
        self._fh = open(self.path, "ab", buffering=0)
        try:
            fcntl.flock(self._fh.fileno(), fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError as e:
            raise PilosaError(f"flock: {e}")
        if self._storage is not None:
            self._max_row_id = int(self._storage.max()) // SHARD_WIDTH if self._storage.any() else 0
        self._bump()

    def _bump(self):
        self.version += 1
        _EPOCH[0] += 1

    def cache_path(self) -> str:
        return self.path + ".cache"

    def _open_cache(self):
        if self.cache_type == CACHE_TYPE_NONE:
            return
        self._cache_pending = False
        p = self.cache_path()
        if not os.path.exists(p):
            return
        # the protobuf Cache message read natively (a corrupt one is rebuilt)
        _, ids, ok = _roaring.read_cache_files([p], 1)
        if not ok[0]:
            return
        st = self._rw()
        ids = np.asarray(ids, dtype=np.uint64)
        if len(ids) and hasattr(self._cache, "bulk_add_many"):
            # one native call counts every cached row (openCache's CountRange per id)
            self._cache.bulk_add_many(ids, st.count_rows(ids, CONTAINERS_PER_ROW))
        else:
            for rid in ids.tolist():
                self._cache.bulk_add(rid, st.count_range(rid * SHARD_WIDTH, (rid + 1) * SHARD_WIDTH))
        self._cache.invalidate()

    def flush_cache(self):
        if self.cache_type == CACHE_TYPE_NONE or self._cache_pending:
            return  # cache never opened: the cache file on disk is current
        from pilosa_amd.wire import pb
        with self.mu:
            ids = self.cache.ids()
        data = pb.Cache(IDs=ids).SerializeToString()
        tmp = self.cache_path() + ".tmp"
        with open(tmp, "wb") as fh:
            fh.write(data)
        os.replace(tmp, self.cache_path())

    def close(self):
        with self.mu:
            try:
                self.flush_cache()
            except OSError:
                pass
            self._drop_mapped()
            if self._fh is not None:
                try:
                    fcntl.flock(self._fh.fileno(), fcntl.LOCK_UN)
                except OSError:
                    pass
                self._fh.close()
                self._fh = None

    # ------------------------------------------------------------ op log
    def _log(self, typ: int, value: int = 0, values: Optional[np.ndarray] = None, roaring: bytes = b"",
             opn: int = 0):
        if self._fh is None:
            return
        vals = values if values is not None else np.zeros(0, dtype=np.uint64)
        self._fh.write(_roaring.encode_op(typ, value, vals, roaring, opn))

    def _increment_opn(self, changed: int):
        if changed <= 0:
            return
        self.opn += changed
        self.ops += 1
        self._bump()
        if self.opn > self.max_opn:
            q = getattr(self, "snapshot_queue", None)
            if q is not None:
                q.enqueue(self)
            else:
                self.snapshot()

    def snapshot(self):
        """Write storage + truncate the op log (write -> fsync -> rename).

        Writers are only blocked while the storage is serialised and while
        the file is swapped: the write + fsync of the snapshot runs outside
        ``mu`` (unless the caller already holds it, e.g. ``set_row``).  Ops
        appended to the old file meanwhile are copied onto the new one before
        the rename, so none is lost; a snapshot that finds the file replaced
        under it (a newer snapshot, ``read_from``) discards its own.  The
        reference holds the fragment lock throughout (fragment.go:2240-2290).
        No second lock is taken, so a snapshot queued in the background and
        one run synchronously under ``mu`` cannot deadlock."""
        tmp = f"{self.path}.{os.getpid()}.{threading.get_ident()}.snapshotting"
        with self.mu:
            if self._fh is None and not os.path.exists(self.path):
                return  # closed/deleted while queued
            cold = self._storage is None
            if cold:
                # stream the mapped file + overlay straight to the new file:
                # the fragment is never read into heap (under mu: the overlay
                # must not change while it is written out)
                st = self._cold()
                if self._storage is not None:
                    cold = False   # past the map-count cap _cold() read it into heap
                else:
                    st.write_snapshot(tmp)
            if not cold:
                data = self.storage.to_bytes()
            gen = self._file_gen
            mark = self._file_size()
            opn0, ops0 = self.opn, self.ops
        with open(tmp, "r+b" if cold else "wb") as fh:
            if not cold:
                fh.write(data)
            fh.flush()
            os.fsync(fh.fileno())
        with self.mu:
            if gen != self._file_gen or (self._fh is None and not os.path.exists(self.path)):
                os.unlink(tmp)    # replaced (newer snapshot, read_from) or closed meanwhile
                return
            end = self._file_size()
            if end > mark:
                with open(self.path, "rb") as src, open(tmp, "ab") as dst:
                    src.seek(mark)
                    dst.write(src.read(end - mark))
                    dst.flush()
                    os.fsync(dst.fileno())
            if self._fh is not None:
                try:
                    fcntl.flock(self._fh.fileno(), fcntl.LOCK_UN)
                except OSError:
                    pass
                self._fh.close()
            os.replace(tmp, self.path)
            self._file_gen += 1
            if self._storage is None and self._mapped is not None:
                # re-map the new file: the overlay is in it now (plus any ops
                # appended meanwhile, which the new view replays)
                self._mapped = _roaring.MappedBitmap(self.path)
            self._fh = open(self.path, "ab", buffering=0)
            fcntl.flock(self._fh.fileno(), fcntl.LOCK_EX | fcntl.LOCK_NB)
            self.opn -= opn0
            self.ops -= ops0
            if self.stats:
                self.stats.count("snapshot", 1)

    def _file_size(self) -> int:
        if self._fh is not None:
            return os.fstat(self._fh.fileno()).st_size
        return os.path.getsize(self.path) if os.path.exists(self.path) else 0

    def upgrade_bsi_v2(self, bit_depth: int) -> bool:
        """Rewrite a v1 BSI fragment in the v2 layout (reference
        fragment.go:2717-2757 ``upgradeRoaringBSIv2``, view.go:436-454).  v1
        kept the bit planes at rows ``0..bitDepth-1`` and the not-null row at
        ``bitDepth``; v2 has exists=0, sign=1 and the planes from row 2.
        Returns True when the fragment was rewritten."""
        with self.mu:
            if self._storage is None and self._flags_hint & ROARING_FLAG_BSI_V2:
                return False
            if self.storage.flags & ROARING_FLAG_BSI_V2:
                return False
            vals = self.storage.slice()
            w = np.uint64(SHARD_WIDTH_EXP)
            rows = vals >> w
            low = vals & np.uint64(SHARD_WIDTH - 1)
            new_rows = np.where(rows == np.uint64(bit_depth), np.uint64(BSI_EXISTS_BIT),
                                rows + np.uint64(BSI_OFFSET_BIT))
            other = Bitmap(np.sort((new_rows << w) | low))
            other.flags = ROARING_FLAG_BSI_V2
            self.storage = other
        self.snapshot()  # write -> fsync -> rename, as the reference's tmp file + rename
        return True

    # ------------------------------------------------------------ rows
    def row(self, row_id: int) -> Row:
        with self.mu:
            bm = self._rw().offset_range(self.shard * SHARD_WIDTH, row_id * SHARD_WIDTH,
                                           (row_id + 1) * SHARD_WIDTH)
        return Row.from_segment(self.shard, bm)

    def row_bitmap(self, row_id: int) -> Bitmap:
        with self.mu:
            return self._rw().offset_range(self.shard * SHARD_WIDTH, row_id * SHARD_WIDTH,
                                             (row_id + 1) * SHARD_WIDTH)

    def row_count(self, row_id: int) -> int:
        with self.mu:
            return self._rw().count_range(row_id * SHARD_WIDTH, (row_id + 1) * SHARD_WIDTH)

    def row_intersection_count(self, row_id: int, other: "Fragment", other_row: int) -> int:
        """|row_id ∩ other.other_row| read in place (no row extraction).

        Host fast path for Count(Intersect(Row, Row)); the reference builds both
        rows with OffsetRange and intersects them (fragment.go:559-580,
        executor.go executeCount).  Locks are taken in a fixed order so two
        counts over the same pair of fragments cannot deadlock."""
        first, second = (self, other) if id(self) <= id(other) else (other, self)
        with first.mu:
            if second is first:
                return self.storage.range_intersection_count(row_id * SHARD_WIDTH, other.storage,
                                                             other_row * SHARD_WIDTH, SHARD_WIDTH)
            with second.mu:
                return self.storage.range_intersection_count(row_id * SHARD_WIDTH, other.storage,
                                                             other_row * SHARD_WIDTH, SHARD_WIDTH)

    def _pos(self, row_id: int, col: int) -> int:
        lo = self.shard * SHARD_WIDTH
        if col < lo or col >= lo + SHARD_WIDTH:
            raise PilosaError(f"column:{col} out of bounds")
        return pos(row_id, col)

    def bit(self, row_id: int, col: int) -> bool:
        p = self._pos(row_id, col)
        with self.mu:
            return self._rw().contains(p)

    DIRTY_LIMIT = 4096
    DELTA_LIMIT = 1 << 24     # recorded positions per subscriber before falling back to container keys

    # A dirty subscription is [rows, container keys, deltas, recorded positions]:
    # rows / keys changed in ways only the fragment storage can describe, and
    # the ordered write batches ("pos", sorted positions, clear) / ("roaring",
    # Bitmap, clear) that the device can replay itself (DeviceView.apply_deltas).
    def _note_rows(self, rows):
        for k, d in self._dirty_subs.items():
            if d is not None:
                d[0].update(rows)
                if len(d[0]) + len(d[1]) > self.DIRTY_LIMIT:
                    self._dirty_subs[k] = None

    def _note_container(self, pos: int):
        """A single-bit change: only container (row, key) of ``pos`` changed."""
        key = int(pos) >> 16
        for k, d in self._dirty_subs.items():
            if d is not None:
                d[1].add(key)
                if len(d[0]) + len(d[1]) > self.DIRTY_LIMIT:
                    self._dirty_subs[k] = None

    def _note_delta(self, kind: str, data, clear: bool, n: int):
        for k, d in self._dirty_subs.items():
            if d is None:
                continue
            d[2].append((kind, data, clear))
            d[3] += n
            if d[3] > self.DELTA_LIMIT or len(d[2]) > self.DIRTY_LIMIT:
                # too much to replay: degrade to the containers the batches touched
                if any(kd != "pos" for kd, _, _ in d[2]):
                    self._dirty_subs[k] = None
                    continue
                for _, dd, _ in d[2]:
                    d[1].update(np.unique(dd >> np.uint64(16)).tolist())
                d[2].clear()
                d[3] = 0
                if len(d[0]) + len(d[1]) > self.DIRTY_LIMIT:
                    self._dirty_subs[k] = None

    def _note_unknown(self):
        for k in self._dirty_subs:
            self._dirty_subs[k] = None

    def take_dirty(self, token):
        """(rows, container keys, deltas) changed since ``token`` last asked;
        container keys are row*16 + local key, deltas the ordered write
        batches.  None = unknown -> refresh everything; the first call
        registers the token and returns None."""
        with self.mu:
            if token not in self._dirty_subs:
                self._dirty_subs[token] = [set(), set(), [], 0]
                return None
            d = self._dirty_subs[token]
            self._dirty_subs[token] = [set(), set(), [], 0]
            return None if d is None else (d[0], d[1], d[2])

    def drop_dirty(self, token):
        with self.mu:
            self._dirty_subs.pop(token, None)

    def _after_row_change(self, row_id: int, bulk: bool = False, pos: Optional[int] = None, clear: bool = False):
        if self._dirty_subs:
            if pos is None:
                self._note_rows((row_id,))
            else:
                self._note_delta("pos", np.array([pos], np.uint64), clear, 1)
        self.checksums.pop(row_id // HASH_BLOCK_SIZE, None)
        if self.cache_type != CACHE_TYPE_NONE:
            n = self._rw().count_range(row_id * SHARD_WIDTH, (row_id + 1) * SHARD_WIDTH)
            if bulk:
                self.cache.bulk_add(row_id, n)
            else:
                self.cache.add(row_id, n)
        if row_id > self.max_row_id:
            self.max_row_id = row_id

    def _after_rows_change(self, rows: np.ndarray, note: bool = True):
        """Vectorised :meth:`_after_row_change` for bulk imports: one native
        call counts every touched row (fragment.go bulkImport cache refresh)."""
        if not len(rows):
            return
        if self._dirty_subs and note:
            self._note_rows(rows.tolist())
        for b in np.unique(rows // np.uint64(HASH_BLOCK_SIZE)).tolist():
            self.checksums.pop(int(b), None)
        if self.cache_type != CACHE_TYPE_NONE:
            counts = self._rw().count_rows(rows, CONTAINERS_PER_ROW)
            bulk = getattr(self.cache, "bulk_add_many", None)
            if bulk is not None:
                bulk(rows, counts)
            else:
                add = self.cache.bulk_add
                for rid, n in zip(rows.tolist(), counts.tolist()):
                    add(rid, n)
        mx = int(rows.max())
        if mx > self.max_row_id:
            self.max_row_id = mx

    def _unprotected_set_bit(self, row_id: int, col: int) -> bool:
        p = self._pos(row_id, col)
        changed = self._rw().add(p)
        if not changed:
            return False
        self._log(OP_ADD, p)
        self._after_row_change(row_id, pos=p)
        self._increment_opn(1)
        if self.stats:
            self.stats.count("setBit", 1)
        return True

    def _unprotected_clear_bit(self, row_id: int, col: int) -> bool:
        p = self._pos(row_id, col)
        changed = self._rw().remove(p)
        if not changed:
            return False
        self._log(OP_REMOVE, p)
        self._after_row_change(row_id, pos=p, clear=True)
        self._increment_opn(1)
        if self.stats:
            self.stats.count("clearBit", 1)
        return True

    def set_bit(self, row_id: int, col: int) -> bool:
        with self.mu:
            changed = False
            if self.mutex or self.bool_field:
                existing = self._vector_get(col)
                if existing is not None and existing != row_id:
                    self._unprotected_clear_bit(existing, col)
                    changed = True
            return self._unprotected_set_bit(row_id, col) or changed

    def clear_bit(self, row_id: int, col: int) -> bool:
        with self.mu:
            return self._unprotected_clear_bit(row_id, col)

    def _vector_get(self, col: int) -> Optional[int]:
        rows = self._rw().rows_with_column(col % SHARD_WIDTH, CONTAINERS_PER_ROW)
        if len(rows) > 1:
            raise PilosaError("found multiple row values for column")
        if len(rows) == 1:
            r = int(rows[0])
            if self.bool_field and r not in (FALSE_ROW_ID, TRUE_ROW_ID):
                raise PilosaError("found non-boolean value")
            return r
        return None

    def set_row(self, row: Row, row_id: int) -> bool:
        """Replace ``row_id`` with the segment of ``row`` for this shard."""
        with self.mu:
            seg = row.segment(self.shard)
            src = seg if seg is not None else Bitmap()
            self.storage.set_row_from(row_id, src, self.shard * CONTAINERS_PER_ROW, CONTAINERS_PER_ROW)
            self._after_row_change(row_id, bulk=True)
            if self.cache_type != CACHE_TYPE_NONE:
                self.cache.invalidate()
            self._bump()
            self.snapshot()
            return True

    def clear_row(self, row_id: int) -> bool:
        with self.mu:
            changed = self.storage.clear_row(row_id, CONTAINERS_PER_ROW)
            self._note_rows((row_id,))
            self.cache.add(row_id, 0)
            self.checksums.pop(row_id // HASH_BLOCK_SIZE, None)
            self._bump()
            self.snapshot()
            return changed

    # ------------------------------------------------------------ BSI
    def value(self, col: int, bit_depth: int) -> Tuple[int, bool]:
        with self.mu:
            if not self.bit(BSI_EXISTS_BIT, col):
                return 0, False
            v = 0
            for i in range(bit_depth):
                if self.bit(BSI_OFFSET_BIT + i, col):
                    v |= 1 << i
            if self.bit(BSI_SIGN_BIT, col):
                v = -v
            return v, True

    def _positions_for_values(self, cols: np.ndarray, values: np.ndarray, bit_depth: int, clear: bool):
        cols = np.asarray(cols, dtype=np.uint64) % np.uint64(SHARD_WIDTH)
        values = np.asarray(values, dtype=np.int64)
        uval = np.abs(values).astype(np.uint64)
        sets, clears = [], []
        ex = np.uint64(BSI_EXISTS_BIT * SHARD_WIDTH) + cols
        (clears if clear else sets).append(ex)
        sg = np.uint64(BSI_SIGN_BIT * SHARD_WIDTH) + cols
        neg = (values < 0) & (not clear)
        sets.append(sg[neg])
        clears.append(sg[~neg])
        for i in range(bit_depth):
            p = np.uint64((BSI_OFFSET_BIT + i) * SHARD_WIDTH) + cols
            on = ((uval >> np.uint64(i)) & np.uint64(1)).astype(bool)
            sets.append(p[on])
            clears.append(p[~on])
        s = np.concatenate(sets) if sets else np.zeros(0, np.uint64)
        c = np.concatenate(clears) if clears else np.zeros(0, np.uint64)
        return s, c

    def set_value(self, col: int, bit_depth: int, value: int, clear: bool = False) -> bool:
        with self.mu:
            self._pos(0, col)
            s, c = self._positions_for_values(np.array([col], np.uint64), np.array([value], np.int64), bit_depth,
                                              clear)
            return self._import_positions(s, c, range(bit_depth + 2)) > 0

    def clear_value(self, col: int, bit_depth: int, value: int) -> bool:
        return self.set_value(col, bit_depth, value, clear=True)

    def sum(self, filt: Optional[Row], bit_depth: int) -> Tuple[int, int]:
        """fragment.go:1109.  NB: negatives are filtered too (the reference
        counts all negatives regardless of the filter; we apply it)."""
        consider = self.row(BSI_EXISTS_BIT)
        if filt is not None:
            consider = consider.intersect(filt)
        count = consider.count()
        nrow = self.row(BSI_SIGN_BIT).intersect(consider)
        prow = consider.difference(nrow)
        total = 0
        for i in range(bit_depth):
            r = self.row(BSI_OFFSET_BIT + i)
            total += (1 << i) * (r.intersection_count(prow) - r.intersection_count(nrow))
        return _wrap_i64(total), count

    def min(self, filt: Optional[Row], bit_depth: int) -> Tuple[int, int]:
        consider = self.row(BSI_EXISTS_BIT)
        if filt is not None:
            consider = consider.intersect(filt)
        if consider.count() == 0:
            return 0, 0
        neg = self.row(BSI_SIGN_BIT).intersect(consider)
        if neg.any():
            v, c = self._max_unsigned(neg, bit_depth)
            return -v, c
        return self._min_unsigned(consider, bit_depth)

    def max(self, filt: Optional[Row], bit_depth: int) -> Tuple[int, int]:
        consider = self.row(BSI_EXISTS_BIT)
        if filt is not None:
            consider = consider.intersect(filt)
        if not consider.any():
            return 0, 0
        pos_ = consider.difference(self.row(BSI_SIGN_BIT))
        if not pos_.any():
            v, c = self._min_unsigned(consider, bit_depth)
            return -v, c
        return self._max_unsigned(pos_, bit_depth)

    def _min_unsigned(self, filt: Row, bit_depth: int) -> Tuple[int, int]:
        mn, count = 0, 0
        for i in range(bit_depth - 1, -1, -1):
            row = filt.difference(self.row(BSI_OFFSET_BIT + i))
            count = row.count()
            if count > 0:
                filt = row
            else:
                mn += 1 << i
                if i == 0:
                    count = filt.count()
        return mn, count

    def _max_unsigned(self, filt: Row, bit_depth: int) -> Tuple[int, int]:
        mx, count = 0, 0
        for i in range(bit_depth - 1, -1, -1):
            row = self.row(BSI_OFFSET_BIT + i).intersect(filt)
            count = row.count()
            if count > 0:
                mx += 1 << i
                filt = row
            elif i == 0:
                count = filt.count()
        return mx, count

    def range_op(self, op: str, bit_depth: int, predicate: int) -> Row:
        if op == "==":
            return self._range_eq(bit_depth, predicate)
        if op == "!=":
            return self.row(BSI_EXISTS_BIT).difference(self._range_eq(bit_depth, predicate))
        if op in ("<", "<="):
            return self._range_lt(bit_depth, predicate, op == "<=")
        if op in (">", ">="):
            return self._range_gt(bit_depth, predicate, op == ">=")
        from pilosa_amd.errors import ErrInvalidRangeOperation
        raise ErrInvalidRangeOperation

    def not_null(self) -> Row:
        return self.row(BSI_EXISTS_BIT)

    def _range_eq(self, bit_depth, predicate):
        b = self.row(BSI_EXISTS_BIT)
        up = abs(predicate)
        if predicate < 0:
            b = b.intersect(self.row(BSI_SIGN_BIT))
        else:
            b = b.difference(self.row(BSI_SIGN_BIT))
        for i in range(bit_depth - 1, -1, -1):
            row = self.row(BSI_OFFSET_BIT + i)
            b = b.intersect(row) if (up >> i) & 1 else b.difference(row)
        return b

    def _range_lt(self, bit_depth, predicate, allow_eq):
        b = self.row(BSI_EXISTS_BIT)
        up = abs(predicate)
        if (predicate >= 0 and allow_eq) or (predicate >= -1 and not allow_eq):
            pos_ = self._range_lt_unsigned(b.difference(self.row(BSI_SIGN_BIT)), bit_depth, up, allow_eq)
            return self.row(BSI_SIGN_BIT).union(pos_)
        return self._range_gt_unsigned(b.intersect(self.row(BSI_SIGN_BIT)), bit_depth, up, allow_eq)

    def _range_lt_unsigned(self, filt: Row, bit_depth, predicate, allow_eq):
        keep = Row()
        leading_zeros = True
        for i in range(bit_depth - 1, -1, -1):
            row = self.row(BSI_OFFSET_BIT + i)
            bit = (predicate >> i) & 1
            if leading_zeros:
                if bit == 0:
                    filt = filt.difference(row)
                    continue
                leading_zeros = False
            if i == 0 and not allow_eq:
                if bit == 0:
                    return keep
                return filt.difference(row.difference(keep))
            if bit == 0:
                filt = filt.difference(row.difference(keep))
                continue
            if i > 0:
                keep = keep.union(filt.difference(row))
        return filt

    def _range_gt(self, bit_depth, predicate, allow_eq):
        b = self.row(BSI_EXISTS_BIT)
        up = abs(predicate)
        if (predicate >= 0 and allow_eq) or (predicate >= -1 and not allow_eq):
            return self._range_gt_unsigned(b.difference(self.row(BSI_SIGN_BIT)), bit_depth, up, allow_eq)
        neg = self._range_lt_unsigned(b.intersect(self.row(BSI_SIGN_BIT)), bit_depth, up, allow_eq)
        return b.difference(self.row(BSI_SIGN_BIT)).union(neg)

    def _range_gt_unsigned(self, filt: Row, bit_depth, predicate, allow_eq):
        keep = Row()
        for i in range(bit_depth - 1, -1, -1):
            row = self.row(BSI_OFFSET_BIT + i)
            bit = (predicate >> i) & 1
            if i == 0 and not allow_eq:
                if bit == 1:
                    return keep
                return filt.difference(filt.difference(row).difference(keep))
            if bit == 1:
                filt = filt.difference(filt.difference(row).difference(keep))
                continue
            if i > 0:
                keep = keep.union(filt.intersect(row))
        return filt

    def range_between(self, bit_depth, pmin, pmax) -> Row:
        b = self.row(BSI_EXISTS_BIT)
        umin, umax = abs(pmin), abs(pmax)
        if pmin >= 0:
            return self._range_between_unsigned(b.difference(self.row(BSI_SIGN_BIT)), bit_depth, umin, umax)
        if pmax < 0:
            return self._range_between_unsigned(b.intersect(self.row(BSI_SIGN_BIT)), bit_depth, umax, umin)
        pos_ = self._range_lt_unsigned(b.difference(self.row(BSI_SIGN_BIT)), bit_depth, umax, True)
        neg = self._range_lt_unsigned(b.intersect(self.row(BSI_SIGN_BIT)), bit_depth, umin, True)
        return pos_.union(neg)

    def _range_between_unsigned(self, filt: Row, bit_depth, pmin, pmax):
        keep1, keep2 = Row(), Row()
        for i in range(bit_depth - 1, -1, -1):
            row = self.row(BSI_OFFSET_BIT + i)
            b1, b2 = (pmin >> i) & 1, (pmax >> i) & 1
            if b1 == 1:
                filt = filt.difference(filt.difference(row).difference(keep1))
            elif i > 0:
                keep1 = keep1.union(filt.intersect(row))
            if b2 == 0:
                filt = filt.difference(row.difference(keep2))
            elif i > 0:
                keep2 = keep2.union(filt.difference(row))
        return filt

    # ------------------------------------------------------------ min/max row
    def min_row_id(self) -> Tuple[int, bool]:
        if not self.storage.any():
            return 0, False
        return int(self.storage.min()) // SHARD_WIDTH, True

    def min_row(self, filt: Optional[Row]) -> Tuple[int, int]:
        mn, ok = self.min_row_id()
        if not ok:
            return 0, 0
        if filt is None:
            return mn, 1
        for r in self.rows(mn):
            c = self.row(r).intersection_count(filt)
            if c > 0:
                return r, c
        return 0, 0

    def max_row(self, filt: Optional[Row]) -> Tuple[int, int]:
        mn, ok = self.min_row_id()
        if not ok:
            return 0, 0
        mx = int(self.storage.max()) // SHARD_WIDTH
        if filt is None:
            return mx, 1
        for r in reversed(self.rows(mn)):
            c = self.row(r).intersection_count(filt)
            if c > 0:
                return r, c
        return 0, 0

    # ------------------------------------------------------------ rows listing
    def rows(self, start: int = 0, column: Optional[int] = None, limit: Optional[int] = None,
             row_filter: Optional[Sequence[int]] = None) -> List[int]:
        """Non-empty row ids >= start (fragment.go:2675-2712 with the
        column / rows / limit filters of :2601-2667)."""
        with self.mu:
            if column is not None:
                ids = self.storage.rows_with_column(column % SHARD_WIDTH, CONTAINERS_PER_ROW)
            else:
                ids = self.storage.row_ids(CONTAINERS_PER_ROW)
        ids = ids[ids >= np.uint64(start)] if len(ids) else ids
        if row_filter is not None:
            ids = ids[np.isin(ids, np.asarray(row_filter, dtype=np.uint64))]
        out = [int(x) for x in ids]
        if limit is not None:
            out = out[:limit]
        return out

    def row_iterator(self, wrap: bool, row_filter: Optional[Sequence[int]] = None) -> "RowIterator":
        """Iterator over the non-empty rows (fragment.go rowIterator, the
        GroupBy building block): next() -> (row, id, wrapped)."""
        return RowIterator(self, wrap, row_filter)

    # ------------------------------------------------------------ TopN
    def top(self, opt: TopOptions) -> List[Pair]:
        pairs = self._top_bitmap_pairs(opt.row_ids)
        n = 0 if opt.row_ids else opt.n
        filters = None
        if opt.filter_name and opt.filter_values:
            filters = set(_hashable(v) for v in opt.filter_values)
        tan = 0
        min_t = max_t = 0.0
        src_count = 0
        if opt.tanimoto_threshold > 0 and opt.src is not None:
            tan = opt.tanimoto_threshold
            src_count = opt.src.count()
            min_t = float(src_count * tan) / 100
            max_t = float(src_count * 100) / float(tan)
        heap: List[Tuple[int, int]] = []  # (count, -id) min-heap
        results: List[Pair] = []
        for row_id, cnt in pairs:
            if cnt == 0:
                continue
            if tan > 0:
                if cnt <= min_t or cnt >= max_t:
                    continue
            elif cnt < opt.min_threshold:
                continue
            if filters is not None:
                attrs = opt.attr_store.attrs(row_id) if opt.attr_store is not None else None
                if not attrs or attrs.get(opt.filter_name) is None or \
                        _hashable(attrs.get(opt.filter_name)) not in filters:
                    continue
            if n == 0 or len(heap) < n:
                count = cnt
                if opt.src is not None:
                    count = opt.src.intersection_count(self.row(row_id))
                if count == 0:
                    continue
                if tan > 0:
                    t = math.ceil(float(count * 100) / float(cnt + src_count - count))
                    if t <= tan:
                        continue
                elif count < opt.min_threshold:
                    continue
                heapq.heappush(heap, (count, -row_id))
                if n > 0 and len(heap) == n and opt.src is None:
                    break
                continue
            threshold = heap[0][0]
            if threshold < opt.min_threshold or cnt < threshold:
                break
            count = opt.src.intersection_count(self.row(row_id))
            if count < threshold:
                continue
            heapq.heappush(heap, (count, -row_id))
        results = [Pair(-nid, c) for c, nid in heap]
        return sort_pairs(results)

    def _top_bitmap_pairs(self, row_ids: Sequence[int]) -> List[Tuple[int, int]]:
        # no cache: nothing, even for explicit ids (fragment.go topBitmapPairs)
        if self.cache_type == CACHE_TYPE_NONE:
            return list(self.cache.top())
        if not row_ids:
            with self.mu:
                self.cache.invalidate()
                return list(self.cache.top())
        out = []
        for rid in row_ids:
            n = self.cache.get(rid)
            if n > 0:
                out.append((rid, n))
                continue
            c = self.row_count(rid)
            if c > 0:
                out.append((rid, c))
        out.sort(key=lambda kv: (-kv[1], kv[0]))
        return out

    def recalculate_cache(self):
        with self.mu:
            self.cache.recalculate()

    def rebuild_cache(self):
        """Recount every row into the cache (used after bulk device imports)."""
        with self.mu:
            if self.cache_type == CACHE_TYPE_NONE:
                return
            for rid, n in self.storage.row_counts(CONTAINERS_PER_ROW).items():
                self.cache.bulk_add(int(rid), int(n))
            self.cache.recalculate()

    # ------------------------------------------------------------ imports
    def _import_positions(self, set_pos: np.ndarray, clear_pos: np.ndarray, row_set: Iterable[int]) -> int:
        changed = 0
        if len(set_pos):
            set_pos = np.unique(np.asarray(set_pos, dtype=np.uint64))
            n = self._rw().add_many(set_pos, True)
            if n:
                self._log(OP_ADD_BATCH, values=set_pos)
                if self._dirty_subs:
                    self._note_delta("pos", set_pos, False, len(set_pos))
            changed += n
        if len(clear_pos):
            clear_pos = np.unique(np.asarray(clear_pos, dtype=np.uint64))
            n = self._rw().remove_many(clear_pos)
            if n:
                self._log(OP_REMOVE_BATCH, values=clear_pos)
                if self._dirty_subs:
                    self._note_delta("pos", clear_pos, True, len(clear_pos))
            changed += n
        rows = row_set if isinstance(row_set, np.ndarray) else np.fromiter((int(r) for r in row_set), dtype=np.uint64)
        self._after_rows_change(rows.astype(np.uint64, copy=False), note=False)
        if self.cache_type != CACHE_TYPE_NONE:
            self.cache.recalculate()
        self._increment_opn(changed)
        if self.stats:
            self.stats.count("ImportedN", changed)
        self._bump()
        return changed

    def bulk_import(self, row_ids: Sequence[int], col_ids: Sequence[int], clear: bool = False) -> int:
        rows = np.asarray(row_ids, dtype=np.uint64)
        cols = np.asarray(col_ids, dtype=np.uint64)
        if len(rows) != len(cols):
            raise PilosaError(f"mismatch of row/column len: {len(rows)} != {len(cols)}")
        lo = np.uint64(self.shard * SHARD_WIDTH)
        if len(cols) and (np.any(cols < lo) or np.any(cols >= lo + np.uint64(SHARD_WIDTH))):
            bad = int(cols[(cols < lo) | (cols >= lo + np.uint64(SHARD_WIDTH))][0])
            raise PilosaError(f"column:{bad} out of bounds")
        with self.mu:
            if (self.mutex or self.bool_field) and not clear:
                return self._bulk_import_mutex(rows, cols)
            positions = rows * np.uint64(SHARD_WIDTH) + (cols % np.uint64(SHARD_WIDTH))
            row_set = np.unique(rows)
            if clear:
                return self._import_positions(np.zeros(0, np.uint64), positions, row_set)
            return self._import_positions(positions, np.zeros(0, np.uint64), row_set)

    def _bulk_import_mutex(self, rows: np.ndarray, cols: np.ndarray) -> int:
        to_set: Dict[int, int] = {}
        to_clear: List[int] = []
        row_set = set()
        for r, c in zip(rows.tolist(), cols.tolist()):
            existing = self._vector_get(c)
            if existing is not None and existing != r:
                to_clear.append(pos(existing, c))
                row_set.add(existing)
            elif existing is not None and existing == r:
                continue
            if c in to_set:  # a later bit for the same column wins
                prev_row = to_set[c] // SHARD_WIDTH
                row_set.add(prev_row)
            to_set[c] = pos(r, c)
            row_set.add(r)
        return self._import_positions(np.array(list(to_set.values()), np.uint64),
                                      np.array(to_clear, np.uint64), row_set)

    def import_value(self, col_ids: Sequence[int], values: Sequence[int], bit_depth: int, clear: bool = False):
        cols = np.asarray(col_ids, dtype=np.uint64)
        vals = np.asarray(values, dtype=np.int64)
        if len(cols) != len(vals):
            raise PilosaError(f"mismatch of column/value len: {len(cols)} != {len(vals)}")
        # last write per column wins (fragment.go importValueSmallWrite iterates backwards)
        if len(cols):
            _, idx = np.unique(cols[::-1], return_index=True)
            keep = len(cols) - 1 - idx
            cols, vals = cols[keep], vals[keep]
        with self.mu:
            s, c = self._positions_for_values(cols, vals, bit_depth, clear)
            c = np.setdiff1d(c, s)
            return self._import_positions(s, c, range(bit_depth + 2))

    def import_roaring(self, data: bytes, clear: bool = False) -> int:
        with self.mu:
            changed, rowdelta = self._rw().import_roaring(data, clear, CONTAINERS_PER_ROW)
            if changed and self._dirty_subs:
                # the device merges the imported containers itself (K12)
                self._note_delta("roaring", Bitmap.from_bytes(data), clear, int(changed))
            if changed:
                self._log(OP_REMOVE_ROARING if clear else OP_ADD_ROARING, roaring=data, opn=changed)
            any_changed = False
            for rid, d in rowdelta.items():
                if d == 0:
                    continue
                self.checksums.pop(int(rid) // HASH_BLOCK_SIZE, None)
                if int(rid) > self.max_row_id:
                    self.max_row_id = int(rid)
                if self.cache_type != CACHE_TYPE_NONE:
                    any_changed = True
                    self.cache.bulk_add(int(rid), max(0, self.cache.get(int(rid)) + int(d)))
            if any_changed:
                self.cache.recalculate()
            self._increment_opn(changed)
            self._bump()
            return changed

    # ------------------------------------------------------------ anti-entropy
    def blocks(self) -> List[Tuple[int, bytes]]:
        """(block id, xxhash64 checksum) of every 100-row block with data
        (fragment.go:1776-1854; values hashed big-endian)."""
        with self.mu:
            vals = self.storage.slice()
        if len(vals) == 0:
            return []
        bids = vals // np.uint64(HASH_BLOCK_SIZE * SHARD_WIDTH)
        out = []
        bounds = np.flatnonzero(np.diff(bids)) + 1
        starts = np.concatenate([[0], bounds])
        ends = np.concatenate([bounds, [len(vals)]])
        for s, e in zip(starts, ends):
            bid = int(bids[s])
            cached = self.checksums.get(bid)
            if cached is None:
                cached = xxhash.xxh64(vals[s:e].astype(">u8").tobytes()).digest()
                self.checksums[bid] = cached
            out.append((bid, cached))
        return out

    def checksum(self) -> bytes:
        h = xxhash.xxh64()
        for _, c in self.blocks():
            h.update(c)
        return h.digest()

    def block_data(self, block_id: int) -> Tuple[np.ndarray, np.ndarray]:
        lo = block_id * HASH_BLOCK_SIZE * SHARD_WIDTH
        hi = (block_id + 1) * HASH_BLOCK_SIZE * SHARD_WIDTH
        with self.mu:
            v = self.storage.slice_range(lo, hi)
        return v // np.uint64(SHARD_WIDTH), v % np.uint64(SHARD_WIDTH)

    def merge_block(self, block_id: int, data: List[Tuple[Sequence[int], Sequence[int]]]):
        """Majority-vote merge of replica block data (fragment.go:1873-1991).
        Returns (sets, clears) diffs per remote replica.  The reference walks
        the replicas' sorted pair iterators in lockstep; here every replica's
        pairs become sorted position arrays (models/iterator.py) and the vote
        is one counted union over them."""
        from pilosa_amd.models.iterator import pairs_to_positions
        lr, lc = self.block_data(block_id)
        lo, hi = block_id * HASH_BLOCK_SIZE, (block_id + 1) * HASH_BLOCK_SIZE
        sets_all = [pairs_to_positions(lr, lc)]
        for rows, cols in data:
            if len(rows) != len(cols):
                raise PilosaError(f"pair set mismatch: {len(rows)} != {len(cols)}")
            r = np.asarray(rows, dtype=np.uint64)
            c = np.asarray(cols, dtype=np.uint64)
            keep = (r >= np.uint64(lo)) & (r < np.uint64(hi)) & (c < np.uint64(SHARD_WIDTH))
            sets_all.append(pairs_to_positions(r[keep], c[keep]))
        majority = (len(sets_all) + 1) // 2
        uniq, cnt = np.unique(np.concatenate(sets_all), return_counts=True)
        want = uniq[cnt >= majority]
        w = np.uint64(SHARD_WIDTH)

        def split(p):
            return (p // w).tolist(), (p % w).tolist()
        sets = [split(np.setdiff1d(want, have, assume_unique=True)) for have in sets_all]
        clears = [split(np.setdiff1d(have, want, assume_unique=True)) for have in sets_all]
        with self.mu:
            for r, c in zip(*sets[0]):
                self._unprotected_set_bit(r, self.shard * SHARD_WIDTH + c)
            for r, c in zip(*clears[0]):
                self._unprotected_clear_bit(r, self.shard * SHARD_WIDTH + c)
        return sets[1:], clears[1:]

    # ------------------------------------------------------------ backup
    def write_to(self, fileobj) -> None:
        """Tar archive with ``data`` (snapshot) and ``cache`` entries
        (fragment.go:2424-2500)."""
        from pilosa_amd.wire import pb
        with self.mu:
            data = self.storage.to_bytes()
            ids = self.cache.ids()
        cache = pb.Cache(IDs=ids).SerializeToString()
        with tarfile.open(fileobj=fileobj, mode="w|") as tw:
            for name, payload in (("data", data), ("cache", cache)):
                ti = tarfile.TarInfo(name)
                ti.size = len(payload)
                ti.mode = 0o600
                tw.addfile(ti, io.BytesIO(payload))

    def read_from(self, fileobj) -> None:
        from pilosa_amd.wire import pb
        with tarfile.open(fileobj=fileobj, mode="r|") as tr:
            for ti in tr:
                payload = tr.extractfile(ti).read() if ti.isfile() else b""
                if ti.name == "data":
                    with self.mu:
                        self.storage = Bitmap.from_bytes(payload)
                        self._drop_mapped()   # the old mapping views the replaced inode
                        self._note_unknown()
                        tmp = self.path + ".snapshotting"
                        with open(tmp, "wb") as fh:
                            fh.write(payload)
                        if self._fh is not None:
                            try:
                                fcntl.flock(self._fh.fileno(), fcntl.LOCK_UN)
                            except OSError:
                                pass
                            self._fh.close()
                        os.replace(tmp, self.path)
                        self._file_gen += 1
                        self._fh = open(self.path, "ab", buffering=0)
                        fcntl.flock(self._fh.fileno(), fcntl.LOCK_EX | fcntl.LOCK_NB)
                        self.opn = 0
                        self._bump()
                elif ti.name == "cache":
                    m = pb.Cache()
                    m.ParseFromString(payload)
                    with self.mu:
                        self.cache = new_cache(self.cache_type, self.cache_size)
                        for rid in m.IDs:
                            self.cache.bulk_add(rid, self.row_count(rid))
                        self.cache.recalculate()

    # ------------------------------------------------------------ misc
    def for_each_bit(self):
        with self.mu:
            v = self.storage.slice()
        base = self.shard * SHARD_WIDTH
        for x in v.tolist():
            yield x // SHARD_WIDTH, base + (x % SHARD_WIDTH)

    def check(self) -> str:
        return self.storage.check()


class RowIterator:
    """fragment.go:2714-2778 rowIterator: rows in id order; a wrapping
    iterator restarts from the first row (wrapped=True) after the last, a
    non-wrapping one then returns (None, 0, True)."""

    def __init__(self, frag: "Fragment", wrap: bool, row_filter: Optional[Sequence[int]] = None):
        self.f = frag
        self.wrap = wrap
        self.ids = frag.rows(0, row_filter=row_filter)
        self.cur = 0

    def seek(self, row_id: int):
        self.cur = int(np.searchsorted(np.asarray(self.ids, dtype=np.uint64), np.uint64(row_id)))

    def next(self):
        wrapped = False
        if self.cur >= len(self.ids):
            if not self.wrap or not self.ids:
                return None, 0, True
            self.cur = 0
            wrapped = True
        rid = self.ids[self.cur]
        self.cur += 1
        return self.f.row(rid), rid, wrapped


def _wrap_i64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def _hashable(v):
    if isinstance(v, list):
        return tuple(v)
    return v
