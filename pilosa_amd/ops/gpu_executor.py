"""GPU execution of PQL calls over all local shards at once.

The host executor (pilosa_amd/executor.py) hands the *local* part of every
map/reduce to this class; instead of the reference's per-shard worker loop
(executor.go:2564-2611) each call becomes ONE batched kernel launch over the
device arenas of the involved field-views:

* ``count``     Count(<bitmap tree>)                 -> expr_count
* ``bitmap``    Row/Intersect/Union/Difference/Xor/Not/time ranges -> materialize
* ``bsi_sum``   Sum(<filter>, field=f)                -> bsi_sum kernel
* ``topn``      TopN phase-1/phase-2 with src          -> slot-index LDS
                histogram + in-kernel heap walk (ops/topn_index.py); while
                that index is stale: per-shard pair counts + the reference
                heap semantics replayed on host (fragment.top)
* ``group_by``  GroupBy(Rows..., filter)               -> batched k-way counts

Arenas are (re)built lazily from the host fragments and cached per
(index, field, view, shard list); every fragment carries a ``version`` that is
bumped on mutation, so stale arenas are rebuilt before use.  Anything not
expressible on the device raises ``NotImplementedError`` -> host fallback.
"""
from __future__ import annotations

import os
import threading
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from pilosa_amd import shardwidth
from pilosa_amd.errors import PilosaError
from pilosa_amd.utils import tracing
from pilosa_amd.models.cache import Pair, sort_pairs
from pilosa_amd.models.fragment import SHARD_WIDTH, mutation_epoch
from pilosa_amd.models.index import EXISTENCE_FIELD_NAME
from pilosa_amd.models.row import Row
from pilosa_amd.models.view import VIEW_BSI_PREFIX, VIEW_STANDARD
from pilosa_amd.pql import Call

from .device import CompileError, DeviceView, GpuEngine, Leaf, Op

MAX_GROUPS_PER_LAUNCH = 1 << 16
# two-field GroupBy with at least this many row pairs runs as one count matrix
GROUPBY_MATRIX_MIN = int(os.environ.get("PILOSA_GROUPBY_MATRIX_MIN", "1024"))
# minimum spacing of device TopN index rebuilds per view (the reference
# re-ranks its caches at most every 10 s too, cache.go:235-243)
TOPN_INDEX_REBUILD_S = float(os.environ.get("PILOSA_TOPN_INDEX_REBUILD_S", "10"))


class _Empty:
    """Placeholder for a leaf whose field/view does not exist (empty row)."""


EMPTY = _Empty()


def _delta_keys(deltas) -> set:
    """Container keys (row*16 + key) touched by recorded write batches."""
    out = set()
    for kind, data, _ in deltas:
        pos = data if kind == "pos" else data.slice()
        out.update(np.unique(np.asarray(pos, dtype=np.uint64) >> np.uint64(16)).tolist())
    return out


class SubFragment:
    """Device sub-shard ``sub`` of a fragment wider than the device shard
    (shard width 2^21..2^32, pilosa_amd/shardwidth.py): what the arena
    builder reads of a fragment -- lock, version, file, dirty rows -- with
    its own dirty subscription per sub-shard and only the container keys of
    its sub-shard.  Write batches are not replayed on the device at these
    widths: their containers are rebuilt from the storage instead."""
    __slots__ = ("frag", "sub")

    def __init__(self, frag, sub: int):
        self.frag = frag
        self.sub = int(sub)

    @property
    def mu(self):
        return self.frag.mu

    @property
    def version(self):
        return self.frag.version

    @property
    def path(self):
        return self.frag.path

    @property
    def storage(self):
        return self.frag.storage

    def is_cold(self) -> bool:
        return self.frag.is_cold()

    def device_storage(self):
        """This sub-shard's containers re-keyed to the arena (row * 16 + slot)."""
        return self.frag.storage.sub_shard(shardwidth.KEY_SHIFT, self.sub)

    def take_dirty(self, token):
        d = self.frag.take_dirty((token, self.sub))
        if d is None:
            return None
        rows, keys, deltas = d
        keys = set(keys) | _delta_keys(deltas)
        return rows, {k for k in keys if shardwidth.sub_of_key(k) == self.sub}, []

    def drop_dirty(self, token):
        self.frag.drop_dirty((token, self.sub))


def _device_frags(v, shards) -> list:
    """The arena's per-device-shard fragments of holder view ``v`` for host
    ``shards`` (sub-shard proxies above 2^20 columns)."""
    if not shardwidth.WIDE:
        return [v.fragment(s) for s in shards]
    out = []
    for s in shards:
        f = v.fragment(s)
        out.extend(SubFragment(f, i) if f is not None else None for i in range(shardwidth.DEVICE_SUBSHARDS))
    return out


def _fid(f) -> int:
    """Identity of the fragment behind an arena shard (proxies are per call)."""
    return id(f.frag) if isinstance(f, SubFragment) else id(f)


def _dev_storage(f):
    return f.device_storage() if isinstance(f, SubFragment) else f.storage


def _nreq(ns) -> int:
    """The cache prefix a cache-only group needs: its largest n rounded up to
    a power of two (0 = all).  Rounded so batches of varied n share one node
    candidate space / count-matrix memo per bucket instead of one per
    distinct n (the membership kernel still stops each call at its own n)."""
    from .topn_exec import prefix_bucket
    ns = [int(n) for n in ns]
    return 0 if any(n == 0 for n in ns) else prefix_bucket(max(ns))


class GpuExecutor:
    def __init__(self, holder, device="cuda:0", executor=None, hbm_budget: int = 0):
        if not shardwidth.device_supported():
            raise NotImplementedError(f"device arenas hold shards of 2^{shardwidth.MIN_EXPONENT}.."
                                      f"2^{shardwidth.DEVICE_EXPONENT} columns "
                                      f"(PILOSA_SHARD_WIDTH={shardwidth.EXPONENT})")
        self.holder = holder
        self.engine = GpuEngine(device)
        self.device = self.engine.device
        self.executor = executor
        # arena cache in LRU order; hbm_budget > 0 caps the resident bytes
        # (least recently used views are dropped and rebuilt on demand)
        self.hbm_budget = int(hbm_budget)
        self.evictions = 0
        self._arenas: "OrderedDict[Tuple, Tuple[Tuple, DeviceView]]" = OrderedDict()
        self._arena_epoch: Dict[Tuple, int] = {}  # mutation epoch at the last validation of each arena
        self._bsi_views: Dict[Tuple, DeviceView] = {}  # predicate results (small LRU)
        self.mu = threading.RLock()
        self.launches = 0
        # serving Count text path: host prep (parse..launch) vs result wait
        self.text_batches = 0
        self.text_prep_s = 0.0
        self.text_wait_s = 0.0
        self.topn_index_refreshes = 0   # slot indexes brought up to date in place after writes
        self.topn_index_builds = 0      # full slot-index builds, and their wall time (synchronised)
        self.topn_index_build_s = 0.0
        self.topn_index_batches = 0     # src TopN batches / calls answered by a slot index
        self.rebuilds = 0        # full view uploads
        self.shard_updates = 0   # in-place shard segment rewrites
        self.row_updates = 0     # ... of which only the changed rows were re-sent
        self.device_writes = 0   # ... of which write batches were merged on the GPU (K11/K12)
        self.device_write_launches = 0   # ... in this many merge/emit launches (all shards of a refresh share them)
        self.device_writes_on = os.environ.get("PILOSA_DEVICE_WRITES", "1") != "0"
        # cold views load from their fragment files (no host bitmaps)
        self.file_loader = os.environ.get("PILOSA_FILE_LOADER", "1") != "0"
        self.cold_loads = 0
        self.last_load: Dict = {}
        self.plan_threads = int(os.environ.get("PILOSA_PLAN_THREADS", "4"))
        self.topn_index_enabled = os.environ.get("PILOSA_TOPN_INDEX", "1") != "0"
        self._topn_indexes: Dict[Tuple, Tuple] = {}  # (index, field, shards) -> (rank caches, index, built_at)
        self._rank_cache_map: Dict[Tuple, Tuple] = {}  # (index, field, shards) -> (signature, DeviceRankCaches)
        # SPMD ranks of one node (parallel/collectives.Comm): TopN batches merge
        # their candidates / re-counts node-wide (every rank runs the same calls)
        self.comm = None
        self._spaces: Dict[Tuple, Tuple] = {}
        # (index, field, shards, nreq) -> (rank-cache serial, NodeCandidates or None):
        # node candidate spaces of mesh cache-only batches (refreshed collectively)
        self._cand_spaces: Dict[Tuple, Tuple] = {}
        # mesh plain cache-only TopN: (index, field, shard-set id, nreq) ->
        # (generation, rank-cache serial, fits, space, NodeCandidates, ids)
        self._plain_cands: Dict[Tuple, Tuple] = {}
        self.topn_mesh_fused = 0        # mesh cache-only groups answered in one all-reduce
        self._frag_lists: Dict[Tuple, Tuple] = {}   # (index, field, shards) -> (epoch, fragments)
        self.topn_decline = ""          # why the last topn_batch returned None (diagnostics)
        self._topn_index_why = ""

    # ------------------------------------------------------------ arenas
    def view_arena(self, index: str, field: str, view: str, shards: Sequence[int]) -> Optional[DeviceView]:
        # (a per-element int() over ~1k shards cost ~60 us per call on the
        # serving path; shard ids are ints already, numpy ints hash equal)
        shards = shards if type(shards) is tuple else tuple(shards)
        key = (index, field, view, shards)
        epoch = mutation_epoch()
        with self.mu:
            # nothing mutated since this arena was last validated: skip the
            # per-shard version signature (the serving hot path)
            if self._arena_epoch.get(key) == epoch:
                hit = self._arenas.get(key)
                if hit is not None:
                    self._arenas.move_to_end(key)
                    return hit[1]
        v = self.holder.view(index, field, view)
        if v is None:
            return None
        frags = _device_frags(v, shards)
        sig = tuple((_fid(f), f.version) if f is not None else None for f in frags)
        with self.mu:
            self._arena_epoch[key] = epoch
            hit = self._arenas.get(key)
            if hit is not None:
                self._arenas.move_to_end(key)
            if hit is not None and hit[0] == sig:
                return hit[1]
            if hit is not None and len(hit[0]) == len(sig) and hit[1].needs_compaction():
                hit[1].compact()   # on the device; a view that cannot be compacted is rebuilt below
            if hit is not None and len(hit[0]) == len(sig) and not hit[1].needs_compaction():
                # only some shards changed: rewrite their segments in place
                dv = hit[1]
                ok = True
                # Ordered write batches are replayed on the device FIRST (K11/K12, all
                # shards in shared launches; only the batches cross PCIe), THEN rows and
                # container keys that only the storage can describe (ClearRow, Store,
                # mutex/bool vectors, ...) are rebuilt from the current storage.  A batch
                # recorded before such a row change is therefore overwritten by the row's
                # current state instead of being re-applied on top of it.
                pending = {}   # si -> write batches for the device
                rebuild = {}   # si -> (rows, container keys) rebuilt from the storage afterwards
                whole = []     # shards whose change is unknown: full segment rewrite
                for si, (old, new, f) in enumerate(zip(hit[0], sig, frags)):
                    if old == new:
                        continue
                    if f is None:
                        ok = False
                        break
                    with f.mu:
                        dirty = f.take_dirty(dv.token) if old is not None and old[0] == _fid(f) else None
                    if dirty is None:
                        whole.append(si)
                        continue
                    rows, keys, deltas = dirty
                    if deltas and self.device_writes_on and dv.device.type == "cuda":
                        pending[si] = deltas
                    elif deltas:
                        keys = set(keys) | _delta_keys(deltas)
                    rebuild[si] = (rows, keys)
                if ok and pending:
                    wl0 = dv.write_launches
                    failed = dv.apply_deltas_multi(pending)
                    self.device_writes += len(pending) - len(failed)
                    self.device_write_launches += dv.write_launches - wl0
                    for si in failed:   # the host rebuilds what the device could not take
                        rows, keys = rebuild[si]
                        rebuild[si] = (rows, set(keys) | _delta_keys(pending[si]))
                for si in sorted(rebuild) if ok else ():
                    rows, keys = rebuild[si]
                    if rows or keys:
                        f = frags[si]
                        with f.mu:
                            good = dv.update_rows(si, rows, f.storage, keys=keys)
                        self.row_updates += good
                        if not good:
                            whole.append(si)
                            continue
                    self.shard_updates += 1
                for si in sorted(set(whole)) if ok else ():
                    f = frags[si]
                    with f.mu:
                        f.take_dirty(dv.token)
                        ok = dv.update_shard(si, _dev_storage(f))
                    if not ok:
                        break
                    self.shard_updates += 1
                if ok:
                    self._arenas[key] = (sig, dv)
                    return dv
            if hit is not None:
                for f in frags:
                    if f is not None:
                        f.drop_dirty(hit[1].token)
            token = object()  # dirty-row subscription of the new arena
            self._evict_for(key)
            dshards = shardwidth.device_shards(shards)
            with tracing.span("GpuExecutor.loadView", gpu=True, field=field, view=view, shards=len(shards)):
                dv = self._load_cold(frags, dshards, token, key) if self.file_loader else None
            if dv is None:
                bms = []
                for f in frags:
                    if f is None:
                        bms.append(None)
                    else:
                        with f.mu:
                            f.take_dirty(token)  # register before the contents are read
                            # a copy taken under the fragment lock: the native
                            # builder reads the bitmaps with no lock held, and a
                            # snapshot's to_bytes() optimises containers in place
                            # (a concurrent rewrite crashed the builder)
                            st = _dev_storage(f)
                            bms.append(st if isinstance(f, SubFragment) or not hasattr(st, "clone") else st.clone())
                dv = DeviceView.from_bitmaps(bms, self.device, shards=dshards, patchable=True)
            dv.token = token
            self.rebuilds += 1
            self._arenas[key] = (sig, dv)
            self._arenas.move_to_end(key)
            self._evict_for(key)
            return dv

    def _load_cold(self, frags, shards, token, key) -> Optional[DeviceView]:
        """Arena straight from the fragment files when every fragment of the
        view is still cold (never read on the host since open): the files are
        then exactly the fragments' state (ops/loader.py).  Writers are held
        off while the files are read; the dirty-row subscription is registered
        first, so writes after the load patch the arena as usual."""
        import contextlib

        from .loader import load_view
        live = [f for f in frags if f is not None]
        if not live or not all(f.is_cold() for f in live):
            return None
        with contextlib.ExitStack() as st:
            for f in live:
                st.enter_context(f.mu)
            if not all(f.is_cold() for f in live):
                return None
            for f in live:
                f.take_dirty(token)
            info: Dict = {}
            subs = [f.sub if f is not None else 0 for f in frags] if shardwidth.WIDE else None
            dv = load_view([f.path if f is not None else "" for f in frags], shards, self.device, patchable=True,
                           stats=info, subs=subs)
        self.cold_loads += 1
        self.last_load = dict(info, view=list(key[:3]))
        return dv

    def _evict_for(self, keep):
        """Drop least recently used arenas while over the HBM budget."""
        if self.hbm_budget <= 0:
            return
        while len(self._arenas) > 1 and self.hbm_bytes() > self.hbm_budget:
            k = next(iter(self._arenas))
            if k == keep:
                break
            _, dv = self._arenas.pop(k)
            self._drop_subscriptions(k, dv)
            self.evictions += 1

    def _drop_subscriptions(self, key, dv):
        v = self.holder.view(key[0], key[1], key[2])
        if v is None or getattr(dv, "token", None) is None:
            return
        for f in _device_frags(v, key[3]):
            if f is not None:
                f.drop_dirty(dv.token)

    def stats(self) -> dict:
        """Device gauges: resident bytes, containers by type."""
        with self.mu:
            views = [dv for _, dv in self._arenas.values()]
        types = {"array": 0, "bitmap": 0, "run": 0}
        for dv in views:
            t = ((dv.t_meta >> 4) & 3)
            for name, code in (("array", 1), ("bitmap", 2), ("run", 3)):
                types[name] += int((t == code).sum())
        return {"arenas": len(views), "arenaBytes": self.hbm_bytes(), "containers": types,
                "launches": self.launches, "rebuilds": self.rebuilds, "shardUpdates": self.shard_updates,
                "rowUpdates": self.row_updates, "deviceWrites": self.device_writes,
                "deviceWriteLaunches": self.device_write_launches, "evictions": self.evictions, "hbmBudget": self.hbm_budget}

    def invalidate(self):
        with self.mu:
            self._arenas.clear()
            self._arena_epoch.clear()
            self._bsi_views.clear()
            self._topn_indexes.clear()
            self._rank_cache_map.clear()
            self._frag_lists.clear()

    BSI_CACHE = 8

    def _bsi_count(self, index: str, c: Call, shards: Sequence[int]) -> Optional[int]:
        """Count(Row(v <op> x)) in one fused predicate+count launch."""
        n = self._bsi_count_async(index, c, shards)
        if n is None or isinstance(n, int):
            return n
        return int(self.engine.to_host(n)[0])

    def _bsi_count_async(self, index: str, c: Call, shards: Sequence[int]):
        """The fused count launched: device int64[1], an int when known
        without a launch, None for the plain (NOT NULL) path."""
        f, b, kind, args = self._ex().bsi_predicate(index, c)
        if kind == "empty":
            return 0
        if kind == "notnull":
            return None  # the exists row: plain Count(Row) path
        bv = self.view_arena(index, f.name, VIEW_BSI_PREFIX + f.name, shards)
        if bv is None:
            return 0
        if kind == "between":
            op, p1, p2 = "between", int(args[0]), int(args[1])
        else:
            op, p1, p2 = args[0], int(args[1]), 0
        self.launches += 1
        return self.engine.bsi_range_count_async(bv, b.bit_depth, op, p1, p2)

    def bsi_leaf(self, index: str, c: Call, shards: Sequence[int]):
        """Row(v <op> x) -> Leaf over a device-evaluated predicate view
        (bsi_range_kernel); NOT NULL uses the exists row directly."""
        f, b, kind, args = self._ex().bsi_predicate(index, c)
        if kind == "empty":
            return EMPTY
        bv = self.view_arena(index, f.name, VIEW_BSI_PREFIX + f.name, shards)
        if bv is None:
            return EMPTY
        if kind == "notnull":
            return Leaf(bv, 0)
        if kind == "between":
            op, p1, p2 = "between", int(args[0]), int(args[1])
        else:
            op, p1, p2 = args[0], int(args[1]), 0
        key = (id(bv), bv.generation, op, p1, p2, b.bit_depth)
        with self.mu:
            rv = self._bsi_views.get(key)
            if rv is None:
                self.launches += 1
                rv = self.engine.bsi_range_view(bv, b.bit_depth, op, p1, p2)
                rv._src = bv  # keep the source arena alive while cached (id() key)
                if len(self._bsi_views) >= self.BSI_CACHE:
                    self._bsi_views.pop(next(iter(self._bsi_views)))
                self._bsi_views[key] = rv
        return Leaf(rv, 0)

    def bsi_minmax(self, index: str, c: Call, shards: List[int], which: str):
        """Min/Max over the local shards -> ONE ValCount, folded vectorised
        exactly as the executor's per-shard reduce folds them in shard order
        (ValCount.smaller / larger keep the FIRST shard holding the extreme,
        with that shard's count: executor.go ValCount.Smaller).  Building and
        reducing ~1k per-shard objects in Python took most of the request."""
        from pilosa_amd.executor import ValCount
        fname = c.args.get("field")
        f = self.holder.field(index, fname) if isinstance(fname, str) else None
        if f is None or f.bsi_group(fname) is None or len(c.children) > 1:
            raise NotImplementedError
        b = f.bsi_group(fname)
        bv = self.view_arena(index, fname, VIEW_BSI_PREFIX + fname, shards)
        if bv is None:
            return ValCount()
        filt = None
        if len(c.children) == 1:
            filt = self.plan(index, c.children[0], shards)
            if filt is EMPTY:
                return ValCount()
        # per fragment (a wide one: all keys of its sub-shards, fragment.min/max
        # counts every column of the shard holding the value), then the first
        # fragment holding the extreme -- folded on the device, 3 int64 back
        sub = shardwidth.DEVICE_SUBSHARDS if shardwidth.WIDE else 1
        try:
            self.launches += 1
            v, n, found = self.engine.bsi_minmax_folded(filt, bv, b.bit_depth, which, sub)
        except CompileError:
            raise NotImplementedError
        if not found or n <= 0:
            return ValCount()
        return ValCount(v + b.base, n)

    def hbm_bytes(self) -> int:
        with self.mu:
            return sum(dv.nbytes() for _, dv in self._arenas.values())

    # ------------------------------------------------------------ planning
    def _ex(self):
        if self.executor is None:
            raise NotImplementedError
        return self.executor

    def plan(self, index: str, c: Call, shards: Sequence[int]):
        """PQL bitmap call -> Leaf/Op tree (or EMPTY)."""
        n = c.name
        if n in ("Row", "Range", "Bitmap"):
            if c.has_condition_arg():
                return self.bsi_leaf(index, c, shards)
            try:
                fname = c.field_arg()
            except ValueError:
                raise NotImplementedError
            f = self.holder.field(index, fname)
            if f is None:
                raise NotImplementedError  # host path raises the proper error
            rid, ok = c.uint_arg(fname)
            if not ok:
                raise NotImplementedError
            views = self._ex().time_views(f, c)
            if views is None:
                views = [VIEW_STANDARD]
            leaves = []
            for vname in views:
                dv = self.view_arena(index, fname, vname, shards)
                if dv is not None:
                    leaves.append(Leaf(dv, rid))
            if not leaves:
                return EMPTY
            return leaves[0] if len(leaves) == 1 else Op("or", tuple(leaves))
        if n in ("Intersect", "Union", "Difference", "Xor"):
            if not c.children:
                if n == "Union":
                    return EMPTY
                raise NotImplementedError
            kids = [self.plan(index, k, shards) for k in c.children]
            if n == "Intersect":
                if any(k is EMPTY for k in kids):
                    return EMPTY
                return kids[0] if len(kids) == 1 else Op("and", tuple(kids))
            if n == "Union":
                kids = [k for k in kids if k is not EMPTY]
                if not kids:
                    return EMPTY
                return kids[0] if len(kids) == 1 else Op("or", tuple(kids))
            if n == "Difference":
                if kids[0] is EMPTY:
                    return EMPTY
                rest = [k for k in kids[1:] if k is not EMPTY]
                return kids[0] if not rest else Op("andnot", (kids[0], *rest))
            kids = [k for k in kids if k is not EMPTY]  # Xor
            if not kids:
                return EMPTY
            return kids[0] if len(kids) == 1 else Op("xor", tuple(kids))
        if n == "Shift":
            k, _ = c.int_arg("n")
            if len(c.children) != 1 or k < 0:
                raise NotImplementedError  # the host path raises the proper error
            child = self.plan(index, c.children[0], shards)
            if k == 0 or child is EMPTY:
                return child
            # the total shift of a nested chain: its bits reach at most one
            # shard further (one spill level), as long as it stays below the
            # shard width (roaring.go:944-977 carries one container at a time)
            prior = _shift_total(child)
            if k + prior >= SHARD_WIDTH:
                raise NotImplementedError   # carries across several shards: host path
            try:
                if prior:
                    # Shift(Shift(..)): the child's in-shard part shifts and
                    # carries; its spill (already the next shard's bits) shifts
                    # within that shard; the new spill is their union
                    self.launches += 2
                    main, spill = self.engine.shift_views(child, k)
                    se = spill_expr(child)
                    if se is not EMPTY:
                        self.launches += 3
                        moved, _ = self.engine.shift_views(se, k)
                        spill = self.engine.dense_view(Op("or", (Leaf(spill, 0), Leaf(moved, 0))))
                else:
                    self.launches += 2
                    main, spill = self.engine.shift_views(child, k)
            except CompileError:
                raise NotImplementedError
            main._spill = spill
            main._shift_total = prior + k
            return Leaf(main, 0)
        if n == "Not":
            idx = self.holder.index(index)
            if idx is None or idx.existence_field() is None or len(c.children) != 1:
                raise NotImplementedError
            ex = self.view_arena(index, EXISTENCE_FIELD_NAME, VIEW_STANDARD, shards)
            child = self.plan(index, c.children[0], shards)
            if ex is None:
                return EMPTY
            if child is EMPTY:
                return Leaf(ex, 0)
            return Op("andnot", (Leaf(ex, 0), child))
        raise NotImplementedError(n)

    # ------------------------------------------------------------ calls
    def count(self, index: str, child: Call, shards: List[int]) -> int:
        if child.name in ("Row", "Range") and child.has_condition_arg():
            n = self._bsi_count(index, child, shards)
            if n is not None:
                return n
        e = self.plan(index, child, shards)
        if e is EMPTY:
            return 0
        exprs = [e]
        if _has_shift(e):
            se = spill_expr(e)
            if se is not EMPTY:
                exprs.append(se)
        try:
            self.launches += 1
            return int(self.engine.count(exprs).sum())
        except CompileError:
            raise NotImplementedError

    NATIVE_BATCH_MIN = 4

    def _native_fields(self, index: str) -> List[str]:
        """Fields whose ``Row(f=id)`` reads exactly the standard view (set,
        mutex, bool and time fields; BSI fields are excluded)."""
        from pilosa_amd.models.field import FIELD_TYPE_INT
        idx = self.holder.index(index)
        if idx is None:
            return []
        return [f.name for f in idx.fields.values() if f.type != FIELD_TYPE_INT and f.name != EXISTENCE_FIELD_NAME]

    def _count_batch_native(self, index: str, calls: List[Call], shards: List[int]) -> Optional[List[int]]:
        """Serving fast path: the calls' canonical PQL goes through the native
        program compiler (pilosa_amd/native/pql_compile.cpp, ~0.3 us/query)
        instead of Python planning; any call outside its subset is compiled by
        the planner against the same views, anything else returns None."""
        from .planner import NativeCountCompiler, Unsupported
        views: Dict[str, DeviceView] = {}
        for f in self._native_fields(index):
            dv = self.view_arena(index, f, VIEW_STANDARD, shards)
            if dv is not None:
                views[f] = dv
        if not views:
            return None
        comp = NativeCountCompiler(views)
        try:
            progs, vlist, S = comp.compile([str(c) for c in calls])
        except (Unsupported, KeyError, ValueError):
            return None
        if comp.fallbacks:
            return None  # rows missing from every arena (EMPTY) etc.: planner path
        self.launches += 1
        return self.engine.to_host(self.engine.launch_count(self.engine.prepare_progs(progs, vlist, S))).tolist()

    def try_count_text(self, index: str, text: str, shards: List[int], device_out: bool = False):
        """A whole request of ``Count(<Row/set-op tree>)`` calls, compiled from
        the PQL text natively (no Python AST) into one launch.  None when any
        call, field or view needs the general executor path (keys, BSI and
        time-range leaves, unknown fields, ...)."""
        from pilosa_amd import _pql
        from pilosa_amd.models.field import FIELD_TYPE_INT
        t0 = time.perf_counter()
        idx = self.holder.index(index)
        if idx is None or idx.keys:
            return None
        names = _pql.count_text_fields(text)
        views: Dict[str, DeviceView] = {}
        for name in names:
            f = idx.field(name)
            if f is None or f.type == FIELD_TYPE_INT or f.options.keys or name == EXISTENCE_FIELD_NAME:
                return None
            dv = self.view_arena(index, name, VIEW_STANDARD, shards)
            if dv is None:
                return None
            views[name] = dv
        vlist = list(views.values())
        fields = {n: i for i, n in enumerate(views)}
        ranges = self._text_ranges(idx, index, text, shards, vlist) if ("from" in text or "to" in text) else {}
        if ranges is None or not vlist:
            return None
        eng = self.engine
        use_and2 = eng.use_and2 and max(v.container_count for v in vlist) < 0xFFFFFFFF
        # rows absent from a view compile to dense -1 (empty leaf)
        with tracing.span("GpuExecutor.planCountText"):
            got = _pql.plan_count_text(text, fields, [v.rows for v in vlist], use_and2, eng.use_union,
                                       self.plan_threads, ranges)
        if got is None:
            return None
        Q, segs, buf = got
        self.launches += 1
        out = eng.launch_count(eng.prepare_planned(Q, segs, buf, vlist, vlist[0].S))
        # device_out: the int64[Q] device tensor, still being computed (the
        # caller reduces it on the device, e.g. the mesh all-reduce)
        if device_out:
            return out
        t1 = time.perf_counter()
        res = eng.to_host(out).tolist()
        self.text_batches += 1
        self.text_prep_s += t1 - t0
        self.text_wait_s += time.perf_counter() - t1
        return res

    def _text_ranges(self, idx, index: str, text: str, shards: List[int], vlist: List[DeviceView]):
        """The time-range Row(t=<id>, from=, to=) leaves of a request text
        (native scan), each resolved to the slots of its covering views'
        arenas, which are appended to ``vlist`` (executor time_views ->
        views_by_time_range, time.go:104-181).  {range key: [slots]} for
        plan_count_text, or None when a range needs the general path."""
        from pilosa_amd import _pql
        from pilosa_amd.models.field import FIELD_TYPE_TIME
        from pilosa_amd.pql.ast import Call
        out: Dict[str, List[int]] = {}
        slot_of: Dict[Tuple[str, str], int] = {}
        ex = self._ex()
        for fname, fr, to in _pql.count_text_ranges(text):
            f = idx.field(fname)
            if f is None or f.type != FIELD_TYPE_TIME or f.options.keys:
                return None
            args = {k: v for k, v in (("from", fr), ("to", to)) if v is not None}
            try:
                vnames = ex.time_views(f, Call("Row", args))
            except Exception:  # noqa: BLE001 - malformed times: the general path reports them
                return None
            if not vnames:
                return None
            slots = []
            for v in vnames:
                if (fname, v) not in slot_of:
                    dv = self.view_arena(index, fname, v, shards)
                    if dv is None:
                        continue
                    slot_of[(fname, v)] = len(vlist)
                    vlist.append(dv)
                slots.append(slot_of[(fname, v)])
            if not slots:
                return None
            out[f"{fname}\x1f{chr(1) if fr is None else fr}\x1f{chr(1) if to is None else to}"] = slots
        return out

    TIME_GROUP_MIN = 2

    def _count_time_rows(self, index: str, calls: List[Call], shards: List[int]) -> Dict[int, int]:
        """Count(Row(t=r, from=, to=)) calls of a batch that share (field,
        from, to): one union program per call built vectorised
        (GpuEngine.union_programs over the covering views' dense rows) and
        one launch per group, instead of a Leaf/Op tree and compile_expr per
        call.  Returns {call index: count}; calls it does not take (other
        shapes, small groups, > 16 covering views) are left to the caller."""
        from .device import MAXLEAF
        idx = self.holder.index(index)
        if idx is None:
            return {}
        groups: Dict[Tuple, List[Tuple[int, int]]] = {}
        for i, c in enumerate(calls):
            if len(c.children) != 1:
                continue
            ch = c.children[0]
            if ch.name != "Row" or ch.children or ch.has_condition_arg() or "from" not in ch.args and "to" not in ch.args:
                continue
            try:
                fname = ch.field_arg()
                rid, ok = ch.uint_arg(fname)
            except ValueError:
                continue
            if not ok or idx.field(fname) is None:
                continue
            groups.setdefault((fname, str(ch.args.get("from")), str(ch.args.get("to"))), []).append((i, rid, ch))
        out: Dict[int, int] = {}
        for (fname, _, _), members in groups.items():
            if len(members) < self.TIME_GROUP_MIN:
                continue
            try:
                vnames = self._ex().time_views(idx.field(fname), members[0][2])
            except Exception:  # noqa: BLE001 - malformed times: the general path reports them
                continue
            if vnames is None:
                continue
            dvs = [dv for dv in (self.view_arena(index, fname, v, shards) for v in vnames) if dv is not None]
            if not dvs:
                for i, _, _ in members:
                    out[i] = 0
                continue
            if len(dvs) > MAXLEAF or len({dv.S for dv in dvs}) != 1:
                continue
            rows = np.array([rid for _, rid, _ in members], dtype=np.uint64)
            progs = GpuEngine.union_programs(np.stack([dv.dense_many(rows) for dv in dvs], axis=1))
            self.launches += 1
            got = self.engine.to_host(self.engine.launch_count(self.engine.prepare_progs(progs, dvs, dvs[0].S))).tolist()
            for (i, _, _), v in zip(members, got):
                out[i] = int(v)
        return out

    def try_count_batch(self, index: str, calls: List[Call], shards: List[int]) -> Optional[List[int]]:
        """Many Count() calls of one request -> one launch; calls whose tree
        does not fit the kernel limits are counted on the host.  Time-range
        Row counts sharing a range take the vectorised union path first."""
        done = self._count_time_rows(index, calls, shards) if len(calls) >= self.TIME_GROUP_MIN else {}
        if not done:
            return self._try_count_batch_plain(index, calls, shards)
        rest = [i for i in range(len(calls)) if i not in done]
        out = [0] * len(calls)
        for i, v in done.items():
            out[i] = v
        if rest:
            got = self._try_count_batch_plain(index, [calls[i] for i in rest], shards)
            if got is None:
                return None
            for i, v in zip(rest, got):
                out[i] = v
        return out

    def _try_count_batch_plain(self, index: str, calls: List[Call], shards: List[int]) -> Optional[List[int]]:
        from .device import compile_expr
        if len(calls) >= self.NATIVE_BATCH_MIN:
            got = self._count_batch_native(index, calls, shards)
            if got is not None:
                return got
        # Count(Row(v <op> x)) calls: the fused predicate+count kernel each
        # (no predicate view written and re-read), one D2H for all of them
        fused: Dict[int, object] = {}
        try:
            exprs = []
            for i, c in enumerate(calls):
                if len(c.children) != 1:
                    return None
                ch = c.children[0]
                if ch.name in ("Row", "Range") and ch.has_condition_arg():
                    n = self._bsi_count_async(index, ch, shards)
                    if n is not None:
                        fused[i] = n
                        exprs.append(EMPTY)
                        continue
                exprs.append(self.plan(index, ch, shards))
        except NotImplementedError:
            return None
        out = [0] * len(exprs)
        if fused:
            dev = [(i, t) for i, t in fused.items() if not isinstance(t, int)]
            for i, t in fused.items():
                if isinstance(t, int):
                    out[i] = t
            if dev:
                got = self.engine.to_host(self.engine.torch.cat([t for _, t in dev])).tolist()
                for (i, _), v in zip(dev, got):
                    out[i] = int(v)
        live = []
        for i, e in enumerate(exprs):
            if e is EMPTY:
                continue
            try:
                compile_expr(e, {})
                live.append(i)
            except CompileError:
                out[i] = self._ex().count_host(index, calls[i].children[0], shards)
        if live:
            self.launches += 1
            extra = [(i, spill_expr(exprs[i])) for i in live if _has_shift(exprs[i])]
            extra = [(i, se) for i, se in extra if se is not EMPTY]
            got = self.engine.count([exprs[i] for i in live] + [se for _, se in extra])
            for i, v in zip(live, got[:len(live)]):
                out[i] = int(v)
            for (i, _), v in zip(extra, got[len(live):]):
                out[i] += int(v)
        return out

    def bitmap(self, index: str, c: Call, shards: List[int]) -> Row:
        blk = self.bitmap_block(index, c, shards)
        if blk is None:
            return Row()
        c_, o, pay = blk.host()
        spill = ([], [])
        if blk.spill is not None:
            sc, so, sp = blk.spill.host()
            spill = (self.engine.block_bitmaps(blk.spill.shards, sc, so, sp), blk.spill.shards)
        return row_from_bitmaps(self.engine.block_bitmaps(blk.shards, c_, o, pay), blk.shards, *spill)

    def bitmap_block(self, index: str, c: Call, shards: List[int]):
        """The call's result containers left on the device (DeviceRowBlock,
        spill block attached for Shift), None when empty."""
        e = self.plan(index, c, shards)
        if e is EMPTY:
            return None
        try:
            self.launches += 1
            blk = self.engine.materialize_block(e)
            if blk is not None and _has_shift(e):
                se = spill_expr(e)
                if se is not EMPTY:
                    self.launches += 1
                    blk.spill = self.engine.materialize_block(se)
        except CompileError:
            raise NotImplementedError
        return blk

    def rows(self, index: str, fname: str, c: Call, shards: List[int]) -> List[int]:
        """Rows(field, previous=, column=, limit=, from=, to=) over the local
        shards in one rows_kernel launch per view (fragment.go:2601-2712)."""
        from pilosa_amd.executor import MAX_INT
        if self.holder.index(index) is None:
            raise NotImplementedError
        f = self.holder.field(index, fname)
        if f is None:
            raise NotImplementedError  # host path raises the proper error
        prev, has_prev = c.uint_arg("previous")
        start = prev + 1 if has_prev else 0
        col, has_col = c.uint_arg("column")
        lim, has_lim = c.uint_arg("limit")
        limit = lim if has_lim else MAX_INT
        if has_col and col // SHARD_WIDTH not in shards:
            return []
        ids = np.zeros(0, np.uint64)
        for vname in self._ex().rows_views(f, c):
            dv = self.view_arena(index, fname, vname, shards)
            if dv is None:
                continue
            self.launches += 1
            ids = np.union1d(ids, self.engine.row_ids(dv, col if has_col else None))
        ids = ids[ids >= np.uint64(start)]
        return [int(x) for x in ids[:limit]]

    MINMAX_ROW_CHUNK = 256

    def minmax_row(self, index: str, c: Call, shards: List[int], is_min: bool) -> Pair:
        """MinRow/MaxRow(field, [filter]) over the local shards (K16,
        fragment.go:1230-1268).  Unfiltered: each shard's first/last non-empty
        row from the arena's per-row cardinalities.  Filtered: rows are
        counted against the filter in growing chunks (ascending for MinRow,
        descending for MaxRow) with the pair kernels, all shards per launch,
        until every shard found its first row with a non-zero intersection.
        Per-shard pairs are folded in shard order with the reference's reduce
        (executor.go:517-548)."""
        import torch
        fname = c.args.get("field")
        if not isinstance(fname, str) or self.holder.field(index, fname) is None:
            raise NotImplementedError
        rv = self.view_arena(index, fname, VIEW_STANDARD, shards)
        if rv is None or rv.D == 0 or rv.S == 0:
            return Pair(0, 0)
        S, D = rv.S, rv.D
        rid = np.zeros(S, np.int64)
        cnt = np.zeros(S, np.int64)
        if len(c.children) != 1:
            self.launches += 1
            n = ((rv.t_meta >> 6) & 0x1FFFF).to(torch.int64)
            cs = torch.zeros(n.numel() + 1, dtype=torch.int64, device=rv.device)
            torch.cumsum(n, 0, out=cs[1:])
            rp = rv.t_rowptr.view(S, D + 1).to(torch.int64)
            sb = rv.t_shard_base.to(torch.int64)
            for s0 in range(0, S, 32):
                s1 = min(S, s0 + 32)
                idx = sb[s0:s1, None] + rp[s0:s1]
                nz = (cs[idx[:, 1:]] - cs[idx[:, :-1]]) > 0          # [c, D] row non-empty
                has = nz.any(dim=1)
                pos = nz.to(torch.int8).argmax(dim=1) if is_min else \
                    D - 1 - nz.flip(1).to(torch.int8).argmax(dim=1)
                h, p = has.cpu().numpy(), pos.cpu().numpy()
                rid[s0:s1] = np.where(h, rv.rows[p].astype(np.int64), 0)
                cnt[s0:s1] = h.astype(np.int64)
        else:
            filt = self.plan(index, c.children[0], shards)
            if filt is EMPTY:
                return Pair(0, 0)
            if type(filt) is Leaf and filt.view.S == S:
                fview, fdense = filt.view, filt.view.dense(filt.row)
                if fdense < 0:
                    return Pair(0, 0)
            else:
                try:
                    self.launches += 1
                    fview, fdense = self.engine.dense_view(filt), 0
                except CompileError:
                    raise NotImplementedError
            open_ = np.ones(S, bool)
            lo, chunk = 0, self.MINMAX_ROW_CHUNK
            while open_.any() and lo < D:
                hi = min(D, lo + chunk)
                dense = np.arange(lo, hi, dtype=np.int64) if is_min else np.arange(D - 1 - lo, D - 1 - hi, -1,
                                                                                   dtype=np.int64)
                progs = self.engine.pair_programs(0, fdense, 1, dense)
                self.launches += 1
                m = self.engine.count_per_shard_progs(progs, [fview, rv], S)   # [rows, S]
                hit = m > 0
                first = hit.argmax(axis=0)
                found = hit.any(axis=0) & open_
                rid[found] = rv.rows[dense[first[found]]].astype(np.int64)
                cnt[found] = m[first[found], np.nonzero(found)[0]]
                open_ &= ~found
                lo, chunk = hi, chunk * 4
        if shardwidth.WIDE:
            rid, cnt = _fold_subshards(rid, cnt, is_min, filtered=len(c.children) == 1)
        out = None
        for r, n_ in zip(rid.tolist(), cnt.tolist()):
            v = Pair(r, n_)
            if out is None:
                out = v
            elif out.count > 0 and v.count > 0:
                if is_min:
                    out = out if out.id < v.id else v
                else:
                    out = out if out.id > v.id else v
            elif out.count <= 0:
                out = v
        return out or Pair(0, 0)

    def bsi_sum(self, index: str, c: Call, shards: List[int]):
        import torch

        from pilosa_amd.executor import ValCount, _wrap
        fname = c.args.get("field")
        f = self.holder.field(index, fname) if isinstance(fname, str) else None
        if f is None or f.bsi_group(fname) is None:
            raise NotImplementedError
        b = f.bsi_group(fname)
        bv = self.view_arena(index, fname, VIEW_BSI_PREFIX + fname, shards)
        if bv is None:
            return ValCount()
        filt = None
        if len(c.children) == 1:
            filt = self.plan(index, c.children[0], shards)
            if filt is EMPTY:
                return ValCount()
        try:
            self.launches += 1
            s, n = self.engine.bsi_sum_async([filt], bv, b.bit_depth)
        except CompileError:
            raise NotImplementedError
        base = s._base if s._base is not None and s._base.numel() == 2 and n._base is s._base else None
        s, n = (int(x) for x in self.engine.to_host(base if base is not None else torch.stack([s[:1], n[:1]])).view(-1).tolist())
        return ValCount(_wrap(s + n * b.base), n)

    def bsi_sum_batch(self, index: str, calls: List[Call], shards: List[int]):
        """Many Sum(<filter>, field=v) calls of one request over one BSI field:
        the filters are planned together and summed in one launch -- the
        bit-plane count matrix on the matrix cores (ops/bsi.py) from
        BSI_MATRIX_MIN filters up, else the per-filter kernel with all filters
        in one grid.  None when a call needs the general path."""
        from pilosa_amd.executor import ValCount, _wrap

        from .bsi import BSI_MATRIX_MIN, bsi_sum_matrix
        fname = calls[0].args.get("field")
        if not isinstance(fname, str) or any(c.args.get("field") != fname or len(c.children) > 1 for c in calls):
            return None
        f = self.holder.field(index, fname)
        if f is None or f.bsi_group(fname) is None:
            return None
        b = f.bsi_group(fname)
        bv = self.view_arena(index, fname, VIEW_BSI_PREFIX + fname, shards)
        if bv is None:
            return [ValCount() for _ in calls]
        filters = []
        try:
            for c in calls:
                filters.append(self.plan(index, c.children[0], shards) if c.children else None)
        except NotImplementedError:
            return None
        live = [i for i, x in enumerate(filters) if x is not EMPTY]
        out = [ValCount() for _ in calls]
        if not live:
            return out
        fl = [filters[i] for i in live]
        try:
            self.launches += 1
            if len(fl) >= BSI_MATRIX_MIN:
                s_t, n_t = bsi_sum_matrix(self.engine, fl, bv, b.bit_depth)
            else:
                s_t, n_t = self.engine.bsi_sum_async(fl, bv, b.bit_depth)
        except CompileError:
            return None
        for i, sv, nv in zip(live, s_t.cpu().tolist(), n_t.cpu().tolist()):
            out[i] = ValCount(_wrap(int(sv) + int(nv) * b.base), int(nv))
        return out

    # ------------------------------------------------------------ TopN
    def _topn_setup(self, index: str, c: Call, shards: List[int]):
        """(params, rank caches, view, src plan, (tanimoto, attribute filter))
        of one TopN call, or NotImplementedError for the shapes the host
        answers (more than one child)."""
        ex = self._ex()
        fname, n, ids, threshold, tanimoto, attr_name, attr_values = ex.topn_params(index, c)
        if len(c.children) > 1:
            raise NotImplementedError
        frags = self._topn_frags(index, fname, shards)
        rv = self.view_arena(index, fname, VIEW_STANDARD, shards)
        src = self.plan(index, c.children[0], shards) if c.children else None
        rc = self._rank_caches(index, fname, shards, frags, rv) if rv is not None else None
        keep = None
        if attr_name and attr_values:
            # fragment.top's attribute filter (fragment.go:1586-1600): rows whose
            # attribute value is one of the listed ones
            from pilosa_amd.models.fragment import _hashable
            store = self.holder.field(index, fname).row_attr_store
            want = {_hashable(v) for v in attr_values}

            def keep(rid, store=store, want=want, name=attr_name):
                a = store.attrs(rid)
                return bool(a) and a.get(name) is not None and _hashable(a.get(name)) in want
        return (fname, n, ids, threshold), rc, rv, src, (tanimoto if src is not None else 0, keep)

    def topn(self, index: str, c: Call, shards: List[int]) -> List[Pair]:
        """One TopN call's map step over the local shards (executor.go:905-930):
        phase 1 = per-shard ``fragment.top`` results summed by row (untrimmed),
        with ``ids=`` the per-shard exact re-count of those rows."""
        (fname, n, ids, threshold), rc, rv, src, (tan, keep) = self._topn_setup(index, c, shards)
        if rc is None or src is EMPTY or rc.K == 0:
            return []
        if tan or keep is not None:
            # Tanimoto / attribute filters: device counts, the exact heap walk
            # with both filters replayed on the host (fragment.go:1568-1700)
            return self._topn_pairs_path(rc, rv, src, n, ids, threshold, tan=tan, keep=keep)
        if src is None:
            self.launches += 1
            return rc.shard_pairs_nosrc(0 if ids else n, threshold, ids or None)
        tix = self._topn_index(index, fname, shards, rc, rv)
        if tix is not None:
            self.launches += 1
            self.topn_index_batches += 1
            try:
                return sort_pairs(tix.shard_pairs(self.engine, src, 0 if ids else n, threshold, ids or None))
            except CompileError:
                raise NotImplementedError   # src too large for one device program: host path
        return self._topn_pairs_path(rc, rv, src, n, ids, threshold)

    def _plain_rc(self, index: str, fname: str, shards: List[int], key=None):
        """The field's standard view and rank caches over ``shards``, resolved
        once per mutation epoch (``key`` names the shard list: the mesh's
        shard-set id, so a 1k-shard list is not hashed per request)."""
        key = (index, fname, tuple(shards) if key is None else key)
        epoch = mutation_epoch()
        memo = self.__dict__.setdefault("_plain_memo", {})
        ent = memo.get(key)
        if ent is None or ent[0] != epoch:
            shards = list(shards)
            frags = self._topn_frags(index, fname, shards)
            rv = self.view_arena(index, fname, VIEW_STANDARD, shards)
            rc = self._rank_caches(index, fname, shards, frags, rv) if rv is not None else None
            if len(memo) > 64:
                memo.clear()
            ent = memo[key] = (epoch, rv, rc)
        return ent[1], ent[2]

    def topn_plain_batch(self, index: str, fname: str, ns: Sequence[int], ths: Sequence[int], shards: List[int],
                         skey=None):
        """Cache-only TopN(fname, n=ns[i], threshold=ths[i]) calls over the
        local shards in one fused batch (Executor._topn_plain_fast): the
        field's view and rank caches are resolved once per mutation epoch.
        ``skey`` names the shard list (else the list itself is the key)."""
        if self.comm is not None:
            return None
        rv, rc = self._plain_rc(index, fname, list(shards) if skey is None else shards, skey)
        if rc is None or not rc.K:
            return [[] for _ in ns]
        self.launches += 1
        with tracing.span("GpuExecutor.topnPlainBatch", gpu=True, calls=len(ns)):
            return rc.topn_nosrc(list(ns), list(ths))

    # ------------------------------------------------------------ mesh plain cache-only TopN
    # (parallel/mesh.py OP_TOPN_PLAIN / OP_TOPN_CAND).  A node candidate space
    # is built collectively (refresh_plain_cand, every rank, one generation
    # number from the front end); a batch is then ONE all-reduce whose buffer
    # size comes from the command, and each rank's vote on whether its space
    # is current rides in that buffer (topn_exec.mesh_cache_batch).

    def plain_cand_state(self, index: str, fname: str, shards: List[int], skey, nreq: int):
        """Front end, before issuing a batch, no collective: (generation, U,
        fused-path fits, bucket) of a current node candidate space that
        serves a batch needing the first ``nreq`` ranks -- that bucket's own,
        else the smallest built longer one (the membership kernel stops each
        call at its own n, so a longer prefix gives the same answers: a
        stream of varied n builds one space, as the 1-GPU memos do) -- or
        None when one must be built first."""
        try:
            rc = self._plain_rc(index, fname, shards, skey)[1] if shards else None
        except Exception:  # noqa: BLE001 - the refresh reports it node-wide
            return None
        serial = rc.serial if rc is not None else None
        best = None
        for (i2, f2, k2, b), ent in self._plain_cands.items():
            if i2 != index or f2 != fname or k2 != skey or ent[1] != serial:
                continue
            if b == nreq or (nreq != 0 and (b == 0 or b > nreq)):
                if best is None or (b != 0 and (best[3] == 0 or b < best[3])) or b == nreq:
                    best = (ent[0], len(ent[3]), ent[2], b)
                    if b == nreq:
                        break
        return best

    def refresh_plain_cand(self, index: str, fname: str, shards: List[int], skey, nreq: int, gen: int, comm):
        """Collective on every rank: all-gather each rank's local candidate
        rows of the (field, nreq) group, with its fragment and device-shard
        counts, and keep the node candidate space, this rank's tensors over
        it and whether the fused path fits on every rank (int32 node totals,
        the count-matrix cap) -- a node-wide decision.  Every rank takes part
        in the gather whatever fails locally."""
        import torch

        from .topn_exec import FUSED_MAX_CELLS
        rc = None
        rows = np.zeros(0, np.uint64)
        ok = True
        try:
            if shards:
                rc = self._plain_rc(index, fname, shards, skey)[1]
            if rc is not None:
                rows = rc.local_candidate_rows(nreq)
        except Exception:  # noqa: BLE001 - take part with nothing; the fit check fails below
            rc, ok = None, False
        head = np.array([rc.S if rc is not None else (0 if ok else -1),
                         rc.view.S if rc is not None else 0], np.int64)
        t = torch.from_numpy(np.concatenate([head, rows.view(np.int64)])).to(comm.device)
        parts = [p.cpu().numpy() for p in comm.all_gather_var(t)]
        space = np.unique(np.concatenate([p[2:].view(np.uint64) for p in parts])) if parts else rows
        s_frag = [int(p[0]) for p in parts]
        fits = bool(parts) and min(s_frag) >= 0 and len(space) * max(s_frag + [1]) <= FUSED_MAX_CELLS and \
            sum(int(p[1]) for p in parts) < 2048 and len(space) > 0
        cand = None
        if fits and rc is not None:
            try:
                cand = rc.node_candidates(nreq, space)
            except Exception:  # noqa: BLE001 - this rank then votes stale on every batch
                cand = None
        ids = torch.arange(len(space), dtype=torch.int32, device=comm.device) if fits else None
        if len(self._plain_cands) > 256:
            self._plain_cands.clear()
        self._plain_cands[(index, fname, skey, nreq)] = (int(gen), rc.serial if rc is not None else None, fits,
                                                         space, cand, ids)

    def topn_plain_mesh(self, index: str, fname: str, ns: Sequence[int], ths: Sequence[int], shards: List[int],
                        skey, nreq: int, gen: int, U: int, comm, defer: bool = True):
        """This rank's share of a mesh cache-only batch (every rank, the
        front end included): its partial over the node candidate space of
        generation ``gen`` (size ``U``, from the command) plus its vote, and
        the started all-reduce (topn_exec.mesh_cache_batch).  Never raises
        before the collective: a failure is a declined vote."""
        from .topn_exec import mesh_cache_batch
        rc = None
        ent = self._plain_cands.get((index, fname, skey, nreq))
        stale = declined = 0
        try:
            if shards:
                rc = self._plain_rc(index, fname, shards, skey)[1]
            if ent is None or ent[0] != int(gen) or ent[1] != (rc.serial if rc is not None else None) or \
                    len(ent[3]) != int(U) or not ent[2]:
                stale = 1
            elif rc is not None and ent[4] is None:
                stale = 1   # the space fits but this rank could not build its tensors
        except Exception:  # noqa: BLE001 - reported as a declined vote
            declined = 1
        space = ent[3] if ent is not None and not stale and not declined else None
        ids = ent[5] if ent is not None and not stale and not declined else None
        cand = ent[4] if space is not None else None
        self.launches += 1
        self.topn_mesh_fused += 1
        with tracing.span("GpuExecutor.topnPlainMesh", gpu=True, calls=len(ns)):
            return mesh_cache_batch(rc if cand is not None else None, ns, ths, comm, cand, int(U), stale=stale,
                                    declined=declined, defer=defer, device=self.device, space=space, ids=ids)

    def topn_batch(self, index: str, calls: List[Call], shards: List[int], defer: bool = False, cands=None):
        with tracing.span("GpuExecutor.topnBatch", gpu=True, calls=len(calls)):
            return self._topn_batch(index, calls, shards, defer, cands)

    def capture_cands(self, index: str, calls: List[Call], shards: List[int]) -> Dict[Tuple, Tuple]:
        """The node candidate-space entries of the batch's cache-only groups,
        taken right after the mesh vote: the batch then follows them (fused
        or not, and with which caches) whatever this rank's caches become
        meanwhile (a concurrent write on the front end could flip
        its choice and unpair the node's collectives)."""
        out = {}
        for fname, nreq in self._cand_groups(index, calls, shards):
            ent = self._cand_spaces.get((index, fname, tuple(shards), nreq))
            if ent is not None:
                out[(fname, nreq)] = ent
        return out

    def _topn_batch(self, index: str, calls: List[Call], shards: List[int], defer: bool = False, cands=None):
        """Whole TopN calls (phase 1, candidate union, ids= re-count, trim to
        n: executor.go:863-903) for a batch of calls over local shards, both
        phases on the device.  Calls of one (field, src shape) share launches:
        cache-only calls one scatter-add + one re-count, src calls the slot
        index (16 per hot-rank launch).  The per-field work (fragments, view,
        rank caches, slot index) is resolved once per batch.  None when a call
        needs the general path (the caller then runs each call alone).
        ``defer`` (with ``self.comm``): a pending result whose last
        collectives are still in flight (parallel/collectives.Pending)."""
        allp, finfo = self._batch_info(index, calls, shards)
        params = []
        for c, (fname, n, ids, threshold, tanimoto, attr_name, attr_values) in zip(calls, allp):
            if tanimoto or (attr_name and attr_values) or len(c.children) > 1:
                self.topn_decline = f"shape ({c})"
                return None
            if ids:
                self.topn_decline = "ids"
                return None   # explicit ids= (phase 2 only): the map-step path
            params.append((fname, n, threshold))
        fields = {f: (rv, rc) for f, (_, rv, rc) in finfo.items()}
        srcs = []
        try:
            for c in calls:
                srcs.append(self.plan(index, c.children[0], shards) if c.children else None)
        except NotImplementedError as e:
            self.topn_decline = f"src plan: {e!r}"
            return None
        groups: Dict[Tuple, List[int]] = {}
        for i, (fname, _, _) in enumerate(params):
            groups.setdefault((fname, srcs[i] is None), []).append(i)
        out: List[Optional[List[Pair]]] = [None] * len(calls)
        parts: List[Tuple[List[int], object]] = []
        for (fname, nosrc), members in groups.items():
            rv, rc = fields[fname]
            ent = None
            if nosrc and self.comm is not None and cands is not None:
                ent = cands.get((fname, _nreq([params[i][1] for i in members])))
                if ent is not None and not ent[2]:
                    ent = None      # the space did not fit on some rank: the node takes the union path
            if ent is not None:
                # fused mesh group: every rank takes part, with the captured caches
                live = list(members)
                ns = [params[i][1] for i in live]
                ths = [params[i][2] for i in live]
                self.launches += 1
                self.topn_mesh_fused += 1
                from .topn_exec import mesh_cache_batch
                e_rc, e_cand, _, e_space = ent[4], ent[1], ent[2], ent[3]
                got = mesh_cache_batch(e_rc if e_cand is not None else None, ns, ths, self.comm, e_cand,
                                       len(e_space), defer=defer, device=self.device, space=e_space,
                                       ids=e_cand.ids if e_cand is not None else ent[5])
                parts.append((live, got))
                continue
            live = [i for i in members if rc is not None and rc.K and srcs[i] is not EMPTY]
            for i in members:
                if i not in live:
                    out[i] = []
            if not live:
                continue
            ns = [params[i][1] for i in live]
            ths = [params[i][2] for i in live]
            space = self._node_space((index, fname, tuple(shards)), rv)
            if nosrc:
                self.launches += 1
                got = rc.topn_nosrc(ns, ths, comm=self.comm, space=space, defer=defer)
            else:
                tix = self._topn_index(index, fname, shards, rc, rv, space=space)
                if tix is None:
                    self.topn_decline = f"no slot index ({self._topn_index_why})"
                    return None
                self.launches += 1
                self.topn_index_batches += 1
                try:
                    got = tix.topn(self.engine, [srcs[i] for i in live], ns, ths, comm=self.comm, defer=defer)
                except CompileError:
                    self.topn_decline = "src too large for one device program"
                    return None
            parts.append((live, got))

        def fill(results):
            for (live, _), got in zip(parts, results):
                for i, r in zip(live, got):
                    out[i] = r
            return out
        if defer:
            from pilosa_amd.parallel.collectives import PendingAll
            return PendingAll([g for _, g in parts], fill)
        return fill([g for _, g in parts])

    def topn_batch_ready(self, index: str, calls: List[Call], shards: List[int]) -> bool:
        """Would :meth:`topn_batch` answer these calls on the device, with
        every call taking part in the batch's collectives?  Resolves (and
        builds) what it needs -- rank caches, slot index -- without any
        collective, so the ranks of a node can agree on the answer first
        (parallel/mesh.py OP_TOPN)."""
        if not shards:
            return False
        try:
            allp, finfo = self._batch_info(index, calls, shards)
            tsh = tuple(shards)
            for c, (fname, n, ids, threshold, tanimoto, attr_name, attr_values) in zip(calls, allp):
                if ids or tanimoto or (attr_name and attr_values) or len(c.children) > 1:
                    return False
                _, rv, rc = finfo[fname]
                if rv is None or rc is None or not rc.K:
                    return False
                if c.children:
                    src = self.plan(index, c.children[0], shards)
                    space = self._node_space((index, fname, tsh), rv)
                    if src is EMPTY or self._topn_index(index, fname, shards, rc, rv, space=space) is None:
                        return False
                    if not (type(src) is Leaf and src.view is rv):
                        self.engine.compile_batch([src])   # a src too large for one program declines here
        except (NotImplementedError, PilosaError, CompileError):
            return False
        return True

    def _topn_frags(self, index: str, fname: str, shards: List[int]):
        """The field's standard-view fragments of ``shards`` (cache type
        checked), memoised while no fragment is created, written or dropped
        (the mutation epoch): a TopN request over ~1k shards would otherwise
        spend a millisecond on holder lookups alone."""
        key = (index, fname, tuple(shards))
        epoch = mutation_epoch()
        ent = self._frag_lists.get(key)
        if ent is not None and ent[0] == epoch:
            return ent[1]
        frags = [self.holder.fragment(index, fname, VIEW_STANDARD, s) for s in shards]
        for f in frags:
            if f is not None and f.cache_type == "none":
                from pilosa_amd.errors import PilosaError
                raise PilosaError(f'cannot compute TopN(), field has no cache: "{fname}"')
        self._frag_lists[key] = (epoch, frags)
        return frags

    def _topn_pairs_path(self, rc, rv, src, n: int, ids, threshold: int, tan: int = 0, keep=None) -> List[Pair]:
        """Src TopN without a slot index (while it is rebuilt, or too large for
        LDS): each shard's fragment.top() walks its cache in order and stops
        once a row's cached count falls below the heap threshold, so usually
        only a short prefix of the candidates is ever counted.  Growing
        prefixes are counted on the device (one launch per round for all
        shards), the exact heap logic is replayed natively, and only the
        shards whose replay ran past what was counted are extended."""
        per_shard_pairs = []
        if ids:
            # topBitmapPairs(rowIDs): every listed row with its count in the shard
            want = sorted({int(x) for x in ids})
            cnt = rc.row_counts_for(want)                      # [S, P]
            for si in range(rc.S):
                pr = [(r, int(k)) for r, k in zip(want, cnt[si].tolist()) if k > 0]
                pr.sort(key=lambda p: (-p[1], p[0]))
                per_shard_pairs.append(pr)
        else:
            rows, counts = rc.host_lists()
            for si in range(rc.S):
                live = counts[si] > 0
                per_shard_pairs.append(list(zip(rows[si][live].tolist(), counts[si][live].tolist())))
        if src is None:
            # cache-only with an attribute filter: the cached counts are the counts
            self.launches += 1
            total: Dict[int, int] = {}
            for si in range(rc.S):
                for p in _replay_top(per_shard_pairs[si], None, 0 if ids else n, threshold, keep=keep):
                    total[p.id] = total.get(p.id, 0) + p.count
            return sort_pairs([Pair(k2, v) for k2, v in total.items()])
        src_counts = None
        if tan:
            self.launches += 1
            sc = self.engine.count_per_shard([src])[0]        # |src| per arena shard
            src_counts = sc.reshape(rc.S, rc.M).sum(axis=1) if rc.M > 1 else sc
        counted: Dict[int, np.ndarray] = {}
        depth = [0] * rc.S
        k = max(256, 2 * n) if not ids else max((len(p) for p in per_shard_pairs), default=0)
        pending = list(range(rc.S))
        total: Dict[int, int] = {}
        while pending:
            want = set()
            for si in pending:
                depth[si] = min(len(per_shard_pairs[si]), max(depth[si] * 4, k))
                want.update(rid for rid, _ in per_shard_pairs[si][:depth[si]] if rid not in counted)
            if want:
                rws = sorted(want)
                exprs = [Op("and", (src, Leaf(rv, r))) for r in rws]
                try:
                    for i in range(0, len(exprs), MAX_GROUPS_PER_LAUNCH):
                        self.launches += 1
                        m = self.engine.count_per_shard(exprs[i:i + MAX_GROUPS_PER_LAUNCH])  # [R, arena shards]
                        if rc.M > 1:   # per fragment: the sum over its sub-shards
                            m = m.reshape(len(m), rc.S, rc.M).sum(axis=2)
                        for r, row_counts in zip(rws[i:i + MAX_GROUPS_PER_LAUNCH], m):
                            counted[r] = row_counts
                except CompileError:
                    raise NotImplementedError
            nxt = []
            for si in pending:
                try:
                    got = _replay_top(per_shard_pairs[si], lambda rid, si=si: _counted(counted, rid, si),
                                      0 if ids else n, threshold, tan=tan,
                                      src_count=int(src_counts[si]) if src_counts is not None else 0, keep=keep)
                except _NeedMore:
                    nxt.append(si)
                    continue
                for p in got:
                    total[p.id] = total.get(p.id, 0) + p.count
            pending = nxt
        return sort_pairs([Pair(k2, v) for k2, v in total.items()])

    def _rank_caches(self, index: str, fname: str, shards: List[int], frags, rv):
        """Device rank caches of the view (ops/topn_exec.py), rebuilt when the
        arena changes or a warm fragment's host cache re-ranks.  Cold
        fragments contribute their .cache file ids (never loaded on the host);
        warm ones their live host caches (recalculated as topBitmapPairs does
        with cache.Invalidate, at most every 10 s)."""
        from .topn_exec import DeviceRankCaches
        key = (index, fname, tuple(shards))
        epoch = mutation_epoch()
        with self.mu:
            ent = self._rank_cache_map.get(key)
            if ent is not None and ent[2] == epoch and ent[1].view is rv and ent[1].generation == rv.generation:
                return ent[1]
        sig = []
        for f in frags:
            if f is None:
                sig.append(None)
            elif f.is_cold() and not f.cache_is_live():
                sig.append(("cold", id(f)))
            else:
                with f.mu:   # writers update the rank cache under f.mu (fragment.go:1709-1712)
                    f.cache.invalidate()
                    sig.append(("warm", id(f), getattr(f.cache, "version", -1)))
        sig = (id(rv), rv.generation, tuple(sig))
        with self.mu:
            ent = self._rank_cache_map.get(key)
            if ent is not None and ent[0] == sig:
                self._rank_cache_map[key] = (sig, ent[1], epoch)
                return ent[1]
        rc = DeviceRankCaches(rv, frags)
        with self.mu:
            self._rank_cache_map[key] = (sig, rc, epoch)
        return rc

    def _node_space(self, key, rv) -> Optional[np.ndarray]:
        """Sorted union of every rank's row ids of this view (the common space
        of the node-wide TopN candidates), or None on a single rank.  Never
        runs a collective: the mesh refreshes the spaces of a TopN batch
        collectively first (:meth:`node_space_stale` on every rank, one
        all-reduced vote, then :meth:`refresh_node_spaces` on every rank), so
        a write that moved only one rank's view cannot make the ranks pair
        different collectives."""
        if self.comm is None or rv is None:
            return None
        ent = self._spaces.get(key)
        if ent is None:
            raise NotImplementedError("node row space not gathered (mesh refresh missing)")
        return ent[1]

    def node_space_stale(self, index: str, fname: str, shards: List[int]) -> bool:
        """Does this rank's copy of the node row space of (index, fname) miss
        changes of its own view?  Local check only (see :meth:`_node_space`)."""
        key = (index, fname, tuple(shards))
        rv = self.view_arena(index, fname, VIEW_STANDARD, shards) if shards else None
        sig = (id(rv), rv.rows_gen) if rv is not None else None
        ent = self._spaces.get(key)
        return ent is None or ent[0] != sig

    def refresh_node_spaces(self, index: str, fnames: Sequence[str], shards: List[int], comm) -> None:
        """Collective on every rank, fields in the same order: all-gather the
        ranks' row directories of each field's standard view and keep their
        sorted union as the node row space (a rank without the view adds
        nothing).  Every rank takes part in every gather whatever fails
        locally."""
        import torch
        for fname in fnames:
            key = (index, fname, tuple(shards))
            rv = None
            try:
                rv = self.view_arena(index, fname, VIEW_STANDARD, shards) if shards else None
            except Exception:  # noqa: BLE001 - contribute no rows, decline in the readiness vote
                rv = None
            rows = np.ascontiguousarray(rv.rows if rv is not None else np.zeros(0, np.uint64), dtype=np.uint64)
            t = torch.from_numpy(rows.view(np.int64).copy()).to(comm.device)
            parts = comm.all_gather_var(t)
            space = np.unique(np.concatenate([p.cpu().numpy().view(np.uint64) for p in parts])) if parts else rows
            sig = (id(rv), rv.rows_gen) if rv is not None else None
            self._spaces[key] = (sig, space)

    def _batch_info(self, index: str, calls: List[Call], shards: List[int]):
        """(params per call, {field: (fragments, view, rank caches)}) of a
        TopN batch, resolved once per batch: the mesh asks for readiness,
        staleness and the batch itself on the same ``calls`` list (a 16-call
        request used to resolve its one field ~50 times).  Thread-local,
        keyed by the identity of ``calls`` / ``shards`` and the mutation
        epoch."""
        tl = self.__dict__.setdefault("_tl", threading.local())
        ent = getattr(tl, "batch", None)
        epoch = mutation_epoch()
        if ent is not None and ent[0] is calls and ent[1] == index and ent[2] is shards and ent[3] == epoch:
            return ent[4]
        params = self._batch_params(index, calls)
        fields: Dict[str, Tuple] = {}
        for p in params:
            fname = p[0]
            if fname not in fields:
                frags = self._topn_frags(index, fname, shards)
                rv = self.view_arena(index, fname, VIEW_STANDARD, shards)
                rc = self._rank_caches(index, fname, shards, frags, rv) if rv is not None else None
                fields[fname] = (frags, rv, rc)
        info = (params, fields)
        tl.batch = (calls, index, shards, epoch, info)
        return info

    def _batch_params(self, index: str, calls: List[Call]):
        """topn_params of every call of a batch (schema + text only, the same
        on every rank), memoised per ``calls`` list like _batch_info."""
        tl = self.__dict__.setdefault("_tl", threading.local())
        ent = getattr(tl, "params", None)
        if ent is not None and ent[0] is calls and ent[1] == index:
            return ent[2]
        ex = self._ex()
        params = [ex.topn_params(index, c) for c in calls]
        tl.params = (calls, index, params)
        return params

    def _cand_groups(self, index: str, calls: List[Call], shards: List[int]) -> List[Tuple[str, int]]:
        """(field, nreq) of the batch's cache-only groups, sorted (the same
        on every rank: derived from the command text and schema only)."""
        params = self._batch_params(index, calls)
        ns: Dict[str, List[int]] = {}
        for c, p in zip(calls, params):
            if c.children:
                continue
            ns.setdefault(p[0], []).append(int(p[1]))
        return sorted((f, _nreq(v)) for f, v in ns.items())

    def topn_cand_stale(self, index: str, calls: List[Call], shards: List[int]) -> bool:
        """Does this rank miss the node candidate space of a cache-only group
        of the batch (never built, or built from rank caches since replaced)?
        Local check; the mesh votes on it (parallel/mesh.py OP_TOPN)."""
        _, finfo = self._batch_info(index, calls, shards)
        for fname, nreq in self._cand_groups(index, calls, shards):
            rc = finfo[fname][2]
            ent = self._cand_spaces.get((index, fname, tuple(shards), nreq))
            if ent is None or ent[0] != (rc.serial if rc is not None else None):
                return True
        return False

    def refresh_cand_spaces(self, index: str, calls: List[Call], shards: List[int], comm) -> None:
        """Collective on every rank, groups in the same order: all-gather each
        rank's local candidate rows of a cache-only group (with its fragment
        and device-shard counts) and keep, per group, the node candidate space
        and this rank's tensors over it (DeviceRankCaches.node_candidates).
        The fused one-all-reduce path is enabled only when it fits on every
        rank (int32 node totals, the count-matrix cap): a node-wide decision."""
        import torch

        from .topn_exec import FUSED_MAX_CELLS
        for fname, nreq in self._cand_groups(index, calls, shards):
            rc = None
            rows = np.zeros(0, np.uint64)
            try:
                rc = self._batch_info(index, calls, shards)[1][fname][2]
                if rc is not None:
                    rows = rc.local_candidate_rows(nreq)
            except Exception:  # noqa: BLE001 - take part with nothing; the fit check fails below
                rc = None
            head = np.array([rc.S if rc is not None else -1, rc.view.S if rc is not None else 0], np.int64)
            t = torch.from_numpy(np.concatenate([head, rows.view(np.int64)])).to(comm.device)
            parts = [p.cpu().numpy() for p in comm.all_gather_var(t)]
            space = np.unique(np.concatenate([p[2:].view(np.uint64) for p in parts])) if parts else rows
            s_frag = [int(p[0]) for p in parts]
            fits = min(s_frag) >= 0 and len(space) * max(s_frag) <= FUSED_MAX_CELLS and \
                sum(int(p[1]) for p in parts) < 2048 and len(space) > 0
            key = (index, fname, tuple(shards), nreq)
            cand = None
            if fits and rc is not None:
                try:
                    cand = rc.node_candidates(nreq, space)
                except Exception:  # noqa: BLE001 - contributes zeros; the batch answers without this rank
                    cand = None
            # (serial, candidates, fits node-wide, space, the caches they were
            # built from, tie-break ids): every rank holds an entry after a
            # refresh, so the fused-or-not choice is the same on every rank
            ids = torch.arange(len(space), dtype=torch.int32, device=comm.device) if fits else None
            if len(self._cand_spaces) > 256:
                self._cand_spaces.clear()
            self._cand_spaces[key] = (rc.serial if rc is not None else None, cand, fits, space, rc, ids)

    def _topn_index(self, index: str, fname: str, shards: List[int], rc, rv, space=None):
        """Device slot index (ops/topn_index.py) over the rank caches ``rc``,
        rebuilt when they change, at most once per TOPN_INDEX_REBUILD_S per
        view (stale in between: the pair-count path)."""
        if rv is None or rc is None or not self.topn_index_enabled or rc.K == 0:
            self._topn_index_why = "disabled/empty"
            return None
        # (fragments wider than 2^20 columns: the index is per arena
        # sub-shard, the histograms and walks per fragment)
        from pilosa_amd.ops.topn_index import MAX_SLOTS, DeviceTopNIndex
        key = (index, fname, tuple(shards))
        ent = self._topn_indexes.get(key)
        want = rv.rows if space is None else space
        same_space = ent is not None and (ent[1].space is want or np.array_equal(ent[1].space, want))
        if ent is not None and ent[0] is rc and ent[1].view is rv and not ent[1].stale and same_space:
            return ent[1]
        if ent is not None and ent[1].view is rv and space is None:
            # after writes: re-index only the changed shards, in place (no
            # throttle, no fall back to the pair-count path)
            if ent[1].refresh(rv, rc):
                self._topn_indexes[key] = (rc, ent[1], ent[2])
                self.topn_index_refreshes += 1
                return ent[1]
        now = time.monotonic()
        if ent is not None and now - ent[2] < TOPN_INDEX_REBUILD_S:
            self._topn_index_why = (f"throttled: same_rc={ent[0] is rc} same_view={ent[1].view is rv} "
                                    f"stale={ent[1].stale}")
            return None
        if rc.K > MAX_SLOTS:
            self._topn_index_why = "too many slots"
            return None
        self._topn_indexes.pop(key, None)   # free the old index's HBM before building
        t_b = time.perf_counter()
        try:
            tix = DeviceTopNIndex(rv, rc, space=space)
        except ValueError:
            return None
        if self.device.type == "cuda":
            import torch
            torch.cuda.synchronize(self.device)
        self.topn_index_build_s += time.perf_counter() - t_b
        self.topn_index_builds += 1
        if not tix.ok:
            return None
        self._topn_indexes[key] = (rc, tix, now)
        return tix

    # ------------------------------------------------------------ GroupBy
    def group_by(self, index: str, c: Call, filt: Optional[Call], shards: List[int], child_rows, limit: int):
        from pilosa_amd.executor import FieldRow, GroupCount
        ex = self._ex()
        k = len(c.children)
        if k == 0 or k + (1 if filt is not None else 0) > 16:
            raise NotImplementedError
        fields = []
        arenas = []
        cand: List[List[int]] = []
        for i, ch in enumerate(c.children):
            fname = ch.args.get("_field")
            if not isinstance(fname, str) or self.holder.field(index, fname) is None:
                raise NotImplementedError
            dv = self.view_arena(index, fname, VIEW_STANDARD, shards)
            if dv is None:
                return []
            rows = [int(r) for r in dv.rows] if dv.D else []
            if child_rows[i] is not None:
                keep = set(child_rows[i])
                rows = [r for r in rows if r in keep]
            if not rows:
                return []
            fields.append(fname)
            arenas.append(dv)
            cand.append(rows)
        fexpr = None
        if filt is not None:
            fexpr = self.plan(index, filt, shards)
            if fexpr is EMPTY:
                return []
        start = ex.group_by_start(c)
        if start is not None:
            # a child without previous starts at ITS first row in EACH shard
            # (reference iterator per shard): exact on the merged candidates
            # only when such children all come after the paged ones
            seen_none = False
            for v in start:
                if v is None:
                    seen_none = True
                elif seen_none:
                    raise NotImplementedError
            start = tuple(-1 if v is None else v for v in start)
        if k == 2 and len(cand[0]) * len(cand[1]) >= GROUPBY_MATRIX_MIN and \
                (fexpr is None or type(fexpr) is Leaf) and self._matrix_fits(len(cand[0]), len(cand[1])):
            # two fields: the whole count matrix in one bit-GEMM (MFMA), then
            # the lexicographic walk on the host (ops/groupby.py)
            from .groupby import emit_groups, pair_count_matrix
            self.launches += 1
            mat = pair_count_matrix(arenas[0], cand[0], arenas[1], cand[1],
                                    filt=(fexpr.view, fexpr.row) if fexpr is not None else None,
                                    chunk_bytes=self._groupby_budget() - len(cand[0]) * len(cand[1]) * 12)
            return [GroupCount([FieldRow(fields[0], ra), FieldRow(fields[1], rb)], n)
                    for ra, rb, n in emit_groups(cand[0], cand[1], mat,
                                                 None if start is None else (start[0], start[1] - 1), limit)]
        try:
            groups = self._pruned_groups(arenas, cand, fexpr, start, limit)
        except CompileError:
            raise NotImplementedError
        return [GroupCount([FieldRow(fields[i], key[i]) for i in range(k)], n) for key, n in groups]

    # HBM the two-field count matrix may use (densified rows + the matrix)
    GROUPBY_HBM = int(os.environ.get("PILOSA_GROUPBY_HBM", str(8 << 30)))

    def _groupby_budget(self) -> int:
        budget = self.GROUPBY_HBM
        if self.device.type == "cuda":
            import torch
            free, _ = torch.cuda.mem_get_info(self.device)
            budget = min(budget, int(free * 0.5))
        return budget

    def _matrix_fits(self, ra: int, rb: int) -> bool:
        """The count matrix densifies (ra + rb) rows x 128 KiB for at least one
        shard and keeps an ra x rb int64+int32 matrix; two 1M-row fields would
        need terabytes -> the pruned enumeration instead."""
        from .groupby import WORDS_PER_SHARD
        need = (ra + rb) * WORDS_PER_SHARD * 8 + ra * rb * 12
        return need <= self._groupby_budget()

    def _pruned_groups(self, arenas, cand, fexpr, start, limit: int):
        """GroupBy combinations in lexicographic order with cumulative-
        intersection pruning (reference groupByIterator, executor.go:3060-3230):
        a prefix whose intersection (with the filter) is empty is never
        extended.  The work list holds (prefix, next row index) items in
        lexicographic order; each launch counts the next children of the
        front items (1024 per launch at first, doubling up to
        MAX_GROUPS_PER_LAUNCH), so the output order is lexicographic and the
        walk stops as soon as ``limit`` groups exist -- two 1M-row fields with
        limit=100 cost a couple of launches, not a 10^12-cell matrix."""
        k = len(cand)
        out: List[Tuple[Tuple[int, ...], int]] = []
        todo: List[Tuple[Tuple[int, ...], int]] = [((), 0)]
        budget = 1024
        while todo and len(out) < limit:
            lvl = len(todo[0][0])
            keys: List[Tuple[int, ...]] = []
            rest: List[Tuple[Tuple[int, ...], int]] = []
            i = 0
            while i < len(todo) and len(todo[i][0]) == lvl and len(keys) < budget:
                pre, j = todo[i]
                rows = self._next_rows(cand[lvl], pre, start)
                take = rows[j:j + budget - len(keys)]
                keys.extend(pre + (r,) for r in take)
                if j + len(take) < len(rows):
                    rest.append((pre, j + len(take)))  # unfinished: its remaining children come next
                    i += 1
                    break
                i += 1
            todo = rest + todo[i:]
            budget = min(budget * 2, MAX_GROUPS_PER_LAUNCH)
            if not keys:
                continue
            self.launches += 1
            got = self._count_keys(arenas, keys, fexpr)
            live = [(key, int(v)) for key, v in zip(keys, got) if v > 0]
            if lvl + 1 == k:
                for key, v in live:
                    if start is not None and key < start:
                        continue
                    out.append((key, v))
                    if len(out) >= limit:
                        break
            else:
                # children go before everything after their parents; an
                # unfinished parent's remaining children come after them
                todo = [(key, 0) for key, _ in live] + todo
        return out[:limit]

    def _count_keys(self, arenas, keys: List[Tuple[int, ...]], fexpr) -> np.ndarray:
        """|filter & row_0 & ... & row_l| for every key of one level: programs
        built column-wise with numpy (a left AND-fold over the leaves) instead
        of one expression object per key; a non-leaf filter goes through the
        expression compiler."""
        from .device import OP_AND, QPROG_DTYPE
        if fexpr is not None and type(fexpr) is not Leaf:
            exprs = [Op("and", (fexpr, *[Leaf(arenas[x], key[x]) for x in range(len(key))])) for key in keys]
            return self.engine.count(exprs)
        L0 = 1 if fexpr is not None else 0
        lvl = len(keys[0])
        L = L0 + lvl
        views: List[DeviceView] = []
        slot_of: Dict[int, int] = {}

        def slot(v):
            if id(v) not in slot_of:
                slot_of[id(v)] = len(views)
                views.append(v)
            return slot_of[id(v)]
        Q = len(keys)
        progs = np.zeros(Q, dtype=QPROG_DTYPE)
        progs["nleaf"] = L
        progs["nprog"] = 2 * L - 1
        kk = np.asarray(keys, dtype=np.uint64).reshape(Q, lvl)
        if fexpr is not None:
            progs["leaf_view"][:, 0] = slot(fexpr.view)
            progs["leaf_row"][:, 0] = fexpr.view.dense(fexpr.row)
        for x in range(lvl):
            progs["leaf_view"][:, L0 + x] = slot(arenas[x])
            progs["leaf_row"][:, L0 + x] = arenas[x].dense_many(kk[:, x])
        pg = [0] + [v for i in range(1, L) for v in (i, OP_AND)]
        progs["prog"][:, :len(pg)] = np.asarray(pg, np.uint8)
        eng = self.engine
        return eng.launch_count(eng.prepare_progs(progs, views, views[0].S)).cpu().numpy()

    @staticmethod
    def _next_rows(rows: List[int], prefix: Tuple[int, ...], start: Optional[Tuple[int, ...]]) -> List[int]:
        """Rows of the next field for ``prefix``: while the prefix equals
        ``start``'s, only rows from start's row on (paging,
        Executor.group_by_start)."""
        if start is None or tuple(start[:len(prefix)]) != prefix:
            return rows
        lo = start[len(prefix)]
        return [r for r in rows if r >= lo]


def _fold_subshards(rid: np.ndarray, cnt: np.ndarray, is_min: bool, filtered: bool):
    """Per-device-shard MinRow/MaxRow pairs -> per host shard (shards wider
    than 2^20 columns): the first (last) row over the shard's sub-shards,
    with the filtered count summed over the sub-shards that found it."""
    M = shardwidth.DEVICE_SUBSHARDS
    r, c = rid.reshape(-1, M), cnt.reshape(-1, M)
    big = np.iinfo(np.int64).max
    live = c > 0
    key = np.where(live, r, big if is_min else -1)
    best = key.min(axis=1) if is_min else key.max(axis=1)
    hit = live & (r == best[:, None])
    n = (np.where(hit, c, 0).sum(axis=1) if filtered else hit.any(axis=1).astype(np.int64))
    ok = live.any(axis=1)
    return np.where(ok, best, 0), np.where(ok, n, 0)


def _fold_subshards_value(vals: np.ndarray, cnts: np.ndarray, is_min: bool, M: Optional[int] = None):
    """Per-device-shard (value, count) -> per fragment wider than 2^20
    columns: the min (max) value over its sub-shards with the counts of
    every sub-shard holding that value summed.  (The host reference of
    bsi_minmax_fold_kernel, tests/test_gpu_kernels.py.)"""
    M = shardwidth.DEVICE_SUBSHARDS if M is None else M
    v, c = vals.reshape(-1, M), cnts.reshape(-1, M)
    live = c > 0
    big = np.iinfo(np.int64).max
    key = np.where(live, v, big if is_min else -big)
    best = key.min(axis=1) if is_min else key.max(axis=1)
    n = np.where(live & (v == best[:, None]), c, 0).sum(axis=1)
    return np.where(n > 0, best, 0), n


def _minmax_per_shard(o: np.ndarray, which: str):
    """Per-shard (value, count) of the BSI min/max descents ``o`` int64[S, 16, 10]
    (bitmap_kernels.hip bsi_minmax_kernel, per key: 0/1 max |neg| + count,
    2/3 min pos, 4/5 max pos, 6/7 min |neg|, 8/9 any pos / any neg), vectorised
    over the shards with fragment.min/max's sign rules (fragment.go:1145-1225);
    count 0 = no value in the shard."""
    big = np.iinfo(np.int64).max
    pos = o[:, :, 8] > 0
    neg = o[:, :, 9] > 0
    anyp, anyn = pos.any(axis=1), neg.any(axis=1)

    def pick(vcol, ccol, mask, largest):
        v = np.where(mask, o[:, :, vcol], -1 if largest else big)
        best = v.max(axis=1) if largest else v.min(axis=1)
        cnt = np.where(mask & (o[:, :, vcol] == best[:, None]), o[:, :, ccol], 0).sum(axis=1)
        return best, cnt

    if which == "min":
        vn, cn = pick(0, 1, neg, True)      # -(max magnitude among negatives)
        vp, cp = pick(2, 3, pos, False)
        val = np.where(anyn, -vn, vp)
        cnt = np.where(anyn, cn, np.where(anyp, cp, 0))
    else:
        vp, cp = pick(4, 5, pos, True)
        vn, cn = pick(6, 7, neg, False)     # all negative: -(min magnitude), fragment.max quirk
        val = np.where(anyp, vp, -vn)
        cnt = np.where(anyp, cp, np.where(anyn, cn, 0))
    return val.tolist(), cnt.tolist()


def _shift_total(e) -> int:
    """The largest total Shift of the shifted leaves of a planned expression
    (0: none)."""
    if type(e) is Leaf:
        return int(getattr(e.view, "_shift_total", 0) or 0) if getattr(e.view, "_spill", None) is not None else 0
    if type(e) is Op:
        return max((_shift_total(a) for a in e.args), default=0)
    return 0


def _has_shift(e) -> bool:
    if type(e) is Leaf:
        return getattr(e.view, "_spill", None) is not None
    if type(e) is Op:
        return any(_has_shift(a) for a in e.args)
    return False


def spill_expr(e):
    """The expression evaluated over the next-shard spill of every Shift leaf:
    plain leaves hold no bits past their shard (EMPTY), so an Intersect with
    one drops the spill while Union/Xor/Difference-left keep it -- exactly the
    per-shard Row algebra of the reference (row.go Intersect/Union/...)."""
    if type(e) is Leaf:
        sp = getattr(e.view, "_spill", None)
        return Leaf(sp, 0) if sp is not None else EMPTY
    if type(e) is not Op:
        return EMPTY
    kids = [spill_expr(a) for a in e.args]
    if e.op == "and":
        return EMPTY if any(k is EMPTY for k in kids) else Op("and", tuple(kids))
    if e.op == "andnot":
        if kids[0] is EMPTY:
            return EMPTY
        rest = [k for k in kids[1:] if k is not EMPTY]
        return kids[0] if not rest else Op("andnot", (kids[0], *rest))
    kids = [k for k in kids if k is not EMPTY]  # or / xor
    if not kids:
        return EMPTY
    return kids[0] if len(kids) == 1 else Op(e.op, tuple(kids))


def row_from_bitmaps(bms, shard_list, spill_bms=(), spill_shards=()) -> Row:
    """A Row from per-device-shard result Bitmaps; the bits a shard's Shift
    carried past its last column belong to the next shard's segment (Row.Merge
    in the reference's reduce)."""
    row = Row()
    for s, bm in zip(shard_list, bms):
        if bm is not None and bm.any():
            row.segments[int(s)] = bm
    M = shardwidth.DEVICE_SUBSHARDS   # spill of device shard s belongs to s + M (the next shard)
    for s, bm in zip(spill_shards, spill_bms):
        if bm is not None and bm.any():
            part = _rebase_spill(bm)
            t = int(s) + M
            row.segments[t] = row.segments[t].union(part) if t in row.segments else part
    return row


def _rebase_spill(bm):
    """Spill bitmap of `shard` (positions in shard's column range) -> the same
    bits at shard + 1's columns."""
    from pilosa_amd import _roaring

    cols = np.asarray(bm.slice(), dtype=np.uint64) + np.uint64(SHARD_WIDTH)
    out = _roaring.Bitmap()
    out.add_many(cols)
    return out


class _NeedMore(Exception):
    """A replay reached a candidate whose count was not computed yet."""


def _counted(counted: Dict[int, np.ndarray], rid: int, si: int) -> int:
    row = counted.get(rid)
    if row is None:
        raise _NeedMore
    return int(row[si])


def _replay_top(pairs: List[Tuple[int, int]], count_of, n: int, min_threshold: int, tan: int = 0,
                src_count: int = 0, keep=None) -> List[Pair]:
    """fragment.top() heap logic (fragment.go:1568-1700) with precomputed
    src∩row counts (``count_of``; None = no src, the cached counts), the
    Tanimoto window and the attribute filter ``keep``."""
    import heapq
    import math
    heap: List[Tuple[int, int]] = []
    min_t = max_t = 0.0
    if tan > 0:
        min_t = float(src_count * tan) / 100
        max_t = float(src_count * 100) / float(tan)
    for rid, cnt in pairs:
        if cnt == 0:
            continue
        if tan > 0:
            if cnt <= min_t or cnt >= max_t:
                continue
        elif cnt < min_threshold:
            continue
        if keep is not None and not keep(rid):
            continue
        if n == 0 or len(heap) < n:
            count = cnt if count_of is None else count_of(rid)
            if count == 0:
                continue
            if tan > 0:
                if math.ceil(float(count * 100) / float(cnt + src_count - count)) <= tan:
                    continue
            elif count < min_threshold:
                continue
            heapq.heappush(heap, (count, -rid))
            if count_of is None and n > 0 and len(heap) == n:
                break
            continue
        threshold = heap[0][0]
        if threshold < min_threshold or cnt < threshold:
            break
        count = count_of(rid)
        if count < threshold:
            continue
        heapq.heappush(heap, (count, -rid))
    return sort_pairs([Pair(-nid, cc) for cc, nid in heap])
