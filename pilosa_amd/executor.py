"""PQL executor (reference: executor.go).

``Executor.execute`` = translate keys -> run each call -> attach column attrs
-> translate ids back to keys (executor.go:116-209).  Every read call is a
map/reduce over shards (executor.go:2458-2611): shards are grouped by owning
node (cluster placement); remote nodes get the canonical call string over the
internal client; local shards run either

* on the GPU engine (pilosa_amd/ops/gpu_executor.py) — ONE batched launch over
  all local shards for Count / bitmap calls / Sum / TopN / GroupBy, or
* on the host C++ roaring core, shard by shard (the CPU oracle / fallback).

Result types mirror the reference: Row, int (Count), ValCount, Pair,
list[Pair] (TopN), RowIdentifiers (Rows), list[GroupCount], bool, None.
"""
from __future__ import annotations

import concurrent.futures as cf
import datetime as dt
import os
import re
import threading
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

from pilosa_amd import _roaring
from pilosa_amd.errors import (BadRequestError, ErrBSIGroupNotFound, ErrFieldNotFound, ErrIndexNotFound,
                               ErrIndexRequired, ErrTooManyWrites, PilosaError, wrap)
from pilosa_amd.models.cache import Pair, PairArray, pairs_add, sort_pairs
from pilosa_amd.models.field import FIELD_TYPE_BOOL, FIELD_TYPE_INT, FIELD_TYPE_SET, FIELD_TYPE_TIME
from pilosa_amd.models.fragment import FALSE_ROW_ID, SHARD_WIDTH, TRUE_ROW_ID, TopOptions
from pilosa_amd.models.index import EXISTENCE_FIELD_NAME
from pilosa_amd.models.row import Row
from pilosa_amd.models.timeq import (TIME_FORMAT, min_max_views, parse_time, time_of_view, views_by_time_range)
from pilosa_amd.models.view import VIEW_BSI_PREFIX, VIEW_STANDARD
from pilosa_amd.pql import BETWEEN, EQ, GT, GTE, LT, LTE, NEQ, Call, Condition, Query, parse_string
from pilosa_amd.parallel.mesh import MeshError
from pilosa_amd.utils import tracing

DEFAULT_FIELD = "general"
_FANOUT_LOCK = threading.Lock()
DEFAULT_MIN_THRESHOLD = 1
MAX_INT = (1 << 63) - 1


# a request that is one unfiltered BSI aggregate: Sum|Min|Max(field=<name>)
_BSI_AGG_RE = re.compile(r"\s*(Sum|Min|Max)\(\s*field\s*=\s*([A-Za-z][A-Za-z0-9_-]*)\s*\)\s*$")


class ExecOptions:
    __slots__ = ("remote", "exclude_row_attrs", "exclude_columns", "column_attrs", "mesh_local", "device_counts")

    def __init__(self, remote=False, exclude_row_attrs=False, exclude_columns=False, column_attrs=False):
        self.remote = remote
        self.exclude_row_attrs = exclude_row_attrs
        self.exclude_columns = exclude_columns
        self.column_attrs = column_attrs
        self.mesh_local = False  # set on a rank's own share of a multi-GPU call
        # a Count-only request answered in one device launch returns its counts
        # as the device int64 tensor (callers that reduce on the device: the
        # SPMD multi-GPU bench all-reduces it without a host round trip)
        self.device_counts = False

    def copy(self):
        o = ExecOptions(self.remote, self.exclude_row_attrs, self.exclude_columns, self.column_attrs)
        o.mesh_local = self.mesh_local
        o.device_counts = self.device_counts
        return o


class ValCount:
    __slots__ = ("val", "count")

    def __init__(self, val=0, count=0):
        self.val, self.count = int(val), int(count)

    def add(self, o: "ValCount") -> "ValCount":
        return ValCount(_wrap(self.val + o.val), self.count + o.count)

    def smaller(self, o: "ValCount") -> "ValCount":
        if self.count == 0 or (o.val < self.val and o.count > 0):
            return o
        return ValCount(self.val, self.count)

    def larger(self, o: "ValCount") -> "ValCount":
        if self.count == 0 or (o.val > self.val and o.count > 0):
            return o
        return ValCount(self.val, self.count)

    def to_json(self):
        return {"value": self.val, "count": self.count}

    def __eq__(self, o):
        return isinstance(o, ValCount) and (self.val, self.count) == (o.val, o.count)

    def __repr__(self):
        return f"ValCount({self.val}, {self.count})"


class RowIdentifiers:
    __slots__ = ("rows", "keys")

    def __init__(self, rows=None, keys=None):
        self.rows = list(rows or [])
        self.keys = list(keys) if keys is not None else None

    def to_json(self):
        d = {"rows": self.rows}
        if self.keys:
            d["keys"] = self.keys
            d["rows"] = []
        return d

    def __eq__(self, o):
        return isinstance(o, RowIdentifiers) and self.rows == o.rows and (self.keys or []) == (o.keys or [])

    def __repr__(self):
        return f"RowIdentifiers({self.rows}, {self.keys})"


class FieldRow:
    __slots__ = ("field", "row_id", "row_key")

    def __init__(self, field, row_id, row_key=""):
        self.field, self.row_id, self.row_key = field, int(row_id), row_key

    def to_json(self):
        if self.row_key:
            return {"field": self.field, "rowKey": self.row_key}
        return {"field": self.field, "rowID": self.row_id}

    def __eq__(self, o):
        return isinstance(o, FieldRow) and (self.field, self.row_id, self.row_key) == (o.field, o.row_id, o.row_key)

    def __repr__(self):
        return f"FieldRow({self.field!r}, {self.row_id}{', ' + repr(self.row_key) if self.row_key else ''})"


class GroupCount:
    __slots__ = ("group", "count")

    def __init__(self, group: List[FieldRow], count: int):
        self.group, self.count = group, int(count)

    def key(self):
        return tuple(g.row_id for g in self.group)

    def to_json(self):
        return {"group": [g.to_json() for g in self.group], "count": self.count}

    def __eq__(self, o):
        return isinstance(o, GroupCount) and self.group == o.group and self.count == o.count

    def __repr__(self):
        return f"GroupCount({self.group}, {self.count})"


class QueryResponse:
    def __init__(self, results=None, column_attr_sets=None, err=None):
        self.results = results if results is not None else []
        self.column_attr_sets = column_attr_sets
        self.err = err


def _wrap(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def merge_row_ids(a: List[int], b: List[int], limit: int) -> List[int]:
    out: List[int] = []
    i = j = 0
    while i < len(a) and j < len(b) and len(out) < limit:
        if a[i] < b[j]:
            out.append(a[i]); i += 1
        elif a[i] > b[j]:
            out.append(b[j]); j += 1
        else:
            out.append(a[i]); i += 1; j += 1
    while i < len(a) and len(out) < limit:
        out.append(a[i]); i += 1
    while j < len(b) and len(out) < limit:
        out.append(b[j]); j += 1
    return out


def merge_group_counts(a: List[GroupCount], b: List[GroupCount], limit: int) -> List[GroupCount]:
    limit = min(limit, len(a) + len(b))
    out: List[GroupCount] = []
    i = j = 0
    while i < len(a) and j < len(b) and len(out) < limit:
        ka, kb = a[i].key(), b[j].key()
        if ka < kb:
            out.append(a[i]); i += 1
        elif ka > kb:
            out.append(b[j]); j += 1
        else:
            out.append(GroupCount(a[i].group, a[i].count + b[j].count)); i += 1; j += 1
    while i < len(a) and len(out) < limit:
        out.append(a[i]); i += 1
    while j < len(b) and len(out) < limit:
        out.append(b[j]); j += 1
    return out


GPU_FAULT_LIMIT = int(os.environ.get("PILOSA_GPU_FAULT_LIMIT", "3"))
# process-wide count of device faults answered from the host (tests assert
# that a device-routed query never took this path)
DEVICE_FAULTS = [0]


def _results_equal(a, b) -> bool:
    """Device vs host result equality for the paranoia check (rows compare
    by columns, pairs/group counts by value)."""
    if isinstance(a, Row) and isinstance(b, Row):
        return list(a.columns()) == list(b.columns())
    if isinstance(a, Row) or isinstance(b, Row):
        a = a if not isinstance(a, Row) else list(a.columns())
        b = b if not isinstance(b, Row) else list(b.columns())
    a = a.to_list() if isinstance(a, PairArray) else a
    b = b.to_list() if isinstance(b, PairArray) else b
    if isinstance(a, list) and isinstance(b, list) and all(isinstance(x, Pair) for x in a + b):
        # TopN partials: the host reduce keeps insertion order, the device sorts
        return sorted((p.id, p.count) for p in a) == sorted((p.id, p.count) for p in b)
    return a == b or (not a and not b)


class Executor:
    def __init__(self, holder, cluster=None, client=None, gpu=None, workers: int = 8, max_writes: int = 5000,
                 stats=None):
        self.holder = holder
        self.cluster = cluster
        self.client = client
        self.gpu = gpu            # GpuExecutor or None
        if gpu is not None and getattr(gpu, "executor", False) is None:
            gpu.executor = self   # plans need the executor's BSI/time/TopN helpers
        self.mesh = None          # parallel.mesh.ShardMesh on a multi-GPU node (rank 0 front end)
        # concurrent single-Count requests share GPU launches (ops/coalescer.py)
        self.coalesce = os.environ.get("PILOSA_COALESCE", "1") != "0"
        # PILOSA_PARANOIA=1: every device result is re-derived on the host and
        # compared (the reference's roaringparanoia build tag, for the GPU path)
        self.paranoia = os.environ.get("PILOSA_PARANOIA", "0") == "1"
        self.gpu_faults = 0
        # strict: a device fault raises instead of falling back to the host
        # fragments (also PILOSA_GPU_STRICT=1; tests: the device must answer)
        self.strict_gpu = False
        self.logger = None
        self._coalescer = None
        self._topn_coalescer = None
        self.topn_batch_declined = 0
        self.max_writes = max_writes
        # per-call counters go to the holder's client unless given one (executor.go:298-340)
        self.stats = stats if stats is not None else getattr(holder, "stats", None)
        self.pool = cf.ThreadPoolExecutor(max_workers=max(1, workers), thread_name_prefix="shard")

    def close(self):
        self.pool.shutdown(wait=False)
        pool = self.__dict__.get("_fanout")
        if pool is not None:
            pool.shutdown(wait=False)

    # ================================================================ entry
    def execute(self, index: str, q, shards: Optional[Sequence[int]] = None,
                opt: Optional[ExecOptions] = None) -> QueryResponse:
        with tracing.span("Executor.Execute"):
            if isinstance(q, str):
                if self._use_mesh(opt):
                    res = self._mesh_count_text(index, q, shards, opt)
                    if res is not None:
                        return QueryResponse(res)
                fast = self._count_text_fast(index, q, shards, opt)
                if fast is not None:
                    return QueryResponse(fast)
                # Sum / Min / Max(field=f) alone: straight to the call, no parse
                # tree or request dispatch (a BSI aggregate is ~0.5 ms of device
                # streaming; the generic layers were a visible share on top)
                if opt is None and self.gpu is not None:
                    m = _BSI_AGG_RE.match(q)
                    if m is not None:
                        fast = self._bsi_agg_fast(index, m.group(1), m.group(2), shards)
                        if fast is not None:
                            return QueryResponse([fast])
                # a request of several cache-only TopN calls: parsed once, one
                # device batch, columnar results (single calls keep the
                # cross-request coalescer of the general path)
                if opt is None and (self.gpu is not None or self.mesh is not None) and \
                        q.lstrip().startswith("TopN(") and q.count("TopN(") >= 2:
                    try:
                        fast = self._topn_plain_fast(index, q, shards)
                        if fast is None:
                            fast = self._topn_text_fast(index, q, shards)
                    except PilosaError:
                        fast = None   # the general path reports it
                    if fast is not None:
                        return QueryResponse(fast)
                text = q
                q = parse_string(q)
                q.source = text
            if not index:
                raise ErrIndexRequired
            idx = self.holder.index(index)
            if idx is None:
                raise ErrIndexNotFound
            if self.max_writes > 0 and q.write_call_n() > self.max_writes:
                raise ErrTooManyWrites
            opt = opt or ExecOptions()
            if not opt.remote:
                for c in q.calls:
                    self._translate_call(index, idx, c)
            results = self._execute(index, q, list(shards) if shards else [], opt)
            resp = QueryResponse(results)
            if opt.column_attrs:
                cols = set()
                for r in results:
                    if isinstance(r, Row):
                        cols |= {int(c) for c in r.columns()}
                sets = []
                for cid in sorted(cols):
                    a = idx.column_attr_store.attrs(cid)
                    if a:
                        sets.append({"id": cid, "attrs": a})
                if idx.keys:
                    # ColumnAttrSet field order: id / key, then attrs (executor.go ColumnAttrSet)
                    ts = self.holder.translate
                    sets = [{"key": ts.translate_column_to_string(index, s["id"]), "attrs": s["attrs"]} for s in sets]
                resp.column_attr_sets = sets
            if not opt.remote:
                resp.results = [self._translate_result(index, idx, c, r) for c, r in zip(q.calls, results)]
            return resp

    # requests of at least this many Count() calls try the native text path
    COUNT_TEXT_MIN = int(os.environ.get("PILOSA_COUNT_TEXT_MIN", "2"))

    def _count_text_fast(self, index: str, text: str, shards, opt: Optional[ExecOptions],
                         min_calls: Optional[int] = None) -> Optional[List[int]]:
        """Serving fast path for a request that is only Count(<Row/set-op
        tree>) calls over local shards: the PQL text is compiled natively
        straight to device programs (no Python AST; native/pql_compile.cpp)
        and answered in one launch.  None = use the general path (which also
        produces every error the reference would)."""
        gpu = self.gpu
        if gpu is None or (opt is not None and opt.column_attrs):
            return None
        dev_out = opt is not None and opt.device_counts
        if opt is not None and opt.remote and not dev_out:
            return None
        head = text.lstrip()[:6]
        if head != "Count(" and head != "Count ":
            return None
        if text.count("Count") < (self.COUNT_TEXT_MIN if min_calls is None else min_calls):
            return None
        idx = self.holder.index(index)
        if idx is None:
            return None
        shards = list(shards) if shards else (idx.available_shards() or [0])
        if self._has_remote(index, shards, opt or ExecOptions()):
            return None
        fn = getattr(gpu, "try_count_text", None)
        if fn is None:
            return None
        try:
            with tracing.span("Executor.countTextNative", shards=len(shards)):
                res = fn(index, text, shards, device_out=True) if dev_out else fn(index, text, shards)
        except PilosaError:
            raise
        except Exception as err:  # noqa: BLE001 - device fault: general path
            self._gpu_fault(err)
            return None
        if res is not None and self.stats is not None:
            self.stats.count_with_tags("Count", len(res), [f"index:{index}"])
        return res

    def _mesh_count_text(self, index: str, text: str, shards, opt: Optional[ExecOptions]) -> Optional[List[int]]:
        """Multi-GPU node: a request of Count() calls goes to the ranks as
        its PQL text (each compiles its share natively, parallel/mesh.py
        count_text) and comes back as one all-reduced tensor; several such
        requests are in flight at once.  None = general path."""
        if opt is not None and (opt.remote or opt.column_attrs):
            return None
        head = text.lstrip()[:6]
        if (head != "Count(" and head != "Count ") or text.count("Count") < self.COUNT_TEXT_MIN:
            return None
        idx = self.holder.index(index)
        if idx is None or idx.keys or any(f.options.keys for f in idx.fields.values()):
            return None   # key translation happens on the general path
        shards = list(shards) if shards else (idx.available_shards() or [0])
        mesh = self.mesh
        try:
            with tracing.span("Executor.meshCountText", shards=len(shards)):
                return mesh.count_text(index, text, shards)
        except MeshError:
            if not mesh.failed_over:
                raise
            return None   # a rank is gone: this process adopted its shards

    def _execute(self, index: str, q: Query, shards: List[int], opt: ExecOptions) -> List[Any]:
        needs = any(c.name not in ("Clear", "Set", "SetRowAttrs", "SetColumnAttrs") for c in q.calls)
        if not shards and needs:
            idx = self.holder.index(index)
            shards = idx.available_shards() or [0]
        if q.calls and all(c.name == "SetRowAttrs" for c in q.calls):
            return self._bulk_set_row_attrs(index, q.calls, opt)
        # Concurrent requests of one Count() each are batched across requests.
        if len(q.calls) == 1 and q.calls[0].name == "Count" and self.coalesce and \
                (self.gpu is not None or self._use_mesh(opt)) and not self._has_remote(index, shards, opt):
            c = q.calls[0]
            key = (index, tuple(shards), self._use_mesh(opt))
            return [self.coalescer.submit(key, c, lambda: self.execute_call(index, c, shards, opt))]
        # Batch fast path: many Count() calls in one request go to the GPU together.
        if self._use_mesh(opt) and len(q.calls) > 1 and all(c.name == "Count" for c in q.calls) and \
                not self._has_remote(index, shards, opt):
            mesh = self.mesh
            try:
                return mesh.count_batch(index, q.calls, shards)
            except MeshError:
                if not mesh.failed_over:
                    raise  # a rank reported an error: the query's error
                # a rank is gone: this process adopted its shards, answer locally
        # many Sum() calls over one BSI field: one batched device launch
        # (bit-plane matrix on the matrix cores from 32 filters up)
        if self.gpu is not None and len(q.calls) > 1 and all(c.name == "Sum" for c in q.calls) and \
                not opt.remote and not self._use_mesh(opt) and not self._has_remote(index, shards, opt):
            try:
                res = self.gpu.bsi_sum_batch(index, q.calls, shards)
            except PilosaError:
                raise
            except Exception as err:  # noqa: BLE001 - device fault: host path below
                self._gpu_fault(err)
                res = None
            if res is not None:
                if self.stats is not None:
                    self.stats.count_with_tags("Sum", len(res), [f"index:{index}"])
                return res
        # TopN requests on a multi-GPU node: every rank's device runs both
        # phases, candidates and re-counts merge over the collectives
        if self._use_mesh(opt) and q.calls and all(c.name == "TopN" for c in q.calls) and not opt.remote and \
                not self._has_remote(index, shards, opt) and not any("ids" in c.args for c in q.calls):
            for c in q.calls:
                self._validate_call_args(c)
            mesh = self.mesh
            # the request text as sent (ranks parse it once) unless key
            # translation rewrote calls in place
            idx = self.holder.index(index)
            plain = idx is not None and not idx.keys and not any(f.options.keys for f in idx.fields.values())
            try:
                res = mesh.topn_batch(index, q.calls, shards, text=q.source if plain else None)
            except MeshError:
                if not mesh.failed_over:   # (failover detaches self.mesh)
                    raise
                res = None
            if res is not None:
                return res
        # TopN requests on a local GPU: both phases of every call on the device
        # (ops/topn_exec.py); concurrent single-TopN requests share launches
        if self.gpu is not None and q.calls and all(c.name == "TopN" for c in q.calls) and not opt.remote and \
                not self._use_mesh(opt) and not self._has_remote(index, shards, opt):
            for c in q.calls:
                self._validate_call_args(c)
            if any("ids" in c.args for c in q.calls):
                return [self.execute_call(index, c, shards, opt) for c in q.calls]   # phase 2 only: map step
            key = (index, tuple(shards))
            if len(q.calls) == 1 and self.coalesce:
                c = q.calls[0]
                return [self.topn_coalescer.submit(key, c, lambda: self.execute_call(index, c, shards, opt))]
            # multi-call requests run as their own batch: merging concurrent
            # ones serialised them and lost the CPU/GPU overlap between requests
            # (cache-only 15.4k -> 5.2k q/s, src unchanged; 32-query hot-rank
            # launches are slower than two 16-query ones: profiles/r04_e/)
            res = self._run_topn_batch(key, q.calls)
            if res is not None:
                return res
        if self.gpu is not None and len(q.calls) > 1 and all(c.name == "Count" for c in q.calls) and \
                not self._has_remote(index, shards, opt):
            try:
                res = self.gpu.try_count_batch(index, q.calls, shards)
            except PilosaError:
                raise
            except Exception as err:  # noqa: BLE001 - device fault: host path below
                self._gpu_fault(err)
                res = None
            if res is not None:
                return res
        return [self.execute_call(index, c, shards, opt) for c in q.calls]

    @property
    def coalescer(self):
        if self._coalescer is None:
            from pilosa_amd.ops.coalescer import CountCoalescer
            self._coalescer = CountCoalescer(self._run_count_batch)
        return self._coalescer

    @property
    def topn_coalescer(self):
        if self._topn_coalescer is None:
            from pilosa_amd.ops.coalescer import CountCoalescer
            self._topn_coalescer = CountCoalescer(self._run_topn_batch, max_batch=256)
        return self._topn_coalescer

    def _run_topn_batch(self, key, calls):
        index, shards = key
        if self.gpu is None:
            return None
        try:
            res = self.gpu.topn_batch(index, list(calls), list(shards))
            if res is None:
                self.topn_batch_declined += 1
        except PilosaError:
            raise
        except Exception as err:  # noqa: BLE001 - counted; each call then runs alone
            self._gpu_fault(err)
            return None
        if res is not None and self.stats is not None:
            self.stats.count_with_tags("TopN", len(res), [f"index:{index}"])
        if res is not None and self.paranoia:
            for c, r in zip(calls, res):
                want = self._topn(index, c, list(shards), ExecOptions())
                if [(p.id, p.count) for p in r] != [(p.id, p.count) for p in want]:
                    raise AssertionError(f"paranoia: device TopN {r!r} != host TopN {want!r}")
        return res

    def _bsi_agg_fast(self, index: str, name: str, fname: str, shards=None):
        """``Sum|Min|Max(field=fname)`` as the request's only call: the same
        execute_call the general path reaches, without building the request
        from a parse tree.  None = the general path."""
        idx = self.holder.index(index)
        if idx is None or idx.keys:
            return None
        f = idx.field(fname)
        if f is None or f.bsi_group(fname) is None:
            return None   # the general path reports it
        c = Call(name, {"field": fname})
        return self.execute_call(index, c, list(shards) if shards else (idx.available_shards() or [0]), ExecOptions())

    def _topn_plain_fast(self, index: str, text: str, shards=None) -> Optional[List[Any]]:
        """Fast path for a request of plain cache-only calls of one field --
        TopN(f[, n=][, threshold=]) -- recognised natively
        (native/pql_compile.cpp topn_plain): no Call objects or per-call
        argument handling, one fused device batch (ops/topn_exec.py), or on
        a multi-GPU node one mesh batch of a single all-reduce
        (ShardMesh.topn_plain).  None = the parse-based paths."""
        gpu = self.gpu
        mesh = self.mesh if self._use_mesh(None) else None
        if mesh is None and (gpu is None or not hasattr(gpu, "topn_plain_batch")):
            return None
        from pilosa_amd import _pql
        got = _pql.topn_plain(text)
        if got is None:
            return None
        fields, ns, ths = got
        fname = fields[0]
        if any(f != fname for f in fields):
            return None
        idx = self.holder.index(index)
        if idx is None or idx.keys:
            return None
        f = idx.field(fname)
        if f is None or f.type == FIELD_TYPE_INT or f.options.keys or f.options.cache_type == "none":
            return None
        skey = None
        if shards:
            shards = list(shards)
        else:
            # the index's memoised shard tuple, keyed by the shard epoch (no
            # per-request copy or hash of ~1k shard ids)
            ep, tup = idx.available_shards_memo()
            shards, skey = (tup, ("avail", index, ep)) if tup else ([0], None)
        if self._has_remote(index, shards, ExecOptions()):
            return None
        ths = [t or DEFAULT_MIN_THRESHOLD for t in ths]
        if mesh is not None:
            # every rank's GPU, one all-reduce per batch (parallel/mesh.py OP_TOPN_PLAIN)
            try:
                res = mesh.topn_plain(index, fname, ns, ths, shards)
            except MeshError:
                return None
            if res is None or len(res) != len(ns):
                return None
            if self.stats is not None:
                self.stats.count_with_tags("TopN", len(res), [f"index:{index}"])
            return res
        try:
            res = gpu.topn_plain_batch(index, fname, ns, ths, shards, skey=skey)
        except PilosaError:
            return None
        except RuntimeError as err:   # HIP / torch device error: counted, the general path answers
            self._gpu_fault(err)
            return None
        except Exception:  # noqa: BLE001 - not a device fault (e.g. an argument the fast path cannot hold)
            return None
        if res is None or len(res) != len(ns):
            return None
        if self.stats is not None:
            self.stats.count_with_tags("TopN", len(res), [f"index:{index}"])
        return res

    def _topn_text_fast(self, index: str, text: str, shards=None) -> Optional[List[Any]]:
        """Serving fast path for a text made only of cache-only TopN calls
        (the concurrent TopN requests the native HTTP front end groups): the
        text is parsed once and every call runs in ONE device batch (one
        OP_TOPN mesh batch on a multi-GPU node), results columnar
        (PairArray).  None = the general path, which also produces every
        error the reference would (executor.go:863-930)."""
        idx = self.holder.index(index)
        if idx is None or idx.keys or any(f.options.keys for f in idx.fields.values()):
            return None
        opt = ExecOptions()
        mesh = self.mesh if self._use_mesh(opt) else None
        if mesh is None and self.gpu is None:
            return None
        try:
            calls = parse_string(text).calls
        except Exception:  # noqa: BLE001 - the general path reports the parse error
            return None
        if not calls or any(c.name != "TopN" or c.children or "ids" in c.args for c in calls):
            return None
        try:
            for c in calls:
                self._validate_call_args(c)
        except PilosaError:
            return None
        shards = list(shards) if shards else (idx.available_shards() or [0])
        if self._has_remote(index, shards, opt):
            return None
        if mesh is not None:
            try:
                res = mesh.topn_batch(index, calls, shards, text=text)
            except MeshError:
                return None
        else:
            res = self._run_topn_batch((index, tuple(shards)), calls)
        if res is None or len(res) != len(calls) or any(r is None for r in res):
            return None
        return res

    def _run_count_batch(self, key, calls):
        index, shards, mesh = key
        if mesh:
            m = self.mesh
            if m is None:
                return None
            try:
                return m.count_batch(index, list(calls), list(shards))
            except MeshError:
                return None  # each call then runs alone (and reports its own error)
        if self.gpu is None:
            return None
        try:
            return self.gpu.try_count_batch(index, list(calls), list(shards))
        except PilosaError:
            raise
        except Exception as err:  # noqa: BLE001 - counted; each call then runs alone
            self._gpu_fault(err)
            return None

    def _has_remote(self, index, shards, opt) -> bool:
        if self.cluster is None or opt.remote:
            return False
        nodes = self.cluster.nodes
        me = self.cluster.node.id
        if len(nodes) == 1 and nodes[0].id == me:
            return False  # single node: every shard is local
        # placement depends only on (index, shards, membership, replicas):
        # memoised so the serving path does not re-hash every shard per request
        key = (index, tuple(shards), tuple(n.id for n in nodes), self.cluster.replica_n)
        memo = self.__dict__.setdefault("_remote_memo", {})
        hit = memo.get(key)
        if hit is None:
            hit = any(n.id != me for n in self._nodes_for(index, shards, opt))
            if len(memo) > 256:
                memo.clear()
            memo[key] = hit
        return hit

    def _nodes_for(self, index, shards, opt):
        nodes = set()
        for s in shards:
            owners = self.cluster.shard_nodes(index, s)
            if owners:
                nodes.add(owners[0])
        return nodes

    # ================================================================ dispatch
    def execute_call(self, index: str, c: Call, shards: List[int], opt: ExecOptions):
        self._validate_call_args(c)
        if self.stats is not None:
            self.stats.count_with_tags(c.name, 1, [f"index:{index}"])
        n = c.name
        with tracing.span(f"Executor.execute{n}"):
            if n == "Sum":
                return self._sum(index, c, shards, opt)
            if n == "Min":
                return self._minmax(index, c, shards, opt, "min")
            if n == "Max":
                return self._minmax(index, c, shards, opt, "max")
            if n == "MinRow":
                return self._minmax_row(index, c, shards, opt, True)
            if n == "MaxRow":
                return self._minmax_row(index, c, shards, opt, False)
            if n == "Clear":
                return self._clear_bit(index, c, opt)
            if n == "ClearRow":
                return self._clear_row(index, c, shards, opt)
            if n == "Store":
                return self._store(index, c, shards, opt)
            if n == "Count":
                return self._count(index, c, shards, opt)
            if n == "Set":
                return self._set(index, c, opt)
            if n == "SetRowAttrs":
                self._set_row_attrs(index, c, opt)
                return None
            if n == "SetColumnAttrs":
                self._set_column_attrs(index, c, opt)
                return None
            if n == "TopN":
                return self._topn(index, c, shards, opt)
            if n == "Rows":
                return self._rows(index, c, shards, opt)
            if n == "GroupBy":
                return self._group_by(index, c, shards, opt)
            if n == "Options":
                return self._options(index, c, shards, opt)
            return self._bitmap_call(index, c, shards, opt)

    @staticmethod
    def _validate_call_args(c: Call):
        if "ids" in c.args:
            v = c.args["ids"]
            if not isinstance(v, list) or not all(isinstance(x, int) and not isinstance(x, bool) for x in v):
                raise PilosaError(f"invalid call.Args[ids]: {v}")

    def _options(self, index, c: Call, shards, opt: ExecOptions):
        o = opt.copy()
        if "columnAttrs" in c.args:
            if not isinstance(c.args["columnAttrs"], bool):
                raise PilosaError("Query(): columnAttrs must be a bool")
            opt.column_attrs = c.args["columnAttrs"]
        for key, attr in (("excludeRowAttrs", "exclude_row_attrs"), ("excludeColumns", "exclude_columns")):
            if key in c.args:
                if not isinstance(c.args[key], bool):
                    raise PilosaError(f"Query(): {key} must be a bool")
                setattr(o, attr, c.args[key])
        if "shards" in c.args:
            v = c.args["shards"]
            if not isinstance(v, list) or not all(isinstance(s, int) and not isinstance(s, bool) for s in v):
                raise PilosaError("Query(): shards must be a list of unsigned integers")
            shards = [int(s) for s in v]
        if len(c.children) != 1:
            raise PilosaError("Options() requires exactly one child call")
        return self.execute_call(index, c.children[0], shards, o)

    # ================================================================ map/reduce
    def map_reduce(self, index: str, shards: List[int], c: Call, opt: ExecOptions, map_fn: Callable[[int], Any],
                   reduce_fn: Callable[[Any, Any], Any], local_fn: Optional[Callable[[List[int]], Any]] = None):
        """Group shards by owner node; local shards via ``local_fn`` (one
        batched GPU call) or the per-shard ``map_fn``; remote ones via the
        internal client with failover to replicas (executor.go:2458-2518)."""
        with tracing.span("Executor.mapReduce", call=c.name, shards=len(shards)):
            return self._map_reduce(index, shards, c, opt, map_fn, reduce_fn, local_fn)

    def _map_reduce(self, index, shards, c, opt, map_fn, reduce_fn, local_fn):
        by_node = self._shards_by_node(index, shards, opt)
        result = None
        # every remote node is queried at once (one request in flight per
        # node, like the reference's goroutine per node, executor.go:2530-2552)
        # while the local shards run here; the wall time is the slowest node's,
        # not the sum.  Partials are folded in node order (deterministic).
        remote = []
        if not opt.remote:
            for node, nshards in by_node.items():
                if node is not None and (self.cluster is None or node.id != self.cluster.node.id):
                    remote.append(self.fanout.submit(tracing.bind(self._remote_with_failover), index, c, node,
                                                     nshards, opt, map_fn, reduce_fn, local_fn, {node.id}))
        for node, nshards in by_node.items():
            if node is None or (self.cluster is not None and node.id == self.cluster.node.id):
                if self._use_mesh(opt):
                    mesh = self.mesh
                    try:
                        result = reduce_fn(result, mesh.map_local(index, c, nshards, opt, reduce_fn))
                        continue
                    except MeshError:
                        if not mesh.failed_over:
                            raise
                        # failed over: this process now holds every local shard
                with tracing.span("Executor.mapperLocal", shards=len(nshards)):
                    result = reduce_fn(result, self._map_local(nshards, map_fn, reduce_fn, local_fn))
        for fut in remote:
            result = reduce_fn(result, fut.result())
        return result

    @property
    def fanout(self) -> cf.ThreadPoolExecutor:
        """Threads that carry the remote node requests of map/reduce (and
        their replica retries); separate from the shard pool so a fan-out
        never waits behind local shard jobs."""
        pool = self.__dict__.get("_fanout")
        if pool is None:
            with _FANOUT_LOCK:
                pool = self.__dict__.get("_fanout")
                if pool is None:
                    pool = cf.ThreadPoolExecutor(max_workers=32, thread_name_prefix="fanout")
                    self._fanout = pool
        return pool

    def _use_mesh(self, opt) -> bool:
        mesh = self.mesh
        return mesh is not None and (mesh.world > 1 or getattr(mesh, "always", False)) and \
            not getattr(opt, "mesh_local", False)

    def _shards_by_node(self, index, shards, opt) -> Dict[Any, List[int]]:
        if self.cluster is None or opt.remote:
            return {None: list(shards)}
        out: Dict[Any, List[int]] = {}
        for s in shards:
            owners = self.cluster.shard_nodes(index, s)
            live = [n for n in owners if n.state != "DOWN"] or owners
            # prefer the local replica, then the first live owner
            node = next((n for n in live if n.id == self.cluster.node.id), live[0] if live else None)
            out.setdefault(node, []).append(s)
        return out

    def _remote_with_failover(self, index, c, node, nshards, opt, map_fn, reduce_fn, local_fn, tried):
        try:
            with tracing.span("Executor.remoteExec", node=node.id, shards=len(nshards)):
                results = self.client.query_node(node, index, str(c), nshards)
            return results[0] if results else None
        except Exception as err:  # noqa: BLE001 - retry on replicas
            result = None
            regroup: Dict[Any, List[int]] = {}
            for s in nshards:
                cands = [n for n in self.cluster.shard_nodes(index, s) if n.id not in tried]
                if not cands:
                    raise err
                regroup.setdefault(cands[0], []).append(s)
            # the failed node's shards, regrouped by their next replica.  The
            # retries run inline on this worker: this call already holds a
            # fan-out thread, and waiting on futures queued to the same pool
            # starves it when many remote calls fail together (a node dying
            # under load), hanging every map/reduce on the node.
            for n2, ss in regroup.items():
                if n2.id == self.cluster.node.id:
                    part = self._map_local(ss, map_fn, reduce_fn, local_fn)
                else:
                    part = self._remote_with_failover(index, c, n2, ss, opt, map_fn, reduce_fn, local_fn,
                                                      tried | {n2.id})
                result = reduce_fn(result, part)
            return result

    def _map_local(self, shards: List[int], map_fn, reduce_fn, local_fn):
        if local_fn is not None and self.gpu is not None and shards:
            try:
                r = local_fn(shards)
            except NotImplementedError:
                r = NotImplemented
            except PilosaError:
                raise
            except Exception as err:  # noqa: BLE001 - device fault: the host fragments answer
                self._gpu_fault(err)
                r = NotImplemented
            if r is not NotImplemented:
                if self.paranoia:
                    want = self._map_host(shards, map_fn, reduce_fn)
                    if not _results_equal(r, want):
                        raise AssertionError(f"paranoia: device result {r!r} != host result {want!r}")
                return r
        return self._map_host(shards, map_fn, reduce_fn)

    def _map_host(self, shards: List[int], map_fn, reduce_fn):
        result = None
        if len(shards) <= 1:
            for s in shards:
                result = reduce_fn(result, map_fn(s))
            return result
        futs = [self.pool.submit(map_fn, s) for s in shards]
        for f in futs:
            result = reduce_fn(result, f.result())
        return result

    def _gpu_fault(self, err: BaseException):
        """A device call failed (HIP error, lost device, out of memory): the
        query falls back to the host fragments, which are the source of truth
        (SURVEY §5.3); after GPU_FAULT_LIMIT faults the device is detached and
        the node keeps serving from the host path."""
        self.gpu_faults += 1
        if self.stats is not None:
            self.stats.count("gpuFault", 1)
        DEVICE_FAULTS[0] += 1
        if self.strict_gpu or os.environ.get("PILOSA_GPU_STRICT", "0") == "1":
            raise err
        if self.logger is not None:
            self.logger.printf("gpu fault %d (%s: %s), answering from host fragments", self.gpu_faults,
                               type(err).__name__, err)
        if self.gpu_faults >= GPU_FAULT_LIMIT and self.gpu is not None:
            if self.logger is not None:
                self.logger.printf("gpu detached after %d faults", self.gpu_faults)
            self.gpu = None

    # ================================================================ bitmap calls
    def _bitmap_call(self, index: str, c: Call, shards, opt: ExecOptions) -> Row:
        def reduce_fn(prev, v):
            if prev is None:
                prev = Row()
            if v is not None:
                prev.merge(v)
            return prev

        local = (lambda ss: self.gpu.bitmap(index, c, ss)) if self.gpu is not None else None
        try:
            row = self.map_reduce(index, shards, c, opt, lambda s: self.bitmap_call_shard(index, c, s), reduce_fn,
                                  local) or Row()
        except PilosaError as e:
            raise wrap(e, "map reduce") from e   # executor.go:606
        if c.name == "Row" and not c.has_condition_arg():
            if opt.exclude_row_attrs:
                row.attrs = {}
            else:
                idx = self.holder.index(index)
                if "_col" in c.args:
                    row.attrs = idx.column_attr_store.attrs(c.uint_arg("_col")[0]) or {}
                else:
                    fname = c.field_arg()
                    f = idx.field(fname)
                    if f is not None:
                        rid, _ = c.uint_arg(fname)
                        row.attrs = f.row_attr_store.attrs(rid) or {}
        if opt.exclude_columns:
            row.segments = {}
        return row

    def bitmap_call_shard(self, index: str, c: Call, shard: int) -> Row:
        n = c.name
        if n in ("Row", "Range", "Bitmap"):
            return self._row_shard(index, c, shard)
        if n == "Difference":
            if not c.children:
                raise PilosaError("empty Difference query is currently not supported")
            out = None
            for i, ch in enumerate(c.children):
                r = self.bitmap_call_shard(index, ch, shard)
                out = r if i == 0 else out.difference(r)
            return out
        if n == "Intersect":
            if not c.children:
                raise PilosaError("empty Intersect query is currently not supported")
            out = None
            for i, ch in enumerate(c.children):
                r = self.bitmap_call_shard(index, ch, shard)
                out = r if i == 0 else out.intersect(r)
            return out
        if n == "Union":
            rows = [self.bitmap_call_shard(index, ch, shard) for ch in c.children]
            if not rows:
                return Row()
            return rows[0].union(*rows[1:]) if len(rows) > 1 else rows[0]
        if n == "Xor":
            out = Row()
            for i, ch in enumerate(c.children):
                r = self.bitmap_call_shard(index, ch, shard)
                out = r if i == 0 else out.xor(r)
            return out
        if n == "Not":
            if not c.children:
                raise PilosaError("Not() requires an input row")
            if len(c.children) > 1:
                raise PilosaError("Not() only accepts a single row input")
            idx = self.holder.index(index)
            if idx is None:
                raise ErrIndexNotFound
            if idx.existence_field() is None:
                raise PilosaError(f"index does not support existence tracking: {index}")
            ef = self.holder.fragment(index, EXISTENCE_FIELD_NAME, VIEW_STANDARD, shard)
            ex = ef.row(0) if ef is not None else Row()
            return ex.difference(self.bitmap_call_shard(index, c.children[0], shard))
        if n == "Shift":
            k, _ = c.int_arg("n")
            if not c.children:
                raise PilosaError("Shift() requires an input row")
            if len(c.children) > 1:
                raise PilosaError("Shift() only accepts a single row input")
            if k < 0:
                raise PilosaError("cannot shift by negative values")
            r = self.bitmap_call_shard(index, c.children[0], shard)
            return r.shift(k)
        raise PilosaError(f"unknown call: {n}")

    def time_views(self, f, c: Call) -> Optional[List[str]]:
        """Views to union for a Row/Range with from/to, or None for standard."""
        from_t = parse_time(c.args["from"]) if "from" in c.args else None
        to_t = parse_time(c.args["to"]) if "to" in c.args else None
        if c.name == "Row" and from_t is None and to_t is None:
            return None
        q = f.time_quantum()
        if not q:
            return []
        if to_t is None:
            to_t = dt.datetime.utcnow() + dt.timedelta(days=1)
        if from_t is None:
            from_t = dt.datetime(1, 1, 1)
        return views_by_time_range(VIEW_STANDARD, from_t, to_t, q)

    def _row_shard(self, index: str, c: Call, shard: int) -> Row:
        if c.has_condition_arg():
            return self._row_bsi_shard(index, c, shard)
        idx = self.holder.index(index)
        if idx is None:
            raise ErrIndexNotFound
        try:
            fname = c.field_arg()
        except ValueError:
            raise PilosaError("Row() argument required: field")
        f = idx.field(fname)
        if f is None:
            raise ErrFieldNotFound
        try:
            rid, ok = c.uint_arg(fname)
        except ValueError as e:
            raise PilosaError(f"Row() error with arg for row: {e}")
        if not ok:
            raise PilosaError("Row() must specify row")
        views = self.time_views(f, c)
        if views is None:
            frag = self.holder.fragment(index, fname, VIEW_STANDARD, shard)
            return frag.row(rid) if frag is not None else Row()
        if f.stats is not None:
            f.stats.count("range", 1)   # executor.go:1530
        rows = []
        for v in views:
            frag = self.holder.fragment(index, fname, v, shard)
            if frag is not None:
                rows.append(frag.row(rid))
        if not rows:
            return Row()
        return rows[0].union(*rows[1:]) if len(rows) > 1 else rows[0]

    def bsi_predicate(self, index: str, c: Call):
        """Resolve a BSI condition into (field, bsig, kind, args) where kind is
        one of 'empty', 'notnull', 'between', 'op' (executor.go:1536-1665)."""
        if len(c.args) == 0:
            raise PilosaError("Row(): condition required")
        if len(c.args) > 1:
            raise PilosaError("Row(): too many arguments")
        (fname, cond), = c.args.items()
        if not isinstance(cond, Condition):
            raise PilosaError(f'Row(): "{fname}": expected condition argument, got {cond}')
        f = self.holder.field(index, fname)
        if f is None:
            raise ErrFieldNotFound
        b = f.bsi_group(fname)
        if cond.op == NEQ and cond.value is None:
            if b is None:
                raise ErrBSIGroupNotFound
            return f, b, "notnull", ()
        if cond.op == BETWEEN:
            try:
                preds = cond.int_slice_value()
            except ValueError as e:
                raise PilosaError(f"getting condition value: {e}")
            if len(preds) != 2:
                raise PilosaError("Row(): BETWEEN condition requires exactly two integer values")
            if b is None:
                raise ErrBSIGroupNotFound
            lo, hi, oor = b.base_value_between(preds[0], preds[1])
            if oor:
                return f, b, "empty", ()
            if preds[0] <= b.min and preds[1] >= b.max:
                return f, b, "notnull", ()
            return f, b, "between", (lo, hi)
        value = cond.value
        if isinstance(value, bool) or not isinstance(value, int):
            raise PilosaError("Row(): conditions only support integer values")
        if b is None:
            raise ErrBSIGroupNotFound
        bv, oor = b.base_value(cond.op, value)
        if oor and cond.op != NEQ:
            return f, b, "empty", ()
        op = cond.op
        if (op == LT and value > b.max) or (op == LTE and value >= b.max) or \
                (op == GT and value < b.min) or (op == GTE and value <= b.min):
            return f, b, "notnull", ()
        if oor and op == NEQ:
            return f, b, "notnull", ()
        return f, b, "op", (op, bv)

    def _row_bsi_shard(self, index: str, c: Call, shard: int) -> Row:
        f, b, kind, args = self.bsi_predicate(index, c)
        if kind == "empty":
            return Row()
        frag = self.holder.fragment(index, f.name, VIEW_BSI_PREFIX + f.name, shard)
        if frag is None:
            return Row()
        if f.stats is not None:
            f.stats.count("range:bsigroup", 1)   # executor.go:1662
        if kind == "notnull":
            return frag.not_null()
        if kind == "between":
            return frag.range_between(b.bit_depth, args[0], args[1])
        return frag.range_op(args[0], b.bit_depth, args[1])

    # ================================================================ aggregates
    def _count(self, index: str, c: Call, shards, opt) -> int:
        if not c.children:
            raise PilosaError("Count() requires an input bitmap")
        if len(c.children) > 1:
            raise PilosaError("Count() only accepts a single bitmap input")
        child = c.children[0]
        local = (lambda ss: self.gpu.count(index, child, ss)) if self.gpu is not None else None
        r = self.map_reduce(index, shards, c, opt, lambda s: self.count_shard(index, child, s),
                            lambda p, v: (p or 0) + (v or 0), local)
        return int(r or 0)

    def count_host(self, index: str, child: Call, shards) -> int:
        """Count on the host roaring path only (GPU-ineligible trees)."""
        return int(self._map_local(list(shards), lambda s: self.count_shard(index, child, s),
                                   lambda p, v: (p or 0) + (v or 0), None) or 0)

    def _plain_row(self, index: str, c: Call):
        """(field, row id, covering views or None) for a plain Row(f=id) /
        time Row, or None when the call needs the general path (conditions,
        keys, missing fields, bad arguments: their errors come from there)."""
        if c.name != "Row" or c.children or c.has_condition_arg():
            return None
        idx = self.holder.index(index)
        if idx is None:
            return None
        try:
            fname = c.field_arg()
            rid, ok = c.uint_arg(fname)
        except (ValueError, PilosaError):
            return None
        f = idx.field(fname)
        if f is None or not ok or not isinstance(rid, int) or rid < 0:
            return None
        try:
            views = self.time_views(f, c)
        except Exception:  # noqa: BLE001 - malformed times: the general path reports them
            return None
        return fname, rid, views

    def count_shard(self, index: str, child: Call, shard: int) -> int:
        """Count(child) on one shard from the host fragments.

        Count(Row) reads the row's cardinality, Count(Row with from/to) counts
        the union of the covering views, and Count(Intersect(Row, Row)) counts
        the two rows in place -- no row is extracted or intersected
        (reference executeCount -> executeBitmapCallShard -> Row.Count,
        executor.go:728-760).  Anything else runs the general row path."""
        if child.name == "Row":
            pr = self._plain_row(index, child)
            if pr is not None:
                fname, rid, views = pr
                if views is None:
                    frag = self.holder.fragment(index, fname, VIEW_STANDARD, shard)
                    return frag.row_count(rid) if frag is not None else 0
                frags = [fr for fr in (self.holder.fragment(index, fname, v, shard) for v in views)
                         if fr is not None]
                if len(frags) == 1:
                    return frags[0].row_count(rid)
                if frags:
                    locks = sorted(frags, key=id)
                    for fr in locks:
                        fr.mu.acquire()
                    try:
                        return _roaring.Bitmap.range_union_count(
                            [(fr.storage, rid * SHARD_WIDTH) for fr in frags], SHARD_WIDTH)
                    finally:
                        for fr in reversed(locks):
                            fr.mu.release()
                return 0
        elif child.name == "Intersect" and len(child.children) == 2:
            a = self._plain_row(index, child.children[0])
            b = self._plain_row(index, child.children[1])
            if a is not None and b is not None and a[2] is None and b[2] is None:
                fa = self.holder.fragment(index, a[0], VIEW_STANDARD, shard)
                fb = self.holder.fragment(index, b[0], VIEW_STANDARD, shard)
                if fa is None or fb is None:
                    return 0
                return fa.row_intersection_count(a[1], fb, b[1])
        return self.bitmap_call_shard(index, child, shard).count()

    def _bsi_filter_shard(self, index, c: Call, shard):
        if len(c.children) == 1:
            return self.bitmap_call_shard(index, c.children[0], shard)
        return None

    def _sum(self, index: str, c: Call, shards, opt) -> ValCount:
        fname = c.args.get("field")
        if not fname:
            raise PilosaError("Sum(): field required")
        if len(c.children) > 1:
            raise PilosaError("Sum() only accepts a single bitmap input")

        def map_fn(shard):
            f = self.holder.field(index, fname)
            if f is None or f.bsi_group(fname) is None:
                return ValCount()
            b = f.bsi_group(fname)
            frag = self.holder.fragment(index, fname, VIEW_BSI_PREFIX + fname, shard)
            if frag is None:
                return ValCount()
            s, n = frag.sum(self._bsi_filter_shard(index, c, shard), b.bit_depth)
            return ValCount(_wrap(s + n * b.base), n)

        local = (lambda ss: self.gpu.bsi_sum(index, c, ss)) if self.gpu is not None else None
        r = self.map_reduce(index, shards, c, opt, map_fn, lambda p, v: (p or ValCount()).add(v or ValCount()),
                            local)
        r = r or ValCount()
        return r if r.count else ValCount()

    def _minmax(self, index: str, c: Call, shards, opt, which: str) -> ValCount:
        fname = c.args.get("field")
        name = "Min" if which == "min" else "Max"
        if not fname:
            raise PilosaError(f"{name}(): field required")
        if len(c.children) > 1:
            raise PilosaError(f"{name}() only accepts a single bitmap input")

        def map_fn(shard):
            f = self.holder.field(index, fname)
            if f is None or f.bsi_group(fname) is None:
                return ValCount()
            b = f.bsi_group(fname)
            frag = self.holder.fragment(index, fname, VIEW_BSI_PREFIX + fname, shard)
            if frag is None:
                return ValCount()
            filt = self._bsi_filter_shard(index, c, shard)
            v, n = frag.min(filt, b.bit_depth) if which == "min" else frag.max(filt, b.bit_depth)
            return ValCount(v + b.base, n)

        if which == "min":
            red = lambda p, v: (p or ValCount()).smaller(v or ValCount())  # noqa: E731
        else:
            red = lambda p, v: (p or ValCount()).larger(v or ValCount())  # noqa: E731

        def local(ss):
            return self.gpu.bsi_minmax(index, c, ss, which)   # already folded over ss
        r = self.map_reduce(index, shards, c, opt, map_fn, red, local if self.gpu is not None else None) or ValCount()
        return r if r.count else ValCount()

    def _minmax_row(self, index: str, c: Call, shards, opt, is_min: bool) -> Pair:
        fname = c.args.get("field")
        if not fname:
            raise PilosaError(f"{'MinRow' if is_min else 'MaxRow'}(): field required")

        def map_fn(shard):
            if self.holder.field(index, fname) is None:
                return Pair(0, 0)
            frag = self.holder.fragment(index, fname, VIEW_STANDARD, shard)
            if frag is None:
                return Pair(0, 0)
            filt = self._bsi_filter_shard(index, c, shard)
            rid, cnt = frag.min_row(filt) if is_min else frag.max_row(filt)
            return Pair(rid, cnt)

        def red(p, v):
            p = p or Pair(0, 0)
            v = v or Pair(0, 0)
            if p.count > 0 and v.count > 0:
                if is_min:
                    return p if p.id < v.id else v
                return p if p.id > v.id else v
            return p if p.count > 0 else v

        local = (lambda ss: self.gpu.minmax_row(index, c, ss, is_min)) if self.gpu is not None else None
        return self.map_reduce(index, shards, c, opt, map_fn, red, local) or Pair(0, 0)

    # ================================================================ TopN
    def _topn(self, index: str, c: Call, shards, opt) -> List[Pair]:
        ids, has_ids = c.uint_slice_arg("ids")
        n, _ = c.uint_arg("n")
        pairs = self._topn_shards(index, c, shards, opt)
        if not pairs or has_ids or opt.remote:
            return pairs
        other = c.clone()
        other.args["ids"] = sorted(p.id for p in pairs)
        trimmed = self._topn_shards(index, other, shards, opt)
        if n and n < len(trimmed):
            trimmed = trimmed[:n]
        return trimmed

    def _topn_shards(self, index, c: Call, shards, opt) -> List[Pair]:
        local = (lambda ss: self.gpu.topn(index, c, ss)) if self.gpu is not None else None
        r = self.map_reduce(index, shards, c, opt, lambda s: self._topn_shard(index, c, s),
                            lambda p, v: pairs_add(p or [], v or []), local)
        return sort_pairs(r or [])

    _TOPN_PLAIN_ARGS = frozenset(("_field", "n", "threshold"))

    def topn_params(self, index: str, c: Call):
        a = c.args
        if not c.children and a.keys() <= self._TOPN_PLAIN_ARGS:
            # TopN(f, n=.., threshold=..): the common serving shape, without
            # the generic argument accessors (16 of these per request)
            n, th = a.get("n", 0), a.get("threshold", 0)
            if type(n) is int and type(th) is int and n >= 0 and th >= 0:
                fname = a.get("_field") or DEFAULT_FIELD
                f = self.holder.field(index, fname)
                if f is not None and f.type == FIELD_TYPE_INT:
                    raise PilosaError(f'cannot compute TopN() on integer field: "{fname}"')
                return fname, n, [], th or DEFAULT_MIN_THRESHOLD, 0, "", []
        fname = c.args.get("_field") or DEFAULT_FIELD
        n, _ = c.uint_arg("n")
        f = self.holder.field(index, fname)
        if f is not None and f.type == FIELD_TYPE_INT:
            raise PilosaError(f'cannot compute TopN() on integer field: "{fname}"')
        ids, _ = c.uint_slice_arg("ids")
        threshold, _ = c.uint_arg("threshold")
        tanimoto, _ = c.uint_arg("tanimotoThreshold")
        if tanimoto > 100:
            raise PilosaError("Tanimoto Threshold is from 1 to 100 only")
        if len(c.children) > 1:
            raise PilosaError("TopN() can only have one input bitmap")
        attr_name = c.args.get("attrName", "")
        attr_values = c.args.get("attrValues") or []
        return fname, n, ids or [], threshold or DEFAULT_MIN_THRESHOLD, tanimoto, attr_name, attr_values

    def _topn_shard(self, index: str, c: Call, shard: int) -> List[Pair]:
        fname, n, ids, threshold, tanimoto, attr_name, attr_values = self.topn_params(index, c)
        src = self.bitmap_call_shard(index, c.children[0], shard) if len(c.children) == 1 else None
        frag = self.holder.fragment(index, fname, VIEW_STANDARD, shard)
        if frag is None:
            return []
        if frag.cache_type == "none":
            raise PilosaError(f'cannot compute TopN(), field has no cache: "{fname}"')
        f = self.holder.field(index, fname)
        return frag.top(TopOptions(n=n, src=src, row_ids=ids, min_threshold=threshold, filter_name=attr_name,
                                   filter_values=attr_values, tanimoto_threshold=tanimoto,
                                   attr_store=f.row_attr_store if f is not None else None))

    # ================================================================ Rows / GroupBy
    def _rows(self, index: str, c: Call, shards, opt) -> List[int]:
        if isinstance(c.args.get("field"), str):
            c.args["_field"] = c.args["field"]
        fname = c.args.get("_field")
        if not isinstance(fname, str):
            raise PilosaError("Rows() field required")
        col, has_col = c.uint_arg("column")
        if has_col:
            shards = [col // SHARD_WIDTH]
        lim, has_lim = c.uint_arg("limit")
        limit = lim if has_lim else MAX_INT
        local = (lambda ss: self.gpu.rows(index, fname, c, ss)) if self.gpu is not None else None
        r = self.map_reduce(index, shards, c, opt, lambda s: self._rows_shard(index, fname, c, s),
                            lambda p, v: merge_row_ids(p or [], v or [], limit), local)
        return r or []

    def _rows_shard(self, index: str, fname: str, c: Call, shard: int) -> List[int]:
        if self.holder.index(index) is None:
            raise ErrIndexNotFound
        f = self.holder.field(index, fname)
        if f is None:
            raise ErrFieldNotFound
        views = self.rows_views(f, c)
        start = 0
        prev, has_prev = c.uint_arg("previous")
        if has_prev:
            start = prev + 1
        col, has_col = c.uint_arg("column")
        if has_col and col // SHARD_WIDTH != shard:
            return []
        lim, has_lim = c.uint_arg("limit")
        limit = lim if has_lim else MAX_INT
        out: List[int] = []
        for v in views:
            frag = self.holder.fragment(index, fname, v, shard)
            if frag is None:
                continue
            rows = frag.rows(start, column=col if has_col else None, limit=limit if has_lim else None)
            out = merge_row_ids(out, rows, limit)
        return out

    def rows_views(self, f, c: Call) -> List[str]:
        """Views a Rows() call lists: standard, or the covering time views of
        its from/to range clamped to the field's existing views
        (executor.go:1071-1155)."""
        views = [VIEW_STANDARD]
        if f.type == FIELD_TYPE_TIME:
            from_t = parse_time(c.args["from"]) if "from" in c.args else None
            to_t = parse_time(c.args["to"]) if "to" in c.args else None
            if from_t is not None or to_t is not None or f.options.no_standard_view:
                q = f.time_quantum()
                if not q:
                    return []
                mn, mx = min_max_views(list(f.views), q)
                if not mn or not mx:
                    return []
                min_t, max_t = time_of_view(mn, False), time_of_view(mx, True)
                if from_t is None or from_t < min_t:
                    from_t = min_t
                if to_t is None or to_t > max_t:
                    to_t = max_t
                views = views_by_time_range(VIEW_STANDARD, from_t, to_t, q)
        return views

    def _group_by(self, index: str, c: Call, shards, opt) -> List[GroupCount]:
        if not c.children:
            raise PilosaError("need at least one child call")
        lim, has_lim = c.uint_arg("limit")
        limit = lim if has_lim else MAX_INT
        filt, _ = c.call_arg("filter")
        child_rows: List[Optional[List[int]]] = []
        for ch in c.children:
            if isinstance(ch.args.get("field"), str):
                ch.args["_field"] = ch.args["field"]
            if ch.name != "Rows":
                raise PilosaError(f"'{ch.name}' is not a valid child query for GroupBy, must be 'Rows'")
            _, hl = ch.uint_arg("limit")
            _, hc = ch.uint_arg("column")
            if hl or hc:
                rows = self._rows(index, ch, shards, opt)
                if not rows:
                    return []
                child_rows.append(rows)
            else:
                child_rows.append(None)
        previous = c.args.get("previous")
        local = (lambda ss: self.gpu.group_by(index, c, filt, ss, child_rows, limit)) if self.gpu is not None \
            else None
        r = self.map_reduce(index, shards, c, opt,
                            lambda s: self._group_by_shard(index, c, filt, s, child_rows, limit),
                            lambda p, v: merge_group_counts(p or [], v or [], limit), local) or []
        off, has_off = c.uint_arg("offset")
        if has_off and off < len(r):
            r = r[off:]
        if has_lim and limit < len(r):
            r = r[:limit]
        return r

    def group_by_candidates(self, index: str, c: Call, shard: int, child_rows) -> Optional[List[List[int]]]:
        """Per field, the candidate row ids in this shard (None if a field's
        fragment is missing, which makes the shard contribute nothing)."""
        out = []
        for i, ch in enumerate(c.children):
            fname = ch.args.get("_field")
            if not isinstance(fname, str):
                raise PilosaError(f"{ch.name} call must have field with valid (string) field name")
            if self.holder.field(index, fname) is None:
                raise ErrFieldNotFound
            frag = self.holder.fragment(index, fname, VIEW_STANDARD, shard)
            if frag is None:
                return None
            rows = frag.rows(0, row_filter=child_rows[i])
            out.append(rows)
        return out

    @staticmethod
    def group_by_start(c: Call) -> Optional[Tuple[Optional[int], ...]]:
        """Paging start of a GroupBy, or None (no paging).

        Reference groupByIterator (executor.go:3085-3145): a child with
        ``previous=p`` seeks its row iterator to p (the last child to p + 1);
        a child without it starts at its first row; a child whose seek lands
        past p makes the deeper children start from their first row, and
        deeper iterators wrap.  So a shard returns the keys lexicographically
        >= start, with start_i = p_i (last: p + 1) and, for children without
        ``previous`` (None here), that shard's first row of the field
        (resolve_group_start)."""
        k = len(c.children)
        prev = c.args.get("previous")
        if prev is not None:
            if not isinstance(prev, list):
                raise PilosaError(f"'previous' argument must be list, but got {type(prev).__name__}")
            if len(prev) != k:
                raise PilosaError(f"mismatched lengths for previous: {len(prev)} and children: {k}")
            ps = [int(x) for x in prev]
            return tuple(ps[:-1]) + (ps[-1] + 1,)
        start: List[Optional[int]] = []
        any_prev = False
        for i, ch in enumerate(c.children):
            p, ok = ch.uint_arg("previous")
            any_prev |= ok
            start.append((p + 1 if i == k - 1 else p) if ok else None)
        return tuple(start) if any_prev else None

    @staticmethod
    def resolve_group_start(start, cands) -> Optional[Tuple[int, ...]]:
        """group_by_start with each None replaced by the field's first
        candidate row (sorted candidates per field)."""
        if start is None:
            return None
        return tuple(s if s is not None else (int(cands[i][0]) if len(cands[i]) else -1)
                     for i, s in enumerate(start))

    def _group_by_shard(self, index: str, c: Call, filt: Optional[Call], shard: int, child_rows, limit):
        cands = self.group_by_candidates(index, c, shard, child_rows)
        if cands is None or any(len(x) == 0 for x in cands):
            return []
        filt_row = self.bitmap_call_shard(index, filt, shard) if filt is not None else None
        fields = [ch.args["_field"] for ch in c.children]
        start = self.resolve_group_start(self.group_by_start(c), cands)
        frags = [self.holder.fragment(index, f, VIEW_STANDARD, shard) for f in fields]
        results: List[GroupCount] = []
        k = len(fields)

        def rec(level: int, acc: Optional[Row], prefix: Tuple[int, ...]):
            for rid in cands[level]:
                key = prefix + (rid,)
                if start is not None and key < start[:len(key)]:
                    continue
                r = frags[level].row(rid)
                if level == 0 and filt_row is not None:
                    r = r.intersect(filt_row)
                cur = r if acc is None else acc.intersect(r)
                if cur.is_empty():
                    continue
                if level == k - 1:
                    results.append(GroupCount([FieldRow(fields[i], key[i]) for i in range(k)], cur.count()))
                    if len(results) >= limit:
                        return True
                else:
                    if rec(level + 1, cur, key):
                        return True
            return False

        rec(0, None, ())
        return results

    # ================================================================ writes
    def _shard_owned_locally(self, index, shard) -> List[Any]:
        if self.cluster is None:
            return [None]
        return self.cluster.shard_nodes(index, shard)

    def _forward_write(self, index, c: Call, shard, opt, local_fn) -> bool:
        ret = False
        for node in self._shard_owned_locally(index, shard):
            if node is None or node.id == self.cluster.node.id:
                if self._use_mesh(opt) and self.mesh.owner(shard) != self.mesh.rank:
                    if self.mesh.forward_write(index, c, shard, opt):
                        ret = True
                elif local_fn():
                    ret = True
                continue
            if opt.remote:
                continue
            res = self.client.query_node(node, index, str(c), None)
            ret = bool(res[0]) if res else ret
        return ret

    def _set(self, index: str, c: Call, opt) -> bool:
        try:
            col, ok = c.uint_arg("_col")
        except ValueError as e:
            raise PilosaError(f"reading Set() column: {e}")
        if not ok:
            raise PilosaError("Set() column argument 'col' required")
        try:
            fname = c.field_arg()
        except ValueError:
            raise PilosaError("Set() argument required: field")
        idx = self.holder.index(index)
        if idx is None:
            raise ErrIndexNotFound
        f = idx.field(fname)
        if f is None:
            raise ErrFieldNotFound
        shard = col // SHARD_WIDTH
        ef = idx.existence_field()
        if f.type == FIELD_TYPE_INT:
            try:
                val, ok = c.int_arg(fname)
            except ValueError as e:
                raise PilosaError(f"reading Set() row: {e}")
            if not ok:
                raise PilosaError("Set() row argument 'row' required")

            def local():
                if ef is not None:
                    ef.set_bit(0, col)
                return f.set_value(col, val)
            return self._forward_write(index, c, shard, opt, local)
        try:
            rid, ok = c.uint_arg(fname)
        except ValueError as e:
            raise PilosaError(f"reading Set() row: {e}")
        if not ok:
            raise PilosaError("Set() row argument 'row' required")
        ts = None
        if isinstance(c.args.get("_timestamp"), str):
            try:
                ts = dt.datetime.strptime(c.args["_timestamp"], TIME_FORMAT)
            except ValueError:
                raise PilosaError(f"invalid date: {c.args['_timestamp']}")

        def local():
            if ef is not None:
                ef.set_bit(0, col)
            return f.set_bit(rid, col, ts)
        return self._forward_write(index, c, shard, opt, local)

    def _clear_bit(self, index: str, c: Call, opt) -> bool:
        try:
            fname = c.field_arg()
        except ValueError:
            raise PilosaError("Clear() argument required: field")
        idx = self.holder.index(index)
        if idx is None:
            raise ErrIndexNotFound
        f = idx.field(fname)
        if f is None:
            raise ErrFieldNotFound
        try:
            rid, ok = c.uint_arg(fname) if f.type != FIELD_TYPE_INT else c.int_arg(fname)
        except ValueError as e:
            raise PilosaError(f"reading Clear() row: {e}")
        if not ok:
            raise PilosaError("row=<row> argument required to Clear() call")
        col, ok = c.uint_arg("_col")
        if not ok:
            raise PilosaError("column argument to Clear(<COLUMN>, <FIELD>=<ROW>) required")
        shard = col // SHARD_WIDTH
        if f.type == FIELD_TYPE_INT:
            return self._forward_write(index, c, shard, opt, lambda: f.clear_value(col))
        return self._forward_write(index, c, shard, opt, lambda: f.clear_bit(rid, col))

    def _clear_row(self, index: str, c: Call, shards, opt) -> bool:
        try:
            fname = c.field_arg()
        except ValueError:
            raise PilosaError("ClearRow() argument required: field")
        f = self.holder.field(index, fname)
        if f is None:
            raise ErrFieldNotFound
        if f.type not in (FIELD_TYPE_SET, FIELD_TYPE_TIME, "mutex", FIELD_TYPE_BOOL):
            raise PilosaError(f"ClearRow() is not supported on {f.type} field types")
        rid, ok = c.uint_arg(fname)
        if not ok:
            raise PilosaError("ClearRow() row argument 'row' required")

        def map_fn(shard):
            changed = False
            for vname in list(f.views):
                frag = self.holder.fragment(index, fname, vname, shard)
                if frag is not None:
                    changed = frag.clear_row(rid) or changed
            return changed

        r = self.map_reduce(index, shards, c, opt, map_fn, lambda p, v: bool(p) or bool(v))
        return bool(r)

    def _store(self, index: str, c: Call, shards, opt) -> bool:
        try:
            fname = c.field_arg()
        except ValueError:
            raise PilosaError("field required for Store()")
        f = self.holder.field(index, fname)
        if f is None:
            raise ErrFieldNotFound
        if f.type != FIELD_TYPE_SET:
            raise PilosaError(f"can't Store() on a {f.type} field")
        rid, ok = c.uint_arg(fname)
        if not ok:
            raise PilosaError("need the <FIELD>=<ROW> argument on Store()")
        if len(c.children) != 1:
            raise PilosaError("Store() requires a source row")

        def map_fn(shard):
            src = self.bitmap_call_shard(index, c.children[0], shard)
            frag = f.create_view_if_not_exists(VIEW_STANDARD).create_fragment_if_not_exists(shard)
            return frag.set_row(src, rid)

        return bool(self.map_reduce(index, shards, c, opt, map_fn, lambda p, v: bool(p) or bool(v)))

    def _broadcast_call(self, index, calls: List[Call], opt):
        if opt.remote or self.cluster is None:
            return
        q = "\n".join(str(c) for c in calls)
        for node in self.cluster.nodes:
            if node.id == self.cluster.node.id:
                continue
            self.client.query_node(node, index, q, None)

    def _set_row_attrs(self, index: str, c: Call, opt):
        fname = c.args.get("_field")
        if not isinstance(fname, str):
            raise PilosaError("SetRowAttrs() field required")
        f = self.holder.field(index, fname)
        if f is None:
            raise ErrFieldNotFound
        rid, ok = c.uint_arg("_row")
        if not ok:
            raise PilosaError("SetRowAttrs() row field 'row' required")
        attrs = {k: v for k, v in c.args.items() if k not in ("_field", "_row")}
        f.row_attr_store.set_attrs(rid, attrs)
        if f.stats is not None:
            f.stats.count("SetRowAttrs", 1)   # executor.go:2242
        self._broadcast_call(index, [c], opt)

    def _bulk_set_row_attrs(self, index, calls: List[Call], opt):
        m: Dict[str, Dict[int, dict]] = {}
        for c in calls:
            fname = c.args.get("_field")
            if not isinstance(fname, str):
                raise PilosaError("SetRowAttrs() field required")
            if self.holder.field(index, fname) is None:
                raise ErrFieldNotFound
            rid, ok = c.uint_arg("_row")
            if not ok:
                raise PilosaError("SetRowAttrs row field 'row' required")
            attrs = {k: v for k, v in c.args.items() if k not in ("_field", "_row")}
            m.setdefault(fname, {}).setdefault(rid, {}).update(attrs)
        for fname, fm in m.items():
            f = self.holder.field(index, fname)
            f.row_attr_store.set_bulk_attrs(fm)
            if f.stats is not None:
                f.stats.count("SetRowAttrs", 1)   # executor.go:2336
        self._broadcast_call(index, calls, opt)
        return [None] * len(calls)

    def _set_column_attrs(self, index: str, c: Call, opt):
        idx = self.holder.index(index)
        if idx is None:
            raise ErrIndexNotFound
        col, ok = c.uint_arg("_col")
        if not ok:
            raise PilosaError("reading SetColumnAttrs() col errs")
        attrs = {k: v for k, v in c.args.items() if k not in ("_col", "field")}
        idx.column_attr_store.set_attrs(col, attrs)
        if idx.stats is not None:
            idx.stats.count("SetProfileAttrs", 1)   # executor.go:2390
        self._broadcast_call(index, [c], opt)

    # ================================================================ translation
    def _translate_call(self, index: str, idx, c: Call):
        ts = self.holder.translate
        n = c.name
        if n in ("Set", "Clear", "Row", "Range", "SetColumnAttrs", "ClearRow"):
            col_key = "_col"
            try:
                fname = c.field_arg()
            except ValueError:
                fname = ""
            row_key = fname
        elif n == "SetRowAttrs":
            col_key = None
            row_key = "_row"
            fname = c.args.get("_field") if isinstance(c.args.get("_field"), str) else ""
        elif n == "Rows":
            fname = c.args.get("_field") if isinstance(c.args.get("_field"), str) else ""
            row_key, col_key = "previous", "column"
        elif n == "GroupBy":
            return self._translate_group_by(index, idx, c)
        else:
            col_key = "col"
            fname = c.args.get("field") if isinstance(c.args.get("field"), str) else ""
            row_key = "row"
        if col_key is not None:
            v = c.args.get(col_key)
            if idx.keys:
                if v is not None and not isinstance(v, str):
                    raise BadRequestError("column value must be a string when index 'keys' option enabled")
                if isinstance(v, str) and v != "":
                    c.args[col_key] = ts.translate_columns_to_uint64(index, [v])[0]
            elif isinstance(v, str):
                raise BadRequestError("string 'col' value not allowed unless index 'keys' option enabled")
        if fname:
            f = idx.field(fname)
            if f is not None:
                v = c.args.get(row_key)
                if f.type == FIELD_TYPE_BOOL:
                    if row_key in c.args:
                        if not isinstance(v, bool):
                            raise PilosaError(f"getting bool key: invalid bool argument type: {type(v).__name__}")
                        c.args[row_key] = TRUE_ROW_ID if v else FALSE_ROW_ID
                elif f.keys():
                    if v is not None and not isinstance(v, str) and not isinstance(v, Condition):
                        raise BadRequestError("row value must be a string when field 'keys' option enabled")
                    if isinstance(v, str) and v != "":
                        c.args[row_key] = ts.translate_rows_to_uint64(index, fname, [v])[0]
                elif isinstance(v, str):
                    raise BadRequestError("string 'row' value not allowed unless field 'keys' option enabled")
        for ch in c.children:
            self._translate_call(index, idx, ch)

    def _translate_group_by(self, index, idx, c: Call):
        for ch in c.children:
            self._translate_call(index, idx, ch)
        filt = c.args.get("filter")
        if isinstance(filt, Call):
            self._translate_call(index, idx, filt)
        prev = c.args.get("previous")
        if prev is None:
            return
        if not isinstance(prev, list):
            raise PilosaError(f"'previous' argument must be list, but got {type(prev).__name__}")
        if len(prev) != len(c.children):
            raise PilosaError(f"mismatched lengths for previous: {len(prev)} and children: {len(c.children)} in {c}")
        for i, ch in enumerate(c.children):
            f = idx.field(ch.args.get("_field"))
            if f is None:
                raise ErrFieldNotFound
            if f.keys():
                if not isinstance(prev[i], str):
                    raise PilosaError("prev value must be a string when field 'keys' option enabled")
                prev[i] = self.holder.translate.translate_rows_to_uint64(index, f.name, [prev[i]])[0]
            elif isinstance(prev[i], str):
                raise PilosaError(f"got string row val '{prev[i]}' in 'previous' for field {f.name} which doesn't "
                                  f"use string keys")

    def _translate_result(self, index, idx, c: Call, r):
        ts = self.holder.translate
        if isinstance(r, Row):
            if idx.keys:
                out = Row()
                out.attrs = r.attrs
                out.keys = ts.translate_columns_to_strings(index, [int(c) for c in r.columns()])
                return out
            return r
        if isinstance(r, Pair):
            fname = c.args.get("field")
            if isinstance(fname, str) and fname:
                f = idx.field(fname)
                if f is None:
                    raise PilosaError(f'field "{fname}" not found')
                if f.keys():
                    key = ts.translate_row_to_string(index, fname, r.id)
                    if c.name in ("MinRow", "MaxRow"):
                        return Pair(r.id, r.count, key)
                    return Pair(0, r.count, key)
            return r
        # a []Pair result -- TopN's, even empty (executor.go:2832-2846)
        if isinstance(r, PairArray) or isinstance(r, list) and (c.name == "TopN" or (r and isinstance(r[0], Pair))):
            fname = c.args.get("_field")
            if isinstance(fname, str) and fname:
                f = idx.field(fname)
                if f is None:
                    raise PilosaError(f'field "{fname}" not found')
                if f.keys():
                    return [Pair(0, p.count, ts.translate_row_to_string(index, fname, p.id)) for p in r]
            return r
        if isinstance(r, list) and r and isinstance(r[0], GroupCount):
            out = []
            for g in r:
                grp = []
                for fr in g.group:
                    f = idx.field(fr.field)
                    if f is None:
                        raise ErrFieldNotFound
                    key = ts.translate_row_to_string(index, fr.field, fr.row_id) if f.keys() else ""
                    grp.append(FieldRow(fr.field, fr.row_id, key))
                out.append(GroupCount(grp, g.count))
            return out
        if c.name == "Rows" and isinstance(r, list):
            fname = c.args.get("_field")
            f = idx.field(fname) if isinstance(fname, str) else None
            if f is None:
                raise ErrFieldNotFound
            if f.keys():
                return RowIdentifiers(keys=ts.translate_rows_to_strings(index, fname, [int(x) for x in r]))
            return RowIdentifiers(rows=r)
        if c.name == "GroupBy" and isinstance(r, list):
            return r
        if c.name == "TopN" and isinstance(r, list):
            return r
        return r
