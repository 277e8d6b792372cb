"""API facade (reference: api.go).

Validates each method against the cluster state (api.go:100-124, lists
:1382-1414), then drives the holder / executor / cluster.  Schema mutations
are broadcast to the other nodes; imports are routed to the owning nodes
(api.go:919-1112, :305-427).  The HTTP layer (http_handler.py) and the CLI
sit on top of this class.
"""
from __future__ import annotations

import base64
import io
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from pilosa_amd import __version__
from pilosa_amd.errors import (APIMethodNotAllowedError, BadRequestError, ConflictError, ErrClusterDoesNotOwnShard,
                               ErrFieldExists, ErrFieldNotFound, ErrFragmentNotFound, ErrIndexExists,
                               ErrIndexNotFound, ErrNodeIDNotExists, ErrNodeNotCoordinator, ErrResizeNotRunning,
                               NotFoundError, PilosaError, wrap)
from pilosa_amd.executor import ExecOptions, QueryResponse
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.models.fragment import SHARD_WIDTH
from pilosa_amd.parallel.cluster import STATE_DEGRADED, STATE_NORMAL, STATE_RESIZING, STATE_STARTING, URI, Node
from pilosa_amd.pql import ParseError, parse_string
from pilosa_amd.utils import tracing

M_COMMON = {"ClusterMessage", "SetCoordinator", "Schema", "Status", "Info", "Version", "Hosts", "Node",
            "TranslateData"}
M_RESIZING = {"FragmentData", "ResizeAbort"}
M_NORMAL = {"CreateField", "CreateIndex", "DeleteField", "DeleteAvailableShard", "DeleteIndex", "DeleteView",
            "ExportCSV", "FragmentBlockData", "FragmentBlocks", "Field", "FieldAttrDiff", "Import", "ImportValue",
            "ImportRoaring", "Index", "IndexAttrDiff", "Query", "RecalculateCaches", "RemoveNode", "ShardNodes",
            "Views", "ApplySchema", "FragmentData", "TranslateKeys", "MaxShards"}
VALID = {
    STATE_STARTING: M_COMMON,
    STATE_NORMAL: M_COMMON | M_NORMAL,
    STATE_DEGRADED: M_COMMON | M_NORMAL,
    STATE_RESIZING: M_COMMON | M_RESIZING,
}


class QueryRequest:
    def __init__(self, index: str = "", query: str = "", shards: Sequence[int] = (), column_attrs=False,
                 remote=False, exclude_row_attrs=False, exclude_columns=False):
        self.index, self.query, self.shards = index, query, list(shards)
        self.column_attrs, self.remote = column_attrs, remote
        self.exclude_row_attrs, self.exclude_columns = exclude_row_attrs, exclude_columns


class API:
    def __init__(self, server):
        self.server = server

    @property
    def holder(self):
        return self.server.holder

    @property
    def cluster(self):
        return self.server.cluster

    @property
    def executor(self):
        return self.server.executor

    def validate(self, method: str):
        state = self.cluster.state
        if method not in VALID.get(state, set()):
            raise APIMethodNotAllowedError(f"api method {method} not allowed in state {state}")

    # ------------------------------------------------------------ query
    def query(self, req: QueryRequest) -> QueryResponse:
        self.validate("Query")
        with tracing.span("API.Query"):
            try:
                q = parse_string(req.query)
            except ParseError as e:
                raise BadRequestError(f"parsing: {e}")
            opt = ExecOptions(remote=req.remote, exclude_row_attrs=req.exclude_row_attrs,
                              exclude_columns=req.exclude_columns, column_attrs=req.column_attrs)
            t0 = time.perf_counter()
            try:
                resp = self.executor.execute(req.index, q, req.shards or None, opt)
            except PilosaError as e:
                if req.remote:      # the coordinator wraps its own answer
                    raise
                raise wrap(e, "executing") from e   # api.go:154
            dt = time.perf_counter() - t0
            if self.server.long_query_time and dt > self.server.long_query_time:
                self.server.logger.printf("%s %s %.3fs", req.index, req.query[:200], dt)
            resp.calls = q.calls
            return resp

    # ------------------------------------------------------------ schema
    def _count(self, name: str, index: Optional[str] = None):
        """Schema events on the holder's stats client (api.go:183,227,274,461,493)."""
        st = self.holder.stats
        if st is None:
            return
        if index is None:
            st.count(name, 1)
        else:
            st.count_with_tags(name, 1, [f"index:{index}"])

    def create_index(self, name: str, keys: bool = False, track_existence: bool = True, remote: bool = False):
        self.validate("CreateIndex")
        try:
            idx = self.holder.create_index(name, keys=keys, track_existence=track_existence)
        except PilosaError as e:
            if e is ErrIndexExists:
                raise ConflictError(wrap(e, "creating index"))
            raise BadRequestError(wrap(e, "creating index"))
        self._count("createIndex")
        self._mesh_schema()
        if not remote:
            self.server.broadcast({"type": "CreateIndex", "index": name,
                                   "options": {"keys": keys, "trackExistence": track_existence}})
        return idx

    def index(self, name: str):
        self.validate("Index")
        idx = self.holder.index(name)
        if idx is None:
            raise NotFoundError(ErrIndexNotFound)
        return idx

    def delete_index(self, name: str, remote: bool = False):
        self.validate("DeleteIndex")
        try:
            self.holder.delete_index(name)
        except PilosaError as e:
            raise NotFoundError(wrap(e, "deleting index"))
        self._count("deleteIndex")
        if self.server.gpu is not None:
            self.server.gpu.invalidate()
        if getattr(self.server, "mesh", None) is not None:
            self.server.mesh.delete_index(name)
        if not remote:
            self.server.broadcast({"type": "DeleteIndex", "index": name})

    def create_field(self, index: str, name: str, opts: Optional[FieldOptions] = None, remote: bool = False):
        self.validate("CreateField")
        idx = self.holder.index(index)
        if idx is None:
            raise NotFoundError(ErrIndexNotFound)
        try:
            f = idx.create_field(name, opts)
        except PilosaError as e:
            if e is ErrFieldExists:
                raise ConflictError(wrap(e, "creating field"))
            raise BadRequestError(wrap(e, "creating field"))
        self._count("createField", index)
        self._mesh_schema()
        if not remote:
            self.server.broadcast({"type": "CreateField", "index": index, "field": name,
                                   "options": f.options.to_json()})
        return f

    def field(self, index: str, name: str):
        self.validate("Field")
        idx = self.holder.index(index)
        if idx is None:
            raise NotFoundError(ErrIndexNotFound)
        f = idx.field(name)
        if f is None:
            raise NotFoundError(ErrFieldNotFound)
        return f

    def delete_field(self, index: str, name: str, remote: bool = False):
        self.validate("DeleteField")
        idx = self.holder.index(index)
        if idx is None:
            raise NotFoundError(ErrIndexNotFound)
        try:
            idx.delete_field(name)
        except PilosaError as e:
            raise NotFoundError(wrap(e, "deleting field"))
        self._count("deleteField", index)
        if self.server.gpu is not None:
            self.server.gpu.invalidate()
        if getattr(self.server, "mesh", None) is not None:
            self.server.mesh.delete_field(index, name)
        if not remote:
            self.server.broadcast({"type": "DeleteField", "index": index, "field": name})

    def delete_available_shard(self, index: str, field: str, shard: int, remote: bool = False):
        self.validate("DeleteAvailableShard")
        f = self.field(index, field)
        f.remove_available_shard(shard)
        self._count("deleteAvailableShard", index)
        if not remote:
            self.server.broadcast({"type": "DeleteAvailableShard", "index": index, "field": field, "shard": shard})

    def delete_view(self, index: str, field: str, view: str, remote: bool = False):
        self.validate("DeleteView")
        f = self.field(index, field)
        try:
            f.delete_view(view)
        except PilosaError as e:
            raise NotFoundError(e)
        if not remote:
            self.server.broadcast({"type": "DeleteView", "index": index, "field": field, "view": view})

    def views(self, index: str, field: str) -> List[str]:
        self.validate("Views")
        return sorted(self.field(index, field).views)

    def schema(self) -> List[dict]:
        """Indexes and their public fields without views (api.go Schema ->
        holder.limitedSchema, holder.go:299-319)."""
        self.validate("Schema")
        out = []
        for ii in self.holder.schema():
            ii = dict(ii)
            ii["fields"] = [{k: v for k, v in fi.items() if k != "views"} for fi in ii.get("fields", [])]
            out.append(ii)
        return out

    def apply_schema(self, schema: List[dict], remote: bool = False):
        self.validate("ApplySchema")
        self.holder.apply_schema(schema)
        if not remote:
            self.server.broadcast({"type": "ApplySchema", "schema": schema})

    # ------------------------------------------------------------ imports
    def _mesh_schema(self):
        mesh = getattr(self.server, "mesh", None)
        if mesh is not None:
            mesh.apply_schema()

    def _mesh_route(self, index: str, field: str, kind: str, shard: int, payload: dict) -> bool:
        """Multi-GPU node: hand an import for a shard owned by another rank to
        that rank (parallel/mesh.py).  Returns True when it was routed."""
        mesh = getattr(self.server, "mesh", None)
        if mesh is None or mesh.world <= 1 or mesh.owner(shard) == mesh.rank:
            return False
        mesh.forward_import(kind, index, field, shard, payload)
        return True

    def _owns(self, index: str, shard: int):
        if not self.cluster.owns_shard(self.cluster.node.id, index, shard):
            raise ErrClusterDoesNotOwnShard

    def import_bits(self, index: str, field: str, shard: int, row_ids=(), col_ids=(), row_keys=(), col_keys=(),
                    timestamps=(), clear: bool = False, ignore_key_check: bool = False):
        self.validate("Import")
        idx = self.index(index)
        f = idx.field(field)
        if f is None:
            raise NotFoundError(ErrFieldNotFound)
        # numpy arrays (the native request decoder) stay arrays on the id path
        row_ids = row_ids if isinstance(row_ids, np.ndarray) else list(row_ids)
        col_ids = col_ids if isinstance(col_ids, np.ndarray) else list(col_ids)
        if not ignore_key_check:
            if f.keys():
                if len(row_ids):
                    raise BadRequestError("row ids cannot be used because field uses string keys")
                row_ids = self.holder.translate.translate_rows_to_uint64(index, field, list(row_keys))
            if idx.keys:
                if len(col_ids):
                    raise BadRequestError("column ids cannot be used because index uses string keys")
                col_ids = self.holder.translate.translate_columns_to_uint64(index, list(col_keys))
            if idx.keys or f.keys():
                row_ids, col_ids = [int(x) for x in row_ids], [int(x) for x in col_ids]
                by_shard: Dict[int, List[int]] = {}
                for i, c in enumerate(col_ids):
                    by_shard.setdefault(c // SHARD_WIDTH, []).append(i)
                for s, ii in sorted(by_shard.items()):
                    ts = [int(timestamps[i]) for i in ii] if len(timestamps) else []
                    self._route_import(index, field, s, [row_ids[i] for i in ii], [col_ids[i] for i in ii], ts,
                                       clear)
                return
        self._owns(index, shard)
        self._local_import(idx, f, row_ids, col_ids, timestamps, clear)

    def _route_import(self, index, field, shard, rows, cols, ts, clear):
        for node in self.cluster.shard_nodes(index, shard):
            if node.id == self.cluster.node.id:
                idx = self.holder.index(index)
                self._local_import(idx, idx.field(field), rows, cols, ts, clear)
            else:
                self.server.client.import_bits(node, index, field, shard, rows, cols, ts, clear=clear,
                                               ignore_key_check=True)

    def _local_import(self, idx, f, rows, cols, timestamps, clear):
        import datetime as dt
        if len(cols) and self._mesh_route(idx.name, f.name, "bits", int(cols[0]) // SHARD_WIDTH,
                                          {"rows": rows, "cols": cols, "clear": clear,
                                           "timestamps": _ts_list(timestamps)}):
            return
        tss = None
        if len(timestamps) and np.any(np.asarray(timestamps, dtype=np.int64) != 0):
            tss = [dt.datetime.utcfromtimestamp(t / 1e9) if t else None for t in np.asarray(timestamps).tolist()]
        if not clear and idx.existence_field() is not None and len(cols):
            idx.existence_field().import_bits(np.zeros(len(cols), np.uint64), np.asarray(cols, np.uint64))
        f.import_bits(rows, cols, tss, clear=clear)

    def import_values(self, index: str, field: str, shard: int, col_ids=(), values=(), col_keys=(),
                      clear: bool = False, ignore_key_check: bool = False):
        self.validate("ImportValue")
        idx = self.index(index)
        f = idx.field(field)
        if f is None:
            raise NotFoundError(ErrFieldNotFound)
        col_ids = col_ids if isinstance(col_ids, np.ndarray) else list(col_ids)
        values = values if isinstance(values, np.ndarray) else list(values)
        if not ignore_key_check and idx.keys:
            if len(col_ids):
                raise BadRequestError("column ids cannot be used because index uses string keys")
            col_ids = self.holder.translate.translate_columns_to_uint64(index, list(col_keys))
            by_shard: Dict[int, List[int]] = {}
            for i, c in enumerate(col_ids):
                by_shard.setdefault(c // SHARD_WIDTH, []).append(i)
            for s, ii in sorted(by_shard.items()):
                for node in self.cluster.shard_nodes(index, s):
                    cc, vv = [col_ids[i] for i in ii], [values[i] for i in ii]
                    if node.id == self.cluster.node.id:
                        self._local_import_values(idx, f, cc, vv, clear)
                    else:
                        self.server.client.import_values(node, index, field, s, cc, vv, clear=clear,
                                                         ignore_key_check=True)
            return
        self._owns(index, shard)
        self._local_import_values(idx, f, col_ids, values, clear)

    def _local_import_values(self, idx, f, cols, vals, clear):
        if len(cols) and self._mesh_route(idx.name, f.name, "values", int(cols[0]) // SHARD_WIDTH,
                                          {"cols": cols, "values": vals, "clear": clear}):
            return
        if not clear and idx.existence_field() is not None and len(cols):
            idx.existence_field().import_bits(np.zeros(len(cols), np.uint64), np.asarray(cols, np.uint64))
        f.import_values(cols, vals, clear=clear)

    def import_roaring(self, index: str, field: str, shard: int, views: Dict[str, bytes], clear: bool = False,
                       remote: bool = False):
        self.validate("ImportRoaring")
        f = self.field(index, field)
        if f.options.type not in ("set", "time"):   # api.go:384-386
            raise BadRequestError("roaring import is only supported for set and time fields")
        for node in self.cluster.shard_nodes(index, shard):
            if node.id == self.cluster.node.id:
                if not self._mesh_route(index, field, "roaring", shard, {"views": dict(views), "clear": clear}):
                    f.import_roaring(shard, views, clear)
            elif not remote:
                self.server.client.import_roaring(node, index, field, shard, views, clear=clear, remote=True)

    # ------------------------------------------------------------ export / fragments
    def export_csv(self, index: str, field: str, shard: int, w):
        self.validate("ExportCSV")
        f = self.field(index, field)
        self._owns(index, shard)
        frag = self.holder.fragment(index, field, "standard", shard)
        if frag is None:
            raise ErrFragmentNotFound
        idx = self.holder.index(index)
        ts = self.holder.translate
        for row, col in frag.for_each_bit():
            rs = ts.translate_row_to_string(index, field, row) if f.keys() else str(row)
            cs = ts.translate_column_to_string(index, col) if idx.keys else str(col)
            w.write(f"{rs},{cs}\n")

    def fragment_blocks(self, index, field, view, shard):
        self.validate("FragmentBlocks")
        frag = self.holder.fragment(index, field, view, shard)
        if frag is None:
            raise ErrFragmentNotFound
        # Go encodes []byte as base64 (fragment.go FragmentBlock)
        return [{"id": b, "checksum": base64.b64encode(c).decode()} for b, c in frag.blocks()]

    def fragment_block_data(self, index, field, view, shard, block):
        self.validate("FragmentBlockData")
        frag = self.holder.fragment(index, field, view, shard)
        if frag is None:
            raise ErrFragmentNotFound
        return frag.block_data(block)

    def fragment_data(self, index, field, view, shard) -> bytes:
        self.validate("FragmentData")
        frag = self.holder.fragment(index, field, view, shard)
        if frag is None:
            raise ErrFragmentNotFound
        buf = io.BytesIO()
        frag.write_to(buf)
        return buf.getvalue()

    def shard_nodes(self, index: str, shard: int):
        self.validate("ShardNodes")
        return self.cluster.shard_nodes(index, shard)

    def max_shards(self) -> Dict[str, int]:
        out = {}
        for idx in self.holder.index_list():
            sh = idx.available_shards()
            out[idx.name] = max(sh) if sh else 0
        return out

    def recalculate_caches(self, remote: bool = False):
        self.validate("RecalculateCaches")
        mesh = getattr(self.executor, "mesh", None)
        if mesh is not None and mesh.world > 1:
            mesh.recalculate_caches()   # every GPU's holder (rank 0's included)
        else:
            self.holder.recalculate_caches()
        if not remote:
            self.server.broadcast({"type": "RecalculateCaches"})

    # ------------------------------------------------------------ translate
    def translate_keys(self, index: str, field: str, keys: List[str]) -> List[int]:
        self.validate("TranslateKeys")
        ts = self.holder.translate
        if field:
            return ts.translate_rows_to_uint64(index, field, keys)
        return ts.translate_columns_to_uint64(index, keys)

    def translate_data(self, offset: int) -> bytes:
        self.validate("TranslateData")
        return self.holder.translate.read_from(offset)

    # ------------------------------------------------------------ cluster
    def cluster_message(self, msg: dict):
        self.validate("ClusterMessage")
        self.server.receive_message(msg)

    def hosts(self):
        return list(self.cluster.nodes)

    def node(self):
        return self.cluster.node

    def state(self) -> str:
        return self.cluster.state

    def status(self) -> dict:
        return {"state": self.cluster.state, "nodes": [n.to_json() for n in self.cluster.nodes],
                "localID": self.cluster.node.id}

    def info(self) -> dict:
        from pilosa_amd.utils.sysinfo import SystemInfo
        si = SystemInfo()
        gpu = self.server.gpu_info()
        return {"shardWidth": SHARD_WIDTH, "cpuPhysicalCores": si.cpu_cores(), "cpuLogicalCores": si.cpu_threads(),
                "cpuType": si.cpu_model(), "memory": si.mem_total(), "version": __version__, "gpus": gpu}

    def version(self) -> str:
        from pilosa_amd import buildinfo
        return buildinfo.VERSION.lstrip("v")   # handler.go: strings.TrimPrefix(pilosa.Version, "v")

    def set_coordinator(self, node_id: str):
        self.validate("SetCoordinator")
        n = self.cluster.node_by_id(node_id)
        if n is None:
            raise ErrNodeIDNotExists
        old = self.cluster.coordinator()
        self.cluster.set_coordinator(node_id)
        self.server.broadcast({"type": "SetCoordinator", "node": n.to_json()})
        return old, n

    def remove_node(self, node_id: str):
        """Start a REMOVE resize (api.go:1225 RemoveNode -> cluster.nodeLeave).
        A node only in the persisted topology (already gone) can be removed too."""
        self.validate("RemoveNode")
        n = self.cluster.node_by_id(node_id)
        if n is None:
            if not self.cluster.topology.contains_id(node_id):
                raise NotFoundError(f"finding node to remove: {ErrNodeIDNotExists}")
            n = Node(node_id, URI())
        try:
            self.server.node_leave(n)
        except PilosaError as e:
            raise PilosaError(f"calling node leave: {e}") from e
        return n

    def resize_abort(self):
        self.validate("ResizeAbort")
        if not self.server.abort_resize():
            raise ErrResizeNotRunning


def _ts_list(timestamps):
    """Import timestamps (ns since epoch) -> datetimes, as Field.import_bits takes."""
    import datetime as dt
    if timestamps is None or not len(timestamps) or not np.any(np.asarray(timestamps, dtype=np.int64) != 0):
        return None
    return [dt.datetime.utcfromtimestamp(t / 1e9) if t else None for t in np.asarray(timestamps).tolist()]
