"""Holder: root of a node's data directory (reference: holder.go).

Layout: ``<data>/<index>/<field>/views/<view>/fragments/<shard>`` plus
``.meta``/``.data``/``.available.shards``/``.cache`` side files, the node id
(``.id``) and the translate log (``.keys``).  Also owns the cache-flush loop
(holder.go:506-538) and schema export/apply (holder.go:279-346).
"""
from __future__ import annotations

import os
import resource
import shutil
import threading
import uuid
from typing import Dict, List, Optional

from pilosa_amd.errors import ErrIndexExists, ErrIndexNotFound, ErrName, PilosaError, validate_name
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.models.index import Index
from pilosa_amd.models.translate import TranslateFile

FILE_LIMIT = 262144
CACHE_FLUSH_INTERVAL_S = 60.0


class Holder:
    def __init__(self, path: str, max_opn: int = 10000, stats=None, persistent_attrs: bool = True,
                 lazy_fragments: bool = False):
        self.path = path
        # open fragments by header only; storage is read on first host use
        # (a GPU node loads cold fragments straight into HBM, ops/loader.py)
        self.lazy_fragments = lazy_fragments
        self.indexes: Dict[str, Index] = {}
        self.max_opn = max_opn
        self.stats = stats
        self.persistent_attrs = persistent_attrs
        self.translate = TranslateFile(os.path.join(path, ".keys"))
        self.mu = threading.RLock()
        self._closing = threading.Event()
        self._flusher: Optional[threading.Thread] = None
        self.on_create_shard = None   # (index, field, shard) -> None, set by the server (broadcast)
        self.on_schema_change = None  # () -> None, e.g. GPU arena invalidation
        self.snapshot_queue = None    # background snapshots, created by open() (holder.go:160)
        self.logger = None            # open-time warnings (server sets its logger)

    # ------------------------------------------------------------ lifecycle
    def open(self, background: bool = False):
        from pilosa_amd.models.snapshot import SnapshotQueue
        with self.mu:
            os.makedirs(self.path, exist_ok=True)
            if self.snapshot_queue is None:
                self.snapshot_queue = SnapshotQueue(100, 2)
            self._set_file_limit()
            self.translate.open()
            for name in sorted(os.listdir(self.path)):
                p = os.path.join(self.path, name)
                if name.startswith(".") or not os.path.isdir(p):
                    continue
                try:
                    validate_name(name)
                except Exception:  # noqa: BLE001
                    self._log(f"ERROR opening index: {name}, err={ErrName}")   # holder.go Open: logged, skipped
                    continue
                idx = self._new_index(name)
                try:
                    idx.open()
                except PilosaError as e:
                    raise PilosaError(f"open index: name={name}, err={e}") from e
                except OSError as e:
                    raise PilosaError(f"open index: name={name}, err={e.strerror or e}") from e
                self.indexes[name] = idx
        if background:
            self._flusher = threading.Thread(target=self._monitor_cache_flush, daemon=True)
            self._flusher.start()
        return self

    def close(self):
        self._closing.set()
        if self.snapshot_queue is not None:
            self.snapshot_queue.close()
            self.snapshot_queue = None
        with self.mu:
            for idx in self.indexes.values():
                idx.close()
            self.indexes.clear()
            self.translate.close()

    @staticmethod
    def _set_file_limit():
        try:
            soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
            want = min(FILE_LIMIT, hard) if hard != resource.RLIM_INFINITY else FILE_LIMIT
            if soft < want:
                resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
        except (ValueError, OSError):
            pass

    def load_node_id(self) -> str:
        p = os.path.join(self.path, ".id")
        if os.path.exists(p):
            with open(p) as fh:
                nid = fh.read().strip()
            if nid:
                return nid
        nid = str(uuid.uuid4())
        os.makedirs(self.path, exist_ok=True)
        with open(p, "w") as fh:
            fh.write(nid)
        return nid

    def _monitor_cache_flush(self):
        while not self._closing.wait(CACHE_FLUSH_INTERVAL_S):
            self.flush_caches()

    def flush_caches(self):
        for frag in self.all_fragments():
            try:
                frag.flush_cache()
            except OSError:
                pass

    def recalculate_caches(self):
        for frag in self.all_fragments():
            frag.recalculate_cache()

    # ------------------------------------------------------------ indexes
    def _new_index(self, name: str, keys=False, track_existence=True) -> Index:
        # the index (and its fields, views, fragments) count under "index:<name>" (holder.go:442)
        st = self.stats.with_tags(f"index:{name}") if self.stats is not None else None
        idx = Index(os.path.join(self.path, name), name, keys=keys, track_existence=track_existence,
                    max_opn=self.max_opn, stats=st, persistent_attrs=self.persistent_attrs)
        idx.on_create_shard = self._index_created_shard
        idx.snapshot_queue = self.snapshot_queue
        idx.lazy_fragments = self.lazy_fragments
        return idx

    def _index_created_shard(self, idx, field, shard):
        if self.on_create_shard is not None:
            self.on_create_shard(idx.name, field.name, shard)

    def create_index(self, name: str, keys: bool = False, track_existence: bool = True) -> Index:
        with self.mu:
            validate_name(name)
            if name in self.indexes:
                raise ErrIndexExists
            idx = self._new_index(name, keys, track_existence)
            idx.save_meta()
            idx.open()
            self.indexes[name] = idx
            self._changed()
            return idx

    def create_index_if_not_exists(self, name: str, keys: bool = False, track_existence: bool = True) -> Index:
        with self.mu:
            idx = self.indexes.get(name)
            if idx is not None:
                return idx
            return self.create_index(name, keys, track_existence)

    def index(self, name: str) -> Optional[Index]:
        return self.indexes.get(name)

    def index_list(self) -> List[Index]:
        return [self.indexes[n] for n in sorted(self.indexes)]

    def delete_index(self, name: str):
        with self.mu:
            idx = self.indexes.pop(name, None)
            if idx is None:
                raise ErrIndexNotFound
            idx.delete()
            self._changed()

    def field(self, index: str, name: str):
        idx = self.indexes.get(index)
        return idx.field(name) if idx is not None else None

    def view(self, index: str, field: str, name: str):
        f = self.field(index, field)
        return f.view(name) if f is not None else None

    def fragment(self, index: str, field: str, view: str, shard: int):
        v = self.view(index, field, view)
        return v.fragment(shard) if v is not None else None

    def all_fragments(self):
        for idx in list(self.indexes.values()):
            for f in list(idx.fields.values()):
                for v in list(f.views.values()):
                    yield from v.all_fragments()

    def _changed(self):
        if self.on_schema_change is not None:
            self.on_schema_change()

    def has_data(self) -> bool:
        """True when an index is open or the data dir holds an index
        directory (holder.go HasData peeks before Open)."""
        if self.indexes:
            return True
        try:
            return any(not n.startswith(".") and os.path.isdir(os.path.join(self.path, n))
                       for n in os.listdir(self.path))
        except OSError:
            return False

    def _log(self, msg: str):
        lg = getattr(self, "logger", None)
        if lg is not None:
            lg.printf("%s", msg)
        else:
            import sys
            print(msg, file=sys.stderr)

    # ------------------------------------------------------------ schema
    def schema(self) -> List[dict]:
        return [idx.info() for idx in self.index_list()]

    def apply_schema(self, schema: List[dict]):
        """Create missing indexes/fields from a schema (holder.go:322-346)."""
        for ii in schema:
            opts = ii.get("options", {})
            idx = self.create_index_if_not_exists(ii["name"], keys=opts.get("keys", False),
                                                  track_existence=opts.get("trackExistence", True))
            for fi in ii.get("fields", []):
                if idx.field(fi["name"]) is not None:
                    continue
                fo = fi.get("options", {})
                o = FieldOptions(type=fo.get("type", "set"), cache_type=fo.get("cacheType", ""),
                                 cache_size=fo.get("cacheSize", 0), time_quantum=fo.get("timeQuantum", ""),
                                 min=fo.get("min", 0), max=fo.get("max", 0), keys=fo.get("keys", False),
                                 no_standard_view=fo.get("noStandardView", False), base=fo.get("base", 0),
                                 bit_depth=fo.get("bitDepth", 0))
                idx.create_field(fi["name"], o)
                f = idx.field(fi["name"])
                for v in fi.get("views", []):
                    f.create_view_if_not_exists(v["name"] if isinstance(v, dict) else v)

    def available_shards_by_index(self) -> Dict[str, List[int]]:
        return {n: idx.available_shards() for n, idx in self.indexes.items()}

    def delete_all(self):
        self.close()
        shutil.rmtree(self.path, ignore_errors=True)
