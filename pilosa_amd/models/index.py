"""Index: a set of fields sharing one column space (reference: index.go).

``track_existence`` maintains the ``_exists`` field (row 0 set for every
column ever written) that ``Not()`` and column-existence queries use.
Options persist in ``.meta`` (protobuf IndexMeta); column attributes live in
the index's ``.data`` store.
"""
from __future__ import annotations

import os
import shutil
import threading
from typing import Dict, List, Optional

from pilosa_amd.errors import ErrFieldExists, ErrFieldNotFound, ErrName, PilosaError, validate_name
from pilosa_amd.shardwidth import SHARD_WIDTH
from pilosa_amd.models.attrs import MemAttrStore, SQLiteAttrStore
from pilosa_amd.models.cache import CACHE_TYPE_NONE
from pilosa_amd.models.field import Field, FieldOptions
from pilosa_amd.models.fragment import bump_shard_epoch, shard_epoch

EXISTENCE_FIELD_NAME = "_exists"


class Index:
    def __init__(self, path: str, name: str, keys: bool = False, track_existence: bool = True,
                 max_opn: int = 10000, stats=None, persistent_attrs: bool = True):
        validate_name(name)
        self.path = path
        self.name = name
        self.keys = keys
        self.track_existence = track_existence
        self.fields: Dict[str, Field] = {}
        self.max_opn = max_opn
        self.stats = stats
        self.persistent_attrs = persistent_attrs
        self.column_attr_store = SQLiteAttrStore(os.path.join(path, ".data")) if persistent_attrs \
            else MemAttrStore()
        self.mu = threading.RLock()
        self.on_create_shard = None

    def meta_path(self) -> str:
        return os.path.join(self.path, ".meta")

    def save_meta(self):
        from pilosa_amd.wire import pb
        os.makedirs(self.path, exist_ok=True)
        with open(self.meta_path(), "wb") as fh:
            fh.write(pb.IndexMeta(Keys=self.keys, TrackExistence=self.track_existence).SerializeToString())

    def load_meta(self):
        from pilosa_amd.wire import pb
        if os.path.exists(self.meta_path()):
            m = pb.IndexMeta()
            with open(self.meta_path(), "rb") as fh:
                m.ParseFromString(fh.read())
            self.keys, self.track_existence = m.Keys, m.TrackExistence

    def open(self):
        with self.mu:
            os.makedirs(self.path, exist_ok=True)
            self.load_meta()
            try:
                self.column_attr_store.open()
            except Exception as e:  # noqa: BLE001
                raise PilosaError(f"opening attrstore: opening storage: {_attr_err(e)}") from e
            for name in sorted(os.listdir(self.path)):
                p = os.path.join(self.path, name)
                if name.startswith(".") or not os.path.isdir(p):
                    continue
                f = self._new_field(name, None)
                try:
                    f.open()
                except PilosaError as e:
                    raise PilosaError(f"opening fields: open field: name={name}, err={e}") from e
                self.fields[name] = f
                bump_shard_epoch()
            if self.track_existence:
                self._open_existence_field()
        return self

    def _open_existence_field(self):
        if EXISTENCE_FIELD_NAME not in self.fields:
            self._create_field(EXISTENCE_FIELD_NAME, FieldOptions(type="set", cache_type=CACHE_TYPE_NONE))

    def close(self):
        with self.mu:
            for f in self.fields.values():
                f.close()
            self.fields.clear()
            bump_shard_epoch()
            self.column_attr_store.close()

    def delete(self):
        self.close()
        shutil.rmtree(self.path, ignore_errors=True)

    def _new_field(self, name: str, opts: Optional[FieldOptions]) -> Field:
        f = Field(os.path.join(self.path, name), self.name, name, opts, max_opn=self.max_opn, stats=self.stats,
                  persistent_attrs=self.persistent_attrs)
        f.on_create_shard = self._field_created_shard
        f.snapshot_queue = getattr(self, "snapshot_queue", None)
        f.lazy_fragments = getattr(self, "lazy_fragments", False)
        return f

    def _field_created_shard(self, field: Field, shard: int):
        if self.on_create_shard is not None:
            self.on_create_shard(self, field, shard)

    def _create_field(self, name: str, opts: FieldOptions) -> Field:
        f = self._new_field(name, opts)
        f.save_meta()
        f.open()
        self.fields[name] = f
        bump_shard_epoch()
        return f

    def create_field(self, name: str, opts: Optional[FieldOptions] = None) -> Field:
        with self.mu:
            if name == EXISTENCE_FIELD_NAME:
                raise ErrName
            validate_name(name)
            if name in self.fields:
                raise ErrFieldExists
            return self._create_field(name, opts or FieldOptions.default())

    def create_field_if_not_exists(self, name: str, opts: Optional[FieldOptions] = None) -> Field:
        with self.mu:
            f = self.fields.get(name)
            if f is not None:
                return f
            validate_name(name)
            return self._create_field(name, opts or FieldOptions.default())

    def field(self, name: str) -> Optional[Field]:
        return self.fields.get(name)

    def existence_field(self) -> Optional[Field]:
        return self.fields.get(EXISTENCE_FIELD_NAME) if self.track_existence else None

    def public_fields(self) -> List[Field]:
        return [self.fields[n] for n in sorted(self.fields) if n != EXISTENCE_FIELD_NAME]

    def delete_field(self, name: str):
        with self.mu:
            f = self.fields.pop(name, None)
            bump_shard_epoch()
            if f is None:
                raise ErrFieldNotFound
            f.delete()

    def available_shards(self) -> List[int]:
        # memoised on the shard epoch (bumped by every fragment / view /
        # field / remote-shard change): the walk over ~1k fragments per
        # request was a visible share of a serving request
        return list(self.available_shards_memo()[1])

    def available_shards_memo(self):
        """(shard epoch, sorted shard tuple): the tuple is the same object
        while the epoch holds, so a per-request fast path can key memos on the
        epoch instead of hashing ~1k shard ids."""
        ep = shard_epoch()
        memo = self.__dict__.get("_avail_memo")
        if memo is not None and memo[0] == ep:
            return memo
        s = set()
        for f in list(self.fields.values()):
            s |= set(f.available_shards())
        out = sorted(s)
        memo = self._avail_memo = (ep, tuple(out))
        if self.stats is not None and out:
            self.stats.gauge("maxShard", out[-1])   # index.go:257
        return memo

    def options_json(self) -> dict:
        return {"keys": self.keys, "trackExistence": self.track_existence}

    def info(self) -> dict:
        return {"name": self.name, "options": self.options_json(),
                "fields": [f.info() for f in self.public_fields()], "shardWidth": SHARD_WIDTH}


def _attr_err(e: Exception) -> str:
    """The reference's bolt wording for an unreadable attribute database."""
    import sqlite3
    if isinstance(e, sqlite3.DatabaseError):
        return "invalid database"
    return str(e)
