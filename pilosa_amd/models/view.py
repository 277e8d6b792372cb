"""View: shard -> fragment map for one view of a field (reference: view.go).

View names: ``standard``, ``standard_YYYY[MM[DD[HH]]]`` (time quantums) and
``bsig_<field>`` (bit-sliced integers).  Directory:
``<field>/views/<view>/fragments/<shard>``.
"""
from __future__ import annotations

import os
import shutil
import threading
from typing import Callable, Dict, List, Optional

from pilosa_amd.errors import PilosaError
from pilosa_amd.models.fragment import SHARD_WIDTH_EXP, Fragment, bump_shard_epoch, remove_stale_snapshots
from pilosa_amd.models.row import Row

VIEW_STANDARD = "standard"
VIEW_BSI_PREFIX = "bsig_"


class View:
    def __init__(self, path: str, index: str, field: str, name: str, field_obj=None):
        self.path = path
        self.index, self.field, self.name = index, field, name
        self.field_obj = field_obj
        self.fragments: Dict[int, Fragment] = {}
        self.mu = threading.RLock()
        self.on_create_shard: Optional[Callable[[int], None]] = None

    def fragments_path(self) -> str:
        return os.path.join(self.path, "fragments")

    def fragment_path(self, shard: int) -> str:
        return os.path.join(self.fragments_path(), str(shard))

    def _new_fragment(self, shard: int) -> Fragment:
        f = self.field_obj
        opts = f.options if f is not None else None
        cache_type = opts.cache_type if opts is not None else "none"
        cache_size = opts.cache_size if opts is not None else 0
        if self.name.startswith(VIEW_BSI_PREFIX):
            cache_type, cache_size = "none", 0
        frag = Fragment(self.fragment_path(shard), self.index, self.field, self.name, shard,
                        cache_type=cache_type, cache_size=cache_size,
                        max_opn=f.max_opn if f is not None else 10000,
                        mutex=opts is not None and opts.type == "mutex",
                        bool_field=opts is not None and opts.type == "bool",
                        stats=f.stats if f is not None else None)
        frag.row_attr_store = f.row_attr_store if f is not None else None
        frag.snapshot_queue = getattr(f, "snapshot_queue", None)
        frag.lazy = bool(getattr(f, "lazy_fragments", False))
        return frag

    def open(self):
        with self.mu:
            os.makedirs(self.fragments_path(), exist_ok=True)
            names = os.listdir(self.fragments_path())
            remove_stale_snapshots(self.fragments_path(), names)
            for name in names:
                if not name.isdigit():
                    continue
                shard = int(name)
                try:
                    frag = self._new_fragment(shard).open()
                except PilosaError as e:
                    raise PilosaError(f"open fragment: shard={shard}, err=opening storage: {e}") from e
                self.fragments[shard] = frag
                bump_shard_epoch()
        return self

    def close(self):
        with self.mu:
            for f in self.fragments.values():
                f.close()
            self.fragments.clear()
            bump_shard_epoch()

    def fragment(self, shard: int) -> Optional[Fragment]:
        return self.fragments.get(shard)

    def all_fragments(self) -> List[Fragment]:
        with self.mu:
            return [self.fragments[s] for s in sorted(self.fragments)]

    def shards(self) -> List[int]:
        return sorted(self.fragments)

    def create_fragment_if_not_exists(self, shard: int) -> Fragment:
        with self.mu:
            f = self.fragments.get(shard)
            if f is not None:
                return f
            f = self._new_fragment(shard).open()
            self.fragments[shard] = f
            bump_shard_epoch()
        if self.field_obj is not None:
            self.field_obj._note_shard(shard)
        if self.on_create_shard is not None:
            self.on_create_shard(shard)
        return f

    def delete_fragment(self, shard: int):
        with self.mu:
            f = self.fragments.pop(shard, None)
            bump_shard_epoch()
            if f is None:
                from pilosa_amd.errors import ErrFragmentNotFound
                raise ErrFragmentNotFound
            f.close()
            for p in (f.path, f.cache_path()):
                try:
                    os.remove(p)
                except FileNotFoundError:
                    pass

    def delete(self):
        self.close()
        shutil.rmtree(self.path, ignore_errors=True)

    # ------------------------------------------------------------ data
    def row(self, row_id: int) -> Row:
        r = Row()
        for f in self.all_fragments():
            r.merge(f.row(row_id))
        return r

    def set_bit(self, row_id: int, col: int) -> bool:
        return self.create_fragment_if_not_exists(col >> SHARD_WIDTH_EXP).set_bit(row_id, col)

    def clear_bit(self, row_id: int, col: int) -> bool:
        f = self.fragment(col >> SHARD_WIDTH_EXP)
        return f.clear_bit(row_id, col) if f is not None else False

    def value(self, col: int, bit_depth: int):
        f = self.fragment(col >> SHARD_WIDTH_EXP)
        if f is None:
            return 0, False
        return f.value(col, bit_depth)

    def set_value(self, col: int, bit_depth: int, value: int) -> bool:
        return self.create_fragment_if_not_exists(col >> SHARD_WIDTH_EXP).set_value(col, bit_depth, value)

    def clear_value(self, col: int, bit_depth: int, value: int) -> bool:
        f = self.fragment(col >> SHARD_WIDTH_EXP)
        return f.clear_value(col, bit_depth, value) if f is not None else False

    def sum(self, filt: Optional[Row], bit_depth: int):
        s = c = 0
        for f in self.all_fragments():
            fs, fc = f.sum(filt, bit_depth)
            s += fs
            c += fc
        return s, c

    def min(self, filt: Optional[Row], bit_depth: int):
        mn, count, has = 0, 0, False
        for f in self.all_fragments():
            fm, fc = f.min(filt, bit_depth)
            if fc == 0:
                continue
            if not has:
                mn, count, has = fm, count + fc, True
                continue
            if fm < mn:
                mn = fm
                count += fc
        return mn, count

    def max(self, filt: Optional[Row], bit_depth: int):
        mx, count = 0, 0
        for f in self.all_fragments():
            fm, fc = f.max(filt, bit_depth)
            if fc > 0 and fm > mx:
                mx = fm
                count += fc
        return mx, count

    def range_op(self, op: str, bit_depth: int, predicate: int) -> Row:
        r = Row()
        for f in self.all_fragments():
            r = r.union(f.range_op(op, bit_depth, predicate))
        return r
