"""Device-resident container arenas and the batched GPU query engine.

Every field-view of an index that is queried on a GPU is mirrored into HBM as
a *container arena* (layout documented in pilosa_amd/native/pyroaring.cpp):
CSR row directory per local shard + packed container metadata + payload pool.
The HIP kernels in pilosa_amd/kernels/bitmap_kernels.hip evaluate a whole
batch of boolean query programs over all local shards of the arena in one
launch (reference per-shard worker loop: executor.go:2564-2611 — replaced).

Query programs are tiny postfix byte codes over <=16 leaves (a leaf = one row
of one view).  ``Expr`` trees are compiled here.
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from pilosa_amd.utils import tracing

MAXLEAF = 16
MAXPROG = 32
OP_AND, OP_OR, OP_XOR, OP_ANDNOT = 32, 33, 34, 35
# count-batch kernel routes
KIND_AND2, KIND_ROW, KIND_GENERIC, KIND_FLAT, KIND_UNION = 0, 1, 2, 3, 4
# a planned batch's repeated Count(Intersect(a, b)) calls: (from, to) result
# copies applied after the kernels (native/pql_compile.cpp plan_count_text)
KIND_ALIAS = 5
# launch_expr_count modes: expr_count_kernel<0/1/2>, 3 = union_count_kernel
_KERNEL_MODE = {KIND_ROW: 1, KIND_GENERIC: 0, KIND_FLAT: 2, KIND_UNION: 3}


def flat_mask(progs: np.ndarray) -> np.ndarray:
    """Programs that are left folds "l0 l1 op l2 op ..." (flat kernel mode)."""
    pg = progs["prog"].astype(np.int32)
    n = progs["nprog"].astype(np.int64)
    pos = np.arange(pg.shape[1])
    want_leaf = (pos == 0) | (pos % 2 == 1)
    valid = pos[None, :] < n[:, None]
    ok = np.where(valid, (pg < OP_AND) == want_leaf[None, :], True).all(axis=1)
    return ok & (n >= 3) & (n % 2 == 1)
_OPS = {"and": OP_AND, "or": OP_OR, "xor": OP_XOR, "andnot": OP_ANDNOT}

QPROG_DTYPE = np.dtype([("nleaf", "<i4"), ("nprog", "<i4"), ("leaf_view", "<i4", (MAXLEAF,)),
                        ("leaf_row", "<i8", (MAXLEAF,)), ("prog", "u1", (MAXPROG,)), ("pad", "<i8", (3,))])
VIEWDEV_DTYPE = np.dtype([("rowptr", "<u8"), ("shard_base", "<u8"), ("meta", "<u8"), ("payload", "<u8"),
                          ("D", "<i8"), ("keymask", "<u8"), ("shadow", "<u8"), ("shadow_slot", "<u8")])
assert QPROG_DTYPE.itemsize == 256 and VIEWDEV_DTYPE.itemsize == 64

_ext = None
_ext_lock = threading.Lock()
_D2H_POLL = float(os.environ.get("PILOSA_D2H_POLL", "0"))


def kernels():
    """Load the in-tree HIP extension; fail loudly when it is missing."""
    global _ext
    if _ext is None:
        with _ext_lock:
            if _ext is None:
                import importlib

                import torch  # noqa: F401  (loads libtorch for the extension)
                # PILOSA_HIPKERNELS=_hipkernels_kbench: the A/B build with the
                # rejected variants (scripts/kbench.py); the product loads the
                # shipped module
                ext = importlib.import_module("pilosa_amd." + os.environ.get("PILOSA_HIPKERNELS", "_hipkernels"))
                assert ext.QUERYPROG_BYTES == QPROG_DTYPE.itemsize
                assert ext.VIEWDEV_BYTES == VIEWDEV_DTYPE.itemsize
                _ext = ext
    return _ext


# ---------------------------------------------------------------- expressions

@dataclass(frozen=True)
class Leaf:
    view: object          # DeviceView
    row: int              # row id (not dense index)


@dataclass(frozen=True)
class Op:
    op: str               # and / or / xor / andnot
    args: Tuple[object, ...]


class CompileError(Exception):
    pass


def compile_expr(expr, view_index: Dict[int, int]):
    """Compile an Expr tree to (leaf_views, leaf_rows, prog).

    ``view_index`` maps id(DeviceView) -> slot in the batch view table (it is
    extended as new views are seen).  Raises CompileError when the tree does
    not fit the kernel's limits (16 leaves, 32 ops, stack depth 4).
    """
    leaf_views: List[int] = []
    leaf_rows: List[int] = []
    leaf_ids: Dict[Tuple[int, int], int] = {}
    prog: List[int] = []
    depth = [0, 0]  # current, max

    def emit(node):
        if type(node) is Leaf:
            v = node.view
            vi = view_index.get(id(v))
            if vi is None:
                vi = view_index[id(v)] = len(view_index)
            d = v.dense(node.row)
            key = (vi, d)
            k = leaf_ids.get(key)
            if k is None:
                if len(leaf_views) >= MAXLEAF:
                    raise CompileError("too many leaves")
                k = leaf_ids[key] = len(leaf_views)
                leaf_views.append(vi)
                leaf_rows.append(d)
            prog.append(k)
            depth[0] += 1
            if depth[0] > depth[1]:
                depth[1] = depth[0]
            return
        if type(node) is not Op or node.op not in _OPS:
            raise CompileError(f"bad node {node!r}")
        args = node.args
        if len(args) == 0:
            raise CompileError("empty op")
        emit(args[0])
        code = _OPS[node.op]
        for a in args[1:]:
            emit(a)
            prog.append(code)
            depth[0] -= 1
    emit(expr)
    if len(prog) > MAXPROG or depth[1] > 4:
        raise CompileError("program too large")
    return leaf_views, leaf_rows, prog


def _canonical_and2(progs: np.ndarray) -> np.ndarray:
    """Intersect(Row(a), Row(a)) compiles to one leaf with prog [0, 0, AND];
    give it a second (identical) leaf so it takes the pair-kernel route."""
    pg = progs["prog"]
    m = (progs["nprog"] == 3) & (progs["nleaf"] == 1) & (pg[:, 0] == 0) & (pg[:, 1] == 0) & (pg[:, 2] == OP_AND)
    if not m.any():
        return progs
    progs = progs.copy()
    idx = np.nonzero(m)[0]
    progs["nleaf"][idx] = 2
    progs["leaf_row"][idx, 1] = progs["leaf_row"][idx, 0]
    progs["leaf_view"][idx, 1] = progs["leaf_view"][idx, 0]
    progs["prog"][idx, 1] = 1
    return progs


def pack_programs(compiled) -> np.ndarray:
    """List of (leaf_views, leaf_rows, prog) -> QPROG_DTYPE array."""
    Q = len(compiled)
    progs = np.zeros(Q, dtype=QPROG_DTYPE)
    lv = np.zeros((Q, MAXLEAF), np.int32)
    lr = np.zeros((Q, MAXLEAF), np.int64)
    pg = np.zeros((Q, MAXPROG), np.uint8)
    nl = np.zeros(Q, np.int32)
    npg = np.zeros(Q, np.int32)
    for i, (v, r, p) in enumerate(compiled):
        n = len(v)
        nl[i] = n
        lv[i, :n] = v
        lr[i, :n] = r
        npg[i] = len(p)
        pg[i, :len(p)] = p
    progs["nleaf"] = nl
    progs["nprog"] = npg
    progs["leaf_view"] = lv
    progs["leaf_row"] = lr
    progs["prog"] = pg
    return progs


# ---------------------------------------------------------------- arena

class DeviceView:
    """One field-view's containers for a contiguous range of local shards,
    resident on one GPU."""

    # container_merge / container_emit launches (device write replay); a class
    # default so the __new__-built views (from_device, from_host_index) count too
    write_launches = 0

    def __init__(self, rows, rowptr, shard_base, meta, payload, device, shards: Sequence[int] = ()):
        import torch

        self.device = torch.device(device)
        self.rows = np.ascontiguousarray(rows, dtype=np.uint64)
        self.S = int(rowptr.shape[0])
        self.D = int(self.rows.shape[0])
        self.shards = list(shards) if shards else list(range(self.S))
        nb = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
        self.t_rowptr = nb(rowptr.view(np.int32).reshape(-1)).to(self.device, non_blocking=False)
        self.t_shard_base = nb(shard_base.astype(np.int64)).to(self.device)
        self.t_meta = nb(meta.astype(np.int64, copy=False)).to(self.device)
        self.t_payload = nb(payload.view(np.int16)).to(self.device)
        self.container_count = int(shard_base[-1])
        self._row_index = None
        self.generation = 0          # bumped by in-place shard updates
        # what changed since a given generation, for incremental dependents
        # (the TopN slot index refreshes only the shards whose bits changed):
        # shard_gen[si] counts content changes of shard si, rows_gen changes
        # of the dense row directory
        self.shard_gen = np.zeros(self.S, np.int64)
        self.rows_gen = 0
        self._sb_host = np.asarray(shard_base, dtype=np.int64).copy()
        self._cap = None             # per-shard meta capacity (patchable arenas)
        self.payload_used = int(payload.shape[0])
        self.garbage_u16 = 0
        self.write_launches = 0      # container_merge / container_emit launches (device write replay)

    # ------------------------------------------------------------ patchable layout
    @classmethod
    def patchable(cls, rows, rowptr, shard_base, meta, payload, device, shards=(), slack: float = 0.125,
                  payload_slack: float = 0.25) -> "DeviceView":
        """Like the constructor, but every shard's metadata segment and the
        payload get spare capacity so a changed shard can be rewritten in
        place (:meth:`update_shard`) instead of re-uploading the whole view."""
        shard_base = np.asarray(shard_base, dtype=np.int64)
        n = np.diff(shard_base)
        cap = n + np.maximum(16, (n * slack).astype(np.int64))
        nsb = np.zeros(len(shard_base), np.int64)
        nsb[1:] = np.cumsum(cap)
        nmeta = np.zeros(max(int(nsb[-1]), 1), np.int64)
        if len(meta) and int(shard_base[-1]):
            src = np.repeat(nsb[:-1] - shard_base[:-1], n) + np.arange(int(shard_base[-1]))
            nmeta[src] = meta[:int(shard_base[-1])]
        used = int(payload.shape[0])
        pcap = used + max(8 << 20, int(used * payload_slack))  # >= 16 MB of room for patches
        npay = np.zeros(pcap, np.uint16)
        npay[:used] = payload
        self = cls(rows, rowptr, nsb, nmeta, npay, device, shards)
        self.container_count = int(nsb[-1])
        self._cap = cap
        self.payload_used = used
        # host mirrors of the metadata for row-level patches
        self._meta_host = nmeta
        self._rowptr_host = np.asarray(rowptr, dtype=np.int64).reshape(self.S, self.D + 1).copy()
        return self

    def add_rows(self, new_rows) -> bool:
        """Insert row ids into the dense directory in place: every shard gets an
        empty container range for them (device rowptr re-gathered column-wise,
        host mirror likewise), so a write that creates a row patches the arena
        instead of rebuilding it.  Dense indices shift: generation is bumped,
        which invalidates everything keyed on them (TopN index, BSI views)."""
        import torch

        if self._cap is None:
            return False
        new = np.setdiff1d(np.asarray(new_rows, dtype=np.uint64), self.rows)
        if not len(new):
            return True
        merged = np.union1d(self.rows, new).astype(np.uint64)
        if len(merged) >= (1 << 31):
            return False
        # new column c starts where the first old row >= merged[c] starts
        src = np.searchsorted(self.rows, merged).astype(np.int64)
        src = np.concatenate([src, [self.D]])
        D2 = len(merged)
        rp = self.t_rowptr.view(self.S, self.D + 1)
        idx = torch.from_numpy(src).to(self.device)
        self.t_rowptr = torch.index_select(rp, 1, idx).contiguous().view(-1)
        self._rowptr_host = np.take(self._rowptr_host, src, axis=1)
        self.rows = merged
        self.D = D2
        self._row_index = None
        self.generation += 1
        self.rows_gen += 1
        return True

    def update_rows(self, si: int, rows, storage, keys=()) -> bool:
        """Patch local shard ``si`` in place: every container of ``rows`` (row
        ids) and the single containers ``keys`` (row*16 + local key) are
        rebuilt from the fragment storage and spliced into the shard's
        metadata segment; the payload grows by just those containers."""
        import torch

        from pilosa_amd import _roaring

        if self._cap is None:
            return False
        from pilosa_amd import shardwidth
        rows = set(int(r) for r in rows)
        keys = sorted(int(shardwidth.device_key(int(k))) for k in keys)   # arena keys row*16 + j
        keys = [k for k in keys if (k >> 4) not in rows]
        if not rows and not keys:
            return True
        touched = sorted(rows | {k >> 4 for k in keys})
        dense_of = dict(zip(touched, self.dense_many(np.array(touched, np.uint64)).tolist()))
        if any(d < 0 for d in dense_of.values()):
            if not self.add_rows([r for r, d in dense_of.items() if d < 0]):
                return False
            dense_of = dict(zip(touched, self.dense_many(np.array(touched, np.uint64)).tolist()))
        # storage positions are row * ShardWidth + column; the arena's rows are
        # 2^20 columns wide (identity for 2^20-column shards); a wider shard's
        # device sub-shard takes columns [sub * 2^20, (sub + 1) * 2^20) of it
        sw, dw, cw = shardwidth.SHARD_WIDTH, 1 << 20, 1 << 16
        sub = int(self.shards[si]) % shardwidth.DEVICE_SUBSHARDS if shardwidth.WIDE else 0
        base, span = sub * dw, min(sw, dw)
        parts = [storage.offset_range(r * dw, r * sw + base, r * sw + base + span) for r in sorted(rows)]
        parts += [storage.offset_range(k * cw, shardwidth.host_key(k, sub) * cw, (shardwidth.host_key(k, sub) + 1) * cw)
                  for k in keys]
        part = _roaring.Bitmap()
        part.union_in_place(parts)
        rows_s, rp_s, sb_s, meta_s, pay_s = _roaring.build_arena([part], 16, 1)
        n_part = int(sb_s[-1])
        npay = int(pay_s.shape[0]) if n_part else 0
        if self.payload_used + npay > int(self.t_payload.numel()) and not self.grow_payload(npay):
            return False
        new_meta = np.zeros(n_part, np.int64)
        if n_part:
            mm = meta_s[:n_part].astype(np.int64).view(np.uint64)
            off = (mm >> np.uint64(23)) + np.uint64(self.payload_used // 8)
            new_meta = ((mm & np.uint64((1 << 23) - 1)) | (off << np.uint64(23))).view(np.int64)
        fresh = {}  # row id -> new metas of that row (only the rebuilt keys)
        rps = rp_s[0].astype(np.int64) if len(rows_s) else None
        for k, r in enumerate(rows_s.tolist()):
            fresh[int(r)] = new_meta[rps[k]:rps[k + 1]]
        keys_of: Dict[int, set] = {}
        for k in keys:
            keys_of.setdefault(k >> 4, set()).add(k & 15)
        base = int(self._sb_host[si])
        rp_old = self._rowptr_host[si]
        seg_old = self._meta_host[base:base + int(rp_old[-1])]
        counts = np.diff(rp_old)
        pieces, cur = [], 0
        for r in touched:
            d = dense_of[r]
            pieces.append(seg_old[rp_old[cur]:rp_old[d]])
            nm = fresh.get(r, np.zeros(0, np.int64))
            if r not in rows:  # splice single keys into the row's old containers
                old = seg_old[rp_old[d]:rp_old[d + 1]]
                ks = keys_of[r]
                keep = old[~np.isin(old & 15, list(ks))]
                nm = np.concatenate([keep, nm])
                nm = nm[np.argsort(nm & 15, kind="stable")]
            pieces.append(nm)
            counts[d] = len(nm)
            cur = d + 1
        pieces.append(seg_old[rp_old[cur]:rp_old[-1]])
        seg = np.concatenate(pieces)
        if len(seg) > int(self._cap[si]):
            if not self.grow_segment(si, len(seg)):
                return False
            base = int(self._sb_host[si])
        rp_new = np.zeros(self.D + 1, np.int64)
        rp_new[1:] = np.cumsum(counts)
        full = np.zeros(int(self._cap[si]), np.int64)
        full[:len(seg)] = seg
        dev = self.device
        if npay:
            self.t_payload[self.payload_used:self.payload_used + npay].copy_(
                torch.from_numpy(pay_s[:npay].view(np.int16)).to(dev))
        self.t_meta[base:base + len(full)].copy_(torch.from_numpy(full).to(dev))
        self.t_rowptr.view(self.S, self.D + 1)[si].copy_(torch.from_numpy(rp_new.astype(np.int32)).to(dev))
        self._meta_host[base:base + len(full)] = full
        self._rowptr_host[si] = rp_new
        self.payload_used += npay
        self.garbage_u16 += npay
        self.generation += 1
        self.shard_gen[si] += 1
        return True

    def update_shard(self, si: int, bitmap) -> bool:
        """Rewrite local shard ``si`` from a host bitmap in place (metadata
        segment, rowptr row, payload appended at the tail).  False when the
        view must be rebuilt instead: not patchable, a row id outside the
        directory, segment or payload capacity exceeded, or too much garbage."""
        import torch

        from pilosa_amd import _roaring

        if self._cap is None:
            return False
        from pilosa_amd import shardwidth
        # (a wider shard's sub-shard arrives re-keyed to 2^20 columns: ARENA_CPR)
        rows_s, rp_s, sb_s, meta_s, pay_s = _roaring.build_arena([bitmap], shardwidth.ARENA_CPR, 1)
        n_new = int(sb_s[-1])
        if n_new > int(self._cap[si]) and not self.grow_segment(si, n_new):
            return False
        dense = self.dense_many(rows_s) if len(rows_s) else np.zeros(0, np.int64)
        if len(dense) and (dense < 0).any():
            if not self.add_rows(rows_s[dense < 0]):
                return False
            dense = self.dense_many(rows_s)
        npay = int(pay_s.shape[0]) if n_new else 0
        if self.payload_used + npay > int(self.t_payload.numel()) and not self.grow_payload(npay):
            return False
        # rowptr over the view's full row directory
        counts = np.zeros(self.D, np.int64)
        if len(dense):
            counts[dense] = np.diff(rp_s[0].astype(np.int64))
        rowptr = np.zeros(self.D + 1, np.int64)
        rowptr[1:] = np.cumsum(counts)
        m = np.zeros(int(self._cap[si]), np.int64)
        if n_new:
            mm = meta_s[:n_new].astype(np.int64)
            off = (mm.view(np.uint64) >> np.uint64(23)) + np.uint64(self.payload_used // 8)
            m[:n_new] = ((mm.view(np.uint64) & np.uint64((1 << 23) - 1)) | (off << np.uint64(23))).view(np.int64)
        base = int(self._sb_host[si])
        dev = self.device
        self.t_meta[base:base + len(m)].copy_(torch.from_numpy(m).to(dev))
        self.t_rowptr.view(self.S, self.D + 1)[si].copy_(torch.from_numpy(rowptr.astype(np.int32)).to(dev))
        self._meta_host[base:base + len(m)] = m
        self._rowptr_host[si] = rowptr
        if npay:
            self.t_payload[self.payload_used:self.payload_used + npay].copy_(
                torch.from_numpy(pay_s[:npay].view(np.int16)).to(dev))
        self.payload_used += npay
        self.garbage_u16 += npay  # approximate: the shard's previous payload is now unreachable
        self.generation += 1
        self.shard_gen[si] += 1
        return True

    # ------------------------------------------------------------ growth
    def grow_segment(self, si: int, need: int) -> bool:
        """Re-lay the metadata array so shard ``si`` has room for ``need``
        containers: each shard's used part is copied device-to-device into
        the new layout (the payload is untouched), so an overflowing shard
        costs one pass over the metadata instead of a rebuild from the host."""
        import torch

        if self._cap is None:
            return False
        cap = self._cap.copy()
        cap[si] = need + max(16, need // 8)
        nsb = np.zeros(self.S + 1, np.int64)
        nsb[1:] = np.cumsum(cap)
        t_new = torch.zeros(max(int(nsb[-1]), 1), dtype=torch.int64, device=self.device)
        h_new = np.zeros(max(int(nsb[-1]), 1), np.int64)
        for s in range(self.S):
            n = int(self._rowptr_host[s][-1])
            if n:
                a, b = int(self._sb_host[s]), int(nsb[s])
                t_new[b:b + n].copy_(self.t_meta[a:a + n])
                h_new[b:b + n] = self._meta_host[a:a + n]
        self.t_meta, self._meta_host, self._cap = t_new, h_new, cap
        self._sb_host = nsb
        self.t_shard_base = torch.from_numpy(nsb.copy()).to(self.device)
        self.container_count = int(nsb[-1])
        self.generation += 1
        return True

    def grow_payload(self, need_u16: int) -> bool:
        """Room for ``need_u16`` more payload values (a larger buffer, the
        used prefix copied device-to-device)."""
        import torch

        if self._cap is None:
            return False
        want = self.payload_used + need_u16
        if want <= int(self.t_payload.numel()):
            return True
        size = want + max(8 << 20, want // 4)
        try:
            t_new = torch.empty(size, dtype=self.t_payload.dtype, device=self.device)
        except RuntimeError:   # out of device memory: the caller rebuilds
            return False
        t_new[:self.payload_used].copy_(self.t_payload[:self.payload_used])
        self.t_payload = t_new
        self.generation += 1
        return True

    def compact(self) -> bool:
        """Drop the payload left behind by in-place updates on the device:
        live containers are copied into a fresh, packed buffer
        (payload_compact_kernel) and their metadata re-pointed -- instead of
        rebuilding the view from the host fragments."""
        import torch

        if self._cap is None or self.device.type != "cuda":
            return False
        K = kernels()
        dev = self.device
        m = self.t_meta
        C = int(m.numel())
        sb = torch.from_numpy(np.asarray(self._sb_host, np.int64)).to(dev)
        used = torch.from_numpy(np.array([int(r[-1]) for r in self._rowptr_host], np.int64)).to(dev)
        pos = torch.arange(C, device=dev)
        seg = torch.clamp(torch.bucketize(pos, sb[1:], right=True), max=self.S - 1)
        live = (pos - sb[seg]) < used[seg]
        del pos, seg
        t = (m >> 4) & 3
        n = (m >> 6) & 0x1FFFF
        off16 = m >> 23
        size16 = torch.where(t == 1, (n + 7) // 8, torch.where(t == 2, torch.full_like(n, 512), torch.zeros_like(n)))
        runs = torch.nonzero(live & (t == 3)).flatten()
        if runs.numel():
            nr = self.t_payload[off16[runs] * 8].to(torch.int64) & 0xFFFF
            size16[runs] = (8 + 2 * nr + 7) // 8
        live &= t != 0
        size16 = torch.where(live, size16, torch.zeros_like(size16))
        ends = torch.cumsum(size16, 0)
        total16 = int(ends[-1]) if C else 0
        new_off16 = ends - size16
        del ends
        cap_u16 = total16 * 8 + max(8 << 20, total16 * 2)
        try:
            dst = torch.empty(cap_u16, dtype=self.t_payload.dtype, device=dev)
        except RuntimeError:
            return False
        K.payload_compact(m, new_off16, size16, self.t_payload, dst)
        new_meta = torch.where(live, (m & ((1 << 23) - 1)) | (new_off16 << 23), torch.zeros_like(m))
        self.t_meta = new_meta
        self._meta_host = new_meta.cpu().numpy()
        self.t_payload = dst
        self.payload_used = total16 * 8
        self.garbage_u16 = 0
        self.generation += 1
        self.compactions = getattr(self, "compactions", 0) + 1
        return True

    # ------------------------------------------------------------ device write path (K11/K12)
    def _seg_keys(self, si: int):
        """(segment base, shard metadata segment, sorted dense*16+j key of each)."""
        base = int(self._sb_host[si])
        rp = self._rowptr_host[si]
        seg = self._meta_host[base:base + int(rp[-1])]
        keys = np.repeat(np.arange(self.D, dtype=np.int64), np.diff(rp).astype(np.int64)) * 16 + (seg & 15)
        return base, seg, keys

    def apply_positions(self, si: int, positions, clear: bool = False) -> bool:
        """Set (or clear) shard-local positions row * ShardWidth + col of local shard
        ``si`` directly in the arena: container_merge / container_emit on the
        GPU (kernels/write_kernels.hip), only the positions go over PCIe.
        False -> the caller must refresh the shard another way."""
        return not self.apply_deltas_multi({si: [("pos", positions, clear)]})

    def apply_bitmap(self, si: int, bitmap, clear: bool = False) -> bool:
        """ImportRoaringBits on the device: OR (AND-NOT) every container of
        ``bitmap`` (shard-local positions) into the arena, container against
        container (mode 1 of container_merge)."""
        return not self.apply_deltas_multi({si: [("roaring", bitmap, clear)]})

    def apply_deltas(self, si: int, deltas) -> bool:
        """Replay one shard's recorded writes in order."""
        return not self.apply_deltas_multi({si: deltas})

    @staticmethod
    def _runs(deltas):
        """Merge consecutive position batches with the same set/clear flag."""
        out = []
        for kind, data, clear in deltas:
            if kind == "pos" and out and out[-1][0] == "pos" and out[-1][2] == clear:
                out[-1][1].append(np.asarray(data, dtype=np.uint64))
            elif kind == "pos":
                out.append(("pos", [np.asarray(data, dtype=np.uint64)], clear))
            else:
                out.append((kind, data, clear))
        return [(k, np.concatenate(d) if k == "pos" else d, c) for k, d, c in out]

    def apply_deltas_multi(self, per_shard) -> set:
        """Replay the recorded writes of several local shards: the r-th write
        run of every shard goes into the same container_merge /
        container_emit launches (grouped by kind and set/clear), so a refresh
        costs a few launches and transfers, not a few per shard.  Returns the
        shard indices whose replay failed (the caller rebuilds those)."""
        if self._cap is None or self.device.type != "cuda":
            return set(per_shard)
        runs = {si: self._runs(d) for si, d in per_shard.items() if d}
        failed: set = set()
        r = 0
        while True:
            layer = [(si, rs[r]) for si, rs in runs.items() if r < len(rs) and si not in failed]
            if not layer:
                return failed
            for kind in ("pos", "roaring"):
                for clear in (False, True):
                    group = [(si, data) for si, (k, data, c) in layer if k == kind and c == clear]
                    if group:
                        failed |= self._replay_group(group, kind, clear)
            r += 1

    def _replay_group(self, group, kind: str, clear: bool) -> set:
        from pilosa_amd import _roaring, shardwidth
        ks, cpr = shardwidth.KEY_SHIFT, shardwidth.CONTAINERS_PER_ROW

        jobs = []   # (si, container row ids, j, mode-specific arrays)
        for si, data in group:
            if kind == "pos":
                p = np.unique(np.asarray(data, dtype=np.uint64))
                if not len(p):
                    continue
                ck = (p >> np.uint64(16)).astype(np.int64)    # host container keys
                uk, start = np.unique(ck, return_index=True)
                jobs.append([si, (uk >> ks).astype(np.uint64), (uk & (cpr - 1)).astype(np.int32),
                             np.append(start, len(p)).astype(np.int64), (p & np.uint64(0xFFFF)).astype(np.uint16)])
            else:
                rows_s, rp_s, sb_s, meta_s, pay_s = _roaring.build_arena([data], cpr, 1)
                n = int(sb_s[-1])
                if not n:
                    continue
                drow = np.repeat(rows_s.astype(np.uint64), np.diff(rp_s[0].astype(np.int64)))
                dmeta = meta_s[:n].astype(np.int64)
                jobs.append([si, drow, (dmeta & 15).astype(np.int32), dmeta, pay_s])
        if not jobs:
            return set()
        # rows new to the directory: added once for the whole group (sets only)
        allrows = np.unique(np.concatenate([jb[1] for jb in jobs]))
        dense_all = self.dense_many(allrows)
        if (dense_all < 0).any() and not clear:
            if not self.add_rows(allrows[dense_all < 0]):
                return {jb[0] for jb in jobs}
        for jb in jobs:
            dense = self.dense_many(jb[1])
            if clear and (dense < 0).any():     # nothing to clear in rows this view never had
                keep = dense >= 0
                if kind == "pos":
                    counts = np.diff(jb[3])
                    lows = np.concatenate([jb[4][a:b] for a, b, k in zip(jb[3][:-1], jb[3][1:], keep) if k]) \
                        if keep.any() else np.zeros(0, np.uint16)
                    jb[3] = np.concatenate([[0], np.cumsum(counts[keep])]).astype(np.int64)
                    jb[4] = lows
                else:
                    jb[3] = jb[3][keep]
                jb[1], jb[2], dense = jb[1][keep], jb[2][keep], dense[keep]
            jb.append(dense)
        jobs = [jb for jb in jobs if len(jb[1])]
        if not jobs:
            return set()
        return self._merge_jobs(jobs, 0 if kind == "pos" else 1, clear)

    # containers per merge launch: 2 GiB of bitmap scratch (8 KiB each) on a
    # 288 GB device, so an import request's whole batch of shards shares a few launches
    WRITE_CHUNK = 1 << 18

    def _merge_jobs(self, jobs, mode: int, clear: bool) -> set:
        """Merge + emit every job's containers in shared launches, then splice
        each shard's new metadata words into its segment."""
        import torch

        K = kernels()
        dev = self.device
        seg_info, olds, js, qks = [], [], [], []
        for jb in jobs:
            si, dense, j = jb[0], jb[-1], jb[2]
            base, seg, segkeys = self._seg_keys(si)
            qk = dense.astype(np.int64) * 16 + j
            if len(segkeys):
                idx = np.minimum(np.searchsorted(segkeys, qk), len(segkeys) - 1)
                found = segkeys[idx] == qk
                old = np.where(found, seg[idx], -1).astype(np.int64)
            else:
                idx = np.zeros(len(qk), np.int64)
                found = np.zeros(len(qk), bool)
                old = np.full(len(qk), -1, np.int64)
            seg_info.append((si, seg, segkeys, qk, idx, found, old))
            olds.append(old)
            js.append(j)
        U = sum(len(o) for o in olds)
        t_old = torch.from_numpy(np.concatenate(olds)).to(dev)
        t_j = torch.from_numpy(np.ascontiguousarray(np.concatenate(js), dtype=np.int32)).to(dev)
        empty16 = torch.empty(0, dtype=torch.int16, device=dev)
        empty64 = torch.empty(0, dtype=torch.int64, device=dev)
        empty32 = torch.empty(1, dtype=torch.int32, device=dev)
        if mode == 0:
            offs = np.cumsum([0] + [len(jb[4]) for jb in jobs])
            dstart = np.concatenate([jb[3][:-1] + offs[k] for k, jb in enumerate(jobs)] + [[offs[-1]]]).astype(np.int64)
            t_lows = torch.from_numpy(np.concatenate([jb[4] for jb in jobs]).view(np.int16)).to(dev)
        else:
            pays, metas, at16 = [], [], 0
            for jb in jobs:
                mm = jb[3].view(np.uint64)
                metas.append(((mm & np.uint64((1 << 23) - 1)) | (((mm >> np.uint64(23)) + np.uint64(at16))
                                                                 << np.uint64(23))).view(np.int64))
                pays.append(np.ascontiguousarray(jb[4]))
                at16 += len(jb[4]) // 8
            t_dmeta = torch.from_numpy(np.concatenate(metas)).to(dev)
            t_dpay = torch.from_numpy(np.concatenate(pays).view(np.int16)).to(dev)
        new_meta = np.empty(U, np.int64)
        used = self.payload_used
        for c0 in range(0, U, self.WRITE_CHUNK):
            c1 = min(U, c0 + self.WRITE_CHUNK)
            n = c1 - c0
            scratch = torch.empty(n * 1024, dtype=torch.int64, device=dev)
            card = torch.empty(n, dtype=torch.int32, device=dev)
            nruns = torch.empty(n, dtype=torch.int32, device=dev)
            if mode == 0:
                a, b = int(dstart[c0]), int(dstart[c1])
                ds = torch.from_numpy((dstart[c0:c1 + 1] - a).astype(np.int32)).to(dev)
                K.container_merge(t_old[c0:c1], self.t_payload, ds, t_lows[a:b], empty64, empty16, 0, clear, scratch,
                                  card, nruns)
            else:
                K.container_merge(t_old[c0:c1], self.t_payload, empty32, empty16, t_dmeta[c0:c1], t_dpay, 1, clear,
                                  scratch, card, nruns)
            c64, r64 = card.to(torch.int64), nruns.to(torch.int64)
            # the reference's Optimize choice (write_kernels.hip emit_type):
            # run if runs <= 2048 and runs <= n/2, array if n < 4096, else bitmap
            is_run = (r64 <= 2048) & (r64 <= c64 // 2)
            sizes = torch.where(c64 == 0, torch.zeros_like(c64),
                                torch.where(is_run, (8 + 2 * r64 + 7) // 8 * 8,
                                            torch.where(c64 < 4096, (c64 + 7) // 8 * 8, torch.full_like(c64, 4096))))
            ends = torch.cumsum(sizes, 0)
            tot = int(ends[-1])
            if used + tot > int(self.t_payload.numel()):
                self.payload_used, prev = used, self.payload_used
                grown = self.grow_payload(tot)
                self.payload_used = prev
                if not grown:
                    return {jb[0] for jb in jobs}
            off16 = (ends - sizes + used) // 8
            meta_out = torch.empty(n, dtype=torch.int64, device=dev)
            K.container_emit(scratch, card, nruns, off16, t_j[c0:c1], self.t_payload, meta_out)
            self.write_launches += 2   # one merge + one emit launch for every shard of the group
            new_meta[c0:c1] = meta_out.cpu().numpy()
            used += tot
        self.payload_used = used
        failed = set()
        at = 0
        scatter_at, scatter_val = [], []
        for si, seg, segkeys, qk, idx, found, old in seg_info:
            nm = new_meta[at:at + len(qk)]
            at += len(qk)
            keep = nm >= 0
            old_n = (old >> 6) & 0x1FFFF
            old_t = (old >> 4) & 3
            # a run container's size is in its header, not its metadata: count the header only
            self.garbage_u16 += int(np.where(found, np.where(old_t == 2, 4096, np.where(old_t == 3, 8, (old_n + 7) // 8 * 8)),
                                             0).sum())
            base = int(self._sb_host[si])
            if not (found & ~keep).any() and not (~found & keep).any():
                pos = base + idx[found]
                self._meta_host[pos] = nm[found]
                scatter_at.append(pos)
                scatter_val.append(nm[found])
                continue
            kept = np.ones(len(seg), bool)
            kept[idx[found & ~keep]] = False          # containers that became empty
            ins = keep & ~found
            repl = keep & found
            seg2 = seg.copy()
            seg2[idx[repl]] = nm[repl]
            keys = np.concatenate([segkeys[kept], qk[ins]])
            vals = np.concatenate([seg2[kept], nm[ins]])
            order = np.argsort(keys, kind="stable")
            keys, vals = keys[order], vals[order]
            if len(vals) > int(self._cap[si]):
                if scatter_at:   # a re-layout moves segments: flush pending in-place updates first
                    self._flush_meta_scatter(scatter_at, scatter_val)
                    scatter_at, scatter_val = [], []
                if not self.grow_segment(si, len(vals)):
                    failed.add(si)
                    continue
                base = int(self._sb_host[si])
            rp_new = np.zeros(self.D + 1, np.int64)
            rp_new[1:] = np.cumsum(np.bincount(keys >> 4, minlength=self.D)[:self.D])
            full = np.zeros(int(self._cap[si]), np.int64)
            full[:len(vals)] = vals
            self.t_meta[base:base + len(full)].copy_(torch.from_numpy(full).to(dev))
            self.t_rowptr.view(self.S, self.D + 1)[si].copy_(torch.from_numpy(rp_new.astype(np.int32)).to(dev))
            self._meta_host[base:base + len(full)] = full
            self._rowptr_host[si] = rp_new
        if scatter_at:
            self._flush_meta_scatter(scatter_at, scatter_val)
        self.generation += 1
        for jb in jobs:
            self.shard_gen[jb[0]] += 1
        return failed

    def _flush_meta_scatter(self, at, val):
        import torch
        pos = np.concatenate(at)
        if len(pos):
            self.t_meta.index_copy_(0, torch.from_numpy(pos).to(self.device),
                                    torch.from_numpy(np.concatenate(val)).to(self.device))

    def needs_compaction(self) -> bool:
        """Dead payload from in-place updates exceeds half the buffer."""
        return self._cap is not None and self.garbage_u16 > int(self.t_payload.numel()) // 2

    @classmethod
    def from_device(cls, rows: np.ndarray, t_rowptr, t_shard_base, t_meta, t_payload, device, shards,
                    container_count: int) -> "DeviceView":
        """Wrap device tensors produced on the GPU (e.g. BSI predicate results)."""
        import torch

        self = cls.__new__(cls)
        self.device = torch.device(device)
        self.rows = np.ascontiguousarray(rows, dtype=np.uint64)
        self.S = int(t_shard_base.numel()) - 1
        self.D = int(self.rows.shape[0])
        self.shards = list(shards)
        self.t_rowptr, self.t_shard_base, self.t_meta, self.t_payload = t_rowptr, t_shard_base, t_meta, t_payload
        self.container_count = int(container_count)
        self._row_index = None
        self.generation = 0
        self.shard_gen = np.zeros(self.S, np.int64)
        self.rows_gen = 0
        self._cap = None
        self.payload_used = int(t_payload.numel())
        self.garbage_u16 = 0
        return self

    @classmethod
    def from_host_index(cls, rows, rowptr, shard_base, meta, t_payload, payload_used: int, device, shards,
                        cap=None) -> "DeviceView":
        """Wrap an arena index built on the host (ops/loader.py) around an
        already uploaded payload; ``cap`` (per-shard metadata capacity) makes
        the view patchable, the host index arrays then stay as its mirrors."""
        import torch

        self = cls.__new__(cls)
        self.device = torch.device(device)
        self.rows = np.ascontiguousarray(rows, dtype=np.uint64)
        self.S = int(rowptr.shape[0])
        self.D = int(self.rows.shape[0])
        self.shards = list(shards) if shards else list(range(self.S))
        rowptr = np.ascontiguousarray(rowptr, dtype=np.uint32).reshape(self.S, self.D + 1)
        self.t_rowptr = torch.from_numpy(rowptr.view(np.int32).reshape(-1)).to(self.device)
        self.t_shard_base = torch.from_numpy(np.ascontiguousarray(shard_base, dtype=np.int64)).to(self.device)
        self.t_meta = torch.from_numpy(np.ascontiguousarray(meta, dtype=np.int64)).to(self.device)
        self.t_payload = t_payload
        self.container_count = int(shard_base[-1])
        self._row_index = None
        self.generation = 0
        self.shard_gen = np.zeros(self.S, np.int64)
        self.rows_gen = 0
        self._sb_host = np.asarray(shard_base, dtype=np.int64).copy()
        self.payload_used = int(payload_used)
        self.garbage_u16 = 0
        self._cap = None
        if cap is not None:
            self._cap = np.asarray(cap, dtype=np.int64)
            self._meta_host = meta
            self._rowptr_host = rowptr
        return self

    @classmethod
    def from_bitmaps(cls, bitmaps: Sequence[Optional[object]], device, shards=(), patchable: bool = False,
                     cpr: Optional[int] = None):
        """Arena of per-shard bitmaps of shard-local positions row * ShardWidth
        + column (``cpr`` containers per row, default the shard width's; a
        wider shard's sub-shards arrive re-keyed to 2^20 columns,
        ``Bitmap.sub_shard``)."""
        from pilosa_amd import _roaring, shardwidth

        cpr = shardwidth.ARENA_CPR if cpr is None else int(cpr)
        rows, rowptr, sb, meta, payload = _roaring.build_arena(list(bitmaps), cpr, 8)
        if patchable:
            return cls.patchable(rows, rowptr, sb, meta, payload, device, shards)
        return cls(rows, rowptr, sb, meta, payload, device, shards)

    def nbytes(self) -> int:
        n = sum(t.numel() * t.element_size() for t in (self.t_rowptr, self.t_shard_base, self.t_meta,
                                                       self.t_payload))
        sh = getattr(self, "_shadow", None)
        return n + (sh[1].numel() * 8 + sh[2].numel() * 4 if sh is not None else 0)

    def dense(self, row: int) -> int:
        """row id -> dense index (-1 if the row has no containers on this GPU)."""
        rows = self.rows
        if self.D and rows[-1] == self.D - 1:  # identity directory (rows 0..D-1)
            return int(row) if 0 <= row < self.D else -1
        i = int(np.searchsorted(rows, np.uint64(row)))
        if i < self.D and int(rows[i]) == int(row):
            return i
        return -1

    def dense_many(self, rows: np.ndarray) -> np.ndarray:
        rows = np.asarray(rows, dtype=np.uint64)
        i = np.searchsorted(self.rows, rows)
        i = np.minimum(i, max(self.D - 1, 0))
        ok = (self.D > 0) & (self.rows[i] == rows) if self.D else np.zeros(len(rows), bool)
        return np.where(ok, i, -1).astype(np.int64)

    def viewdev(self) -> np.void:
        rec = np.zeros((), dtype=VIEWDEV_DTYPE)
        rec["rowptr"] = self.t_rowptr.data_ptr()
        rec["shard_base"] = self.t_shard_base.data_ptr()
        rec["meta"] = self.t_meta.data_ptr()
        rec["payload"] = self.t_payload.data_ptr()
        rec["D"] = self.D
        km = getattr(self, "_keymask", None)
        if km is not None and km[0] == self.generation:
            rec["keymask"] = km[1].data_ptr()
        sh = getattr(self, "_shadow", None)
        if sh is not None and sh[0] == self.generation:
            rec["shadow"] = sh[1].data_ptr()
            rec["shadow_slot"] = sh[2].data_ptr()
        return rec

    def shadow_fresh(self) -> bool:
        sh = getattr(self, "_shadow", None)
        return sh is not None and sh[0] == self.generation

    # dense bitmap shadows of the hottest rows (pair_kernels.hip SHD): up to
    # SHADOW_ROWS rows, within SHADOW_MAX_BYTES and a quarter of free HBM
    SHADOW_ROWS = int(os.environ.get("PILOSA_SHADOW_ROWS", "256"))
    SHADOW_MAX_BYTES = int(os.environ.get("PILOSA_SHADOW_MAX_GB", "40")) << 30
    SHADOW_MIN_INTERVAL_S = 30.0
    SHADOW_SAMPLE_SHARDS = 8

    def _hot_dense_rows(self, R: int) -> np.ndarray:
        """The R dense rows with the most bits over a sample of shards
        (a hot row of a Zipf-like field is hot in every shard)."""
        D1 = self.D + 1
        picks = sorted(set(np.linspace(0, self.S - 1, min(self.S, self.SHADOW_SAMPLE_SHARDS)).astype(int).tolist()))
        tot = np.zeros(self.D, np.int64)
        sb = self._sb_host
        for si in picks:
            rp = self.t_rowptr[si * D1:(si + 1) * D1].cpu().numpy().astype(np.int64)
            n = int(rp[-1])
            if n == 0:
                continue
            m = self.t_meta[int(sb[si]):int(sb[si]) + n].cpu().numpy()
            card = (m >> 6) & 0x1FFFF
            row = np.repeat(np.arange(self.D, dtype=np.int64), np.diff(rp))
            tot += np.bincount(row, weights=card, minlength=self.D).astype(np.int64)
        R = min(R, int((tot > 0).sum()))
        if R <= 0:
            return np.zeros(0, np.int32)
        top = np.argpartition(-tot, R - 1)[:R]
        return np.sort(top).astype(np.int32)

    def ensure_shadow(self) -> bool:
        """Build (or refresh, at most every SHADOW_MIN_INTERVAL_S after
        writes) the dense bitmap shadows of this view's hottest rows: each
        row's container of every (shard, key) as a 1024-word bitmap in HBM,
        so the pair kernels stage it with one coalesced copy or read it in
        place.  A stale shadow is simply not passed.  Returns whether it is
        fresh."""
        import time

        import torch

        if self.SHADOW_ROWS <= 0 or self.device.type != "cuda" or not self.S or not self.D or \
                not hasattr(kernels(), "shadow_build"):
            return False
        sh = getattr(self, "_shadow", None)
        if sh is not None and sh[0] == self.generation:
            return True
        now = time.monotonic()
        if sh is not None and now - sh[3] < self.SHADOW_MIN_INTERVAL_S:
            return False
        if sh is None and getattr(self, "_shadow_declined", None) == self.generation:
            return False
        per_row = self.S * 16 * 8192
        free, _ = torch.cuda.mem_get_info(self.device)
        R = min(self.SHADOW_ROWS, self.D, int(min(free // 4, self.SHADOW_MAX_BYTES) // per_row))
        rows = self._hot_dense_rows(R) if R >= 8 else np.zeros(0, np.int32)
        if len(rows) < 8:
            self._shadow_declined = self.generation
            return False
        R = len(rows)
        buf = sh[1] if sh is not None and sh[1].numel() == R * self.S * 16 * 1024 else None
        if buf is None:
            self._shadow = None
            buf = torch.empty(R * self.S * 16 * 1024, dtype=torch.int64, device=self.device)
        slot = torch.full((self.D,), -1, dtype=torch.int32)
        slot[torch.from_numpy(rows.astype(np.int64))] = torch.arange(R, dtype=torch.int32)
        slot = slot.to(self.device)
        self.ensure_keymask()
        kernels().shadow_build(self.viewdev_tensor(), self.S, torch.from_numpy(rows).to(self.device), buf)
        # readers on any stream see a complete shadow
        torch.cuda.current_stream(self.device).synchronize()
        self._shadow = (self.generation, buf, slot, now, rows)
        return True

    def viewdev_tensor(self):
        """The ViewDev record as the uint8 host tensor the kernel bindings take."""
        import torch
        return torch.from_numpy(np.frombuffer(self.viewdev().tobytes(), dtype=np.uint8).copy())

    KEYMASK_MIN_INTERVAL_S = 5.0

    def ensure_keymask(self) -> bool:
        """Build the [S][D] key-presence mask table the pair kernels read
        instead of each row's metas (pair_kernels.hip keymask_build_kernel).
        It is tied to the view generation; after writes it is rebuilt at most
        every KEYMASK_MIN_INTERVAL_S seconds, and a stale table is simply not
        passed (the kernels then read metas).  Returns whether it is fresh."""
        import time

        import torch

        if os.environ.get("PILOSA_KEYMASK", "1") == "0" or self.device.type != "cuda":
            return False
        km = getattr(self, "_keymask", None)
        if km is not None and km[0] == self.generation:
            return True
        now = time.monotonic()
        if km is not None and now - km[2] < self.KEYMASK_MIN_INTERVAL_S:
            return False
        n = self.S * self.D
        if n == 0:
            return False
        if km is None or km[1].numel() != n:
            # HBM guard: the table (2 B per (shard, row)) is skipped for views
            # whose row directory is large next to their containers, or when
            # it would not leave the device comfortably free
            need = 2 * n
            sh = getattr(self, "_shadow", None)
            arena = self.nbytes() - (sh[1].numel() * 8 + sh[2].numel() * 4 if sh is not None else 0)
            if need > max(256 << 20, arena // 4):
                return False
            free, _ = torch.cuda.mem_get_info(self.device)
            if need * 4 > free:
                return False
        out = km[1] if km is not None and km[1].numel() == n else torch.empty(n, dtype=torch.int16,
                                                                               device=self.device)
        rec = np.zeros((), dtype=VIEWDEV_DTYPE)
        rec["rowptr"] = self.t_rowptr.data_ptr()
        rec["shard_base"] = self.t_shard_base.data_ptr()
        rec["meta"] = self.t_meta.data_ptr()
        rec["payload"] = self.t_payload.data_ptr()
        rec["D"] = self.D
        kernels().keymask_build(torch.from_numpy(np.frombuffer(rec.tobytes(), dtype=np.uint8).copy()), self.S, out)
        self._keymask = (self.generation, out, now)
        return True


# ---------------------------------------------------------------- engine

class DeviceRowBlock:
    """A row result's containers on the device: per (shard, key) count
    (int32[S*16]; > 4096 = bitmap) and u16 offset (int64[S*16]) into a u16
    payload, for the device shards ``shards``; ``spill`` is the block of the
    bits a Shift carried past each shard's last column (or None).  A rank of
    a multi-GPU node sends its Row partial as these tensors (no host Row, no
    roaring serialisation, parallel/collectives.encode_row_block)."""

    __slots__ = ("shards", "counts", "offs", "payload", "spill")

    def __init__(self, shards, counts, offs, payload, spill=None):
        self.shards, self.counts, self.offs, self.payload, self.spill = list(shards), counts, offs, payload, spill

    def host(self):
        return (self.counts.cpu().numpy(), self.offs.cpu().numpy(), self.payload.cpu().numpy().view(np.uint16))


class GpuEngine:
    """Batched query execution on one GPU (all views must share the shard list)."""

    def __init__(self, device):
        import torch

        self.torch = torch
        self.device = torch.device(device)
        self.ext = kernels()
        self.copy_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        # Count(Intersect(a,b)) route: key-major pair kernels (pair_kernels.hip)
        self.use_and2 = os.environ.get("PILOSA_AND2", "1") != "0"
        self.and2_cq = int(os.environ.get("PILOSA_AND2_CQ", "0"))  # 0 = by batch size
        self.and2_variant = int(os.environ.get("PILOSA_AND2_VARIANT", "6"))
        # dense bitmap shadows of hot rows for the pair kernels (DeviceView.ensure_shadow)
        # (off by default: measured slower -- headline 16.66 vs 16.45 ms, serving
        # 61.5k vs 69.3k req/s, profiles/r05_serve/ -- the staged LDS probes beat
        # reading a 8 KiB shadow in place, and the hot A rows are mostly bitmaps)
        # dense shadows of hot rows (variants 41 / 42): measured slower, built
        # into the kbench module only (profiles/r05_shadow/)
        self.use_shadow = os.environ.get("PILOSA_SHADOW", "0") != "0" and hasattr(kernels(), "shadow_build")
        # Count(Union(leaves)) route: union_count_kernel (bitmap_kernels.hip)
        self.use_union = os.environ.get("PILOSA_UNION_KERNEL", "1") != "0"
        # 2 = union_count2_kernel (flat chunk walk, parallel meta fetch), 1 = union_count_kernel
        self.union_variant = int(os.environ.get("PILOSA_UNION_VARIANT", "2"))

    def _views_tensor(self, views: List["DeviceView"]):
        arr = np.zeros(len(views), dtype=VIEWDEV_DTYPE)
        for i, v in enumerate(views):
            arr[i] = v.viewdev()
        # the same view table (same arenas, same buffers) is uploaded once:
        # a BSI / single-view request otherwise pays one H2D for it per call
        key = arr.tobytes()
        memo = self.__dict__.setdefault("_vt_memo", {})
        hit = memo.get(key)
        torch = self.torch
        cuda = self.device.type == "cuda"
        if hit is not None:
            t, ev = hit
            if cuda:   # another stream may read it: after the upload, and not recycled under it
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                t.record_stream(cur)
            return t
        t = self._h2d(arr.view(np.uint8))
        ev = None
        if cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        if len(memo) >= 64:
            memo.pop(next(iter(memo)))
        memo[key] = (t, ev)
        return t

    def compile_batch(self, exprs: Sequence[object]):
        view_index: Dict[int, int] = {}
        views: Dict[int, DeviceView] = {}

        def collect(node):
            if type(node) is Leaf:
                views[id(node.view)] = node.view
            elif type(node) is Op:
                for a in node.args:
                    collect(a)

        compiled = []
        for e in exprs:
            collect(e)
            compiled.append(compile_expr(e, view_index))
        progs = pack_programs(compiled)
        ordered = [None] * len(view_index)
        for vid, slot in view_index.items():
            ordered[slot] = views[vid]
        S = None
        for v in ordered:
            if S is None:
                S = v.S
            elif v.S != S:
                raise CompileError("views in one batch must share the local shard list")
        return progs, ordered, S or 0

    def _h2d(self, arr: np.ndarray):
        return self._h2d_many([arr])[0]

    def _h2d_many(self, arrs: Sequence[np.ndarray]):
        """Upload several host arrays with ONE copy from pinned memory on the
        engine's copy stream; returns uint8 device views (256B-aligned).

        Pinned staging matters: a pageable hipMemcpyAsync is serviced only
        after the device drains, which serialised batch i+1's upload behind
        batch i's kernel.  The caching host allocator keeps the staging block
        alive until the copy-stream event fires."""
        torch = self.torch
        offs, total = [], 0
        for a in arrs:
            offs.append(total)
            total += (a.nbytes + 255) & ~255
        total = max(total, 256)
        if self.copy_stream is None:
            host = np.zeros(total, np.uint8)
            for a, o in zip(arrs, offs):
                host[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
            d = torch.from_numpy(host).to(self.device)
        else:
            pt = torch.empty(total, dtype=torch.uint8, pin_memory=True)
            host = pt.numpy()
            for a, o in zip(arrs, offs):
                host[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
            with torch.cuda.stream(self.copy_stream):
                d = pt.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            d.record_stream(cur)
        return [d[o:o + a.nbytes] for a, o in zip(arrs, offs)]

    def upload_batch(self, progs: np.ndarray, views: List[DeviceView]):
        tp = self._h2d(progs.view(np.uint8))
        tv = self._views_tensor(views)
        return tp, tv

    def prepare_count(self, exprs: Sequence[object], sort: bool = True):
        """Host half of a count batch: compile, order, split by kernel flavour
        and upload the programs.  Returns a handle for :meth:`launch_count`.

        Queries are reordered by their leaf rows so that consecutive work items
        (same shard, neighbouring queries) touch the same hot containers and
        hit in the XCD's L2; results are scattered back to submission order."""
        progs, views, S = self.compile_batch(exprs)
        return self.prepare_progs(progs, views, S, sort)

    def prepare_progs(self, progs: np.ndarray, views: List["DeviceView"], S: int, sort: bool = True):
        """:meth:`prepare_count` for already compiled QPROG_DTYPE records
        (e.g. from the native PQL compiler, pilosa_amd/native/pql_compile.cpp)."""
        torch = self.torch
        Q = len(progs)
        if not S or not Q:
            return (Q, S, None, [])
        progs = _canonical_and2(progs)
        np_ = progs["nprog"]
        pg = progs["prog"]
        lr = progs["leaf_row"]
        is_row = np_ == 1
        is_and2 = (np_ == 3) & (pg[:, 0] == 0) & (pg[:, 1] == 1) & (pg[:, 2] == OP_AND)
        if not self.use_and2 or max(v.container_count for v in views) >= 0xFFFFFFFF:
            is_row = is_row | is_and2
            is_and2 = np.zeros_like(is_and2)
        flat = flat_mask(progs)
        kind = np.where(is_and2, KIND_AND2, np.where(is_row, KIND_ROW,
                                                      np.where(flat, KIND_FLAT, KIND_GENERIC)))
        # flat folds whose every operator is OR: union count kernel
        pos = np.arange(pg.shape[1])
        is_op = (pos[None, :] % 2 == 0) & (pos[None, :] > 0) & (pos[None, :] < np_[:, None])
        all_or = np.where(is_op, pg == OP_OR, True).all(axis=1)
        if self.use_union:
            kind = np.where((kind == KIND_FLAT) & all_or, KIND_UNION, kind)
        if is_and2.any():
            progs = self._hot_leaf_first(progs, is_and2)
            lr = progs["leaf_row"]
            for v in views:
                v.ensure_keymask()
        shd = bool(is_and2.any()) and self.use_shadow and any([v.ensure_shadow() for v in views])
        varr = np.zeros(len(views), dtype=VIEWDEV_DTYPE)
        for i, v in enumerate(views):
            varr[i] = v.viewdev()
        host = [varr.view(np.uint8)]
        meta = []
        for k in (KIND_AND2, KIND_ROW, KIND_FLAT, KIND_UNION, KIND_GENERIC):
            sel = np.nonzero(kind == k)[0]
            if len(sel) == 0:
                continue
            if sort and len(sel) > 1:
                sel = sel[np.lexsort((lr[sel, 1], lr[sel, 0]))]
            host.append(np.ascontiguousarray(progs[sel]).view(np.uint8))
            host.append(sel.astype(np.int64))
            meta.append((k, len(sel)))
        dev = self._h2d_many(host)
        tv = dev[0]
        parts = [(dev[1 + 2 * i], dev[2 + 2 * i].view(torch.int64), k, n) for i, (k, n) in enumerate(meta)]
        return (Q, S, tv, parts, shd)

    def prepare_planned(self, Q: int, segs, buf: np.ndarray, views: List["DeviceView"], S: int):
        """:meth:`prepare_progs` for a batch planned natively
        (native/pql_compile.cpp plan_count_text): one pinned H2D copy of the
        view table and the planner's buffer (routes' programs + submission
        indices), no host-side numpy work."""
        torch = self.torch
        if not S or not Q:
            return (Q, S, None, [])
        shd = False
        if any(int(kind) == KIND_AND2 for kind, _, _, _ in segs):
            for v in views:
                v.ensure_keymask()
            shd = self.use_shadow and any([v.ensure_shadow() for v in views])
        varr = np.zeros(len(views), dtype=VIEWDEV_DTYPE)
        for i, v in enumerate(views):
            varr[i] = v.viewdev()
        tv, tb = self._h2d_many([varr.view(np.uint8), buf])
        parts = []
        for kind, n, po, oo in segs:
            if int(kind) == KIND_ALIAS:
                parts.append((tb[po:po + n * 8].view(torch.int64), tb[oo:oo + n * 8].view(torch.int64), KIND_ALIAS,
                              int(n)))
                continue
            parts.append((tb[po:po + n * QPROG_DTYPE.itemsize], tb[oo:oo + n * 8].view(torch.int64), int(kind), int(n)))
        return (Q, S, tv, parts, shd)

    @staticmethod
    def _hot_leaf_first(progs: np.ndarray, sel: np.ndarray) -> np.ndarray:
        """For Count(Intersect(a, b)) put the row used most often in the batch
        in leaf 0: the pair kernel stages leaf 0 once per run of equal rows."""
        lr = progs["leaf_row"]
        lv = progs["leaf_view"]
        idx = np.nonzero(sel)[0]
        keys = np.concatenate([lv[idx, 0].astype(np.int64) << 40 | lr[idx, 0], lv[idx, 1].astype(np.int64) << 40 | lr[idx, 1]])
        uniq, inv, cnt = np.unique(keys, return_inverse=True, return_counts=True)
        ca, cb = cnt[inv[:len(idx)]], cnt[inv[len(idx):]]
        swap = idx[(cb > ca) | ((cb == ca) & (keys[len(idx):] < keys[:len(idx)]))]
        if len(swap):
            progs = progs.copy()
            for f in ("leaf_row", "leaf_view"):
                col = progs[f]
                col[swap, 0], col[swap, 1] = col[swap, 1].copy(), col[swap, 0].copy()
        return progs

    def _and2_partial(self, tp, tv, S: int, n: int, shd: bool = False):
        """Per-(shard, key, query) Count(Intersect) partials -> int32[S, 16, n].
        ``shd``: a view of the batch carries dense shadows (variant 41; the
        launcher takes 42 for serving-size batches)."""
        torch = self.torch
        pairs = torch.empty(S * 16 * n * 2, dtype=torch.int32, device=self.device)
        partial = torch.empty(S * 16 * n, dtype=torch.int32, device=self.device)
        variant = 41 if shd and self.and2_variant == 6 else self.and2_variant
        self.ext.and2_count(tp, tv, S, pairs, partial, self.and2_cq, variant)
        return partial.view(S, 16, n)

    def to_host(self, t):
        with tracing.span("GpuEngine.d2h", gpu=True):
            return self._to_host(t)

    def _to_host(self, t):
        """Device tensor -> host tensor through a pinned buffer and an event
        wait.  A plain ``.cpu()`` is a synchronous pageable D2H copy: the HIP
        runtime stages it with blit kernels and holds the stream while it
        waits, so other request threads cannot enqueue their next batch and
        the GPU idles between batches (profiles/r03_clients)."""
        torch = self.torch
        if t.device.type != "cuda":
            return t
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        if _D2H_POLL:
            # poll instead of a blocking wait: other request threads keep
            # launching while this one waits for its batch
            while not ev.query():
                time.sleep(_D2H_POLL)
        else:
            ev.synchronize()
        return h

    def launch_count(self, handle):
        """Device half: launch the kernels; returns the device int64[Q] result."""
        with tracing.span("GpuEngine.launchCount", gpu=True, queries=handle[0], shards=handle[1]):
            return self._launch_count(handle)

    def _launch_count(self, handle):
        torch = self.torch
        Q, S, tv, parts = handle[:4]
        shd = len(handle) > 4 and handle[4]
        out = torch.zeros(Q, dtype=torch.int64, device=self.device)
        for tp, ti, kind, n in parts:
            if kind == KIND_ALIAS:   # repeated calls: their answers copied (the last part)
                out.index_copy_(0, ti, out.index_select(0, tp))
                continue
            if kind == KIND_AND2:
                # column sums scattered into out by one kernel (a strided torch
                # reduce + index_copy cost ~70 us per small serving batch)
                self.ext.partial_sum_scatter(self._and2_partial(tp, tv, S, n, shd).view(-1), S * 16, n, ti, out)
                continue
            else:
                o = torch.zeros(n, dtype=torch.int64, device=self.device)
                mode = _KERNEL_MODE[kind]
                if kind == KIND_UNION and self.union_variant == 2:
                    mode = 4  # union_count2_kernel
                self.ext.expr_count(tp, tv, S, o, None, mode)
            out.index_copy_(0, ti, o)
        return out

    def count_per_shard(self, exprs: Sequence[object]) -> np.ndarray:
        """Counts per (query, local shard) -> int64[Q, S] (TopN per-shard semantics)."""
        progs, views, S = self.compile_batch(exprs)
        return self.count_per_shard_progs(progs, views, S)

    @staticmethod
    def pair_programs(slot_a: int, dense_a: np.ndarray, slot_b: int, dense_b: np.ndarray) -> np.ndarray:
        """Count(Intersect(Row a, Row b)) QueryProg records built directly
        (vectorised; no expression objects) for dense row indices."""
        dense_a = np.broadcast_to(np.asarray(dense_a, np.int64), np.shape(dense_b)) if np.ndim(dense_a) == 0 \
            else np.asarray(dense_a, np.int64)
        dense_b = np.asarray(dense_b, np.int64)
        Q = len(dense_b)
        p = np.zeros(Q, dtype=QPROG_DTYPE)
        p["nleaf"] = 2
        p["nprog"] = 3
        p["leaf_view"][:, 0] = slot_a
        p["leaf_view"][:, 1] = slot_b
        p["leaf_row"][:, 0] = dense_a
        p["leaf_row"][:, 1] = dense_b
        p["prog"][:, 0] = 0
        p["prog"][:, 1] = 1
        p["prog"][:, 2] = OP_AND
        return p

    @staticmethod
    def union_programs(dense: np.ndarray) -> np.ndarray:
        """Count(Union(Row r of view 0, Row r of view 1, ...)) records built
        directly (vectorised) from ``dense[Q, V]`` = the dense index of each
        query's row in each of the V batch views (slots 0..V-1), e.g. the
        covering views of a time-range Row.  Flat OR fold, as compile_expr
        emits it: l0 l1 | l2 | ..."""
        dense = np.asarray(dense, np.int64)
        Q, V = dense.shape
        if not 1 <= V <= MAXLEAF:
            raise CompileError("too many leaves")
        p = np.zeros(Q, dtype=QPROG_DTYPE)
        p["nleaf"] = V
        p["nprog"] = 2 * V - 1
        p["leaf_view"][:, :V] = np.arange(V)
        p["leaf_row"][:, :V] = dense
        prog = [0] + [x for k in range(1, V) for x in (k, OP_OR)]
        p["prog"][:, :len(prog)] = prog
        return p

    def count_per_shard_progs(self, progs: np.ndarray, views: List["DeviceView"], S: int,
                              as_tensor: bool = False):
        """:meth:`count_per_shard` for compiled records.  Count(Intersect)
        batches take the pair kernels, ordered by leaf rows for reuse."""
        torch = self.torch
        Q = len(progs)
        if not S or not Q:
            z = np.zeros((Q, S), dtype=np.int64)
            return torch.from_numpy(z) if as_tensor else z
        progs = _canonical_and2(progs)
        np_, pg = progs["nprog"], progs["prog"]
        varr = np.zeros(len(views), dtype=VIEWDEV_DTYPE)
        for i, v in enumerate(views):
            varr[i] = v.viewdev()
        if self.use_and2 and max(v.container_count for v in views) < 0xFFFFFFFF and \
                bool(np.all((np_ == 3) & (pg[:, 0] == 0) & (pg[:, 1] == 1) & (pg[:, 2] == OP_AND))):
            progs = self._hot_leaf_first(progs, np.ones(Q, bool))
            lr = progs["leaf_row"]
            order = np.lexsort((lr[:, 1], lr[:, 0]))
            tv, tp, to = self._h2d_many([varr.view(np.uint8), np.ascontiguousarray(progs[order]).view(np.uint8),
                                         order.astype(np.int64)])
            part = self._and2_partial(tp, tv, S, Q).sum(dim=1, dtype=torch.int64)  # [S, Q] in sorted order
            out = torch.empty((Q, S), dtype=torch.int64, device=self.device)
            out.index_copy_(0, to.view(torch.int64), part.t())
            return out if as_tensor else out.cpu().numpy()
        tv, tp = self._h2d_many([varr.view(np.uint8), progs.view(np.uint8)])
        ps = torch.zeros(Q * S, dtype=torch.int64, device=self.device)
        empty = torch.empty(0, dtype=torch.int64, device=self.device)
        self.ext.expr_count(tp, tv, S, empty, None, 2 if bool(flat_mask(progs).all()) else 0, ps)
        ps = ps.view(Q, S)
        return ps if as_tensor else ps.cpu().numpy()

    def count_async(self, exprs: Sequence[object]):
        """Launch counts for a batch; returns the device int64[Q] result tensor.

        Count(Row) / Count(Intersect(a,b)) programs go to the low-register fast
        kernel, everything else to the generic tile interpreter."""
        return self.launch_count(self.prepare_count(exprs))

    def count(self, exprs: Sequence[object]) -> np.ndarray:
        return self.count_async(exprs).cpu().numpy()

    def _materialize(self, progs: np.ndarray, views: List["DeviceView"], S: int):
        torch = self.torch
        Q = len(progs)
        tp, tv = self.upload_batch(progs, views)
        counts = torch.zeros(Q * S * 16, dtype=torch.int32, device=self.device)
        self.ext.expr_count(tp, tv, S, torch.empty(0, dtype=torch.int64, device=self.device), counts,
                            2 if bool(flat_mask(progs).all()) else 0)
        sizes = torch.where(counts > 4096, torch.full_like(counts, 4096), (counts + 7) // 8 * 8).to(torch.int64)
        sizes = torch.where(counts > 0, sizes, torch.zeros_like(sizes))
        offs = torch.cumsum(sizes, 0) - sizes
        total = int(sizes.sum().item())
        outp = torch.zeros(max(total, 8), dtype=torch.int16, device=self.device)
        if total:
            self.ext.expr_materialize(tp, tv, S, counts, offs, outp)
        return counts, offs, outp

    def materialize_batch(self, exprs: Sequence[object], S: int):
        """Device result containers of a batch of expressions over S local
        shards: (counts int32[Q*S*16], u16 offsets int64[Q*S*16], payload
        int16[]); container (q, s, j) is an array when 0 < n <= 4096, else a
        bitmap of 4096 u16."""
        progs, views, S2 = self.compile_batch(exprs)
        if S2 != S:
            raise CompileError(f"expressions span {S2} shards, expected {S}")
        return self._materialize(progs, views, S)

    def materialize_block(self, expr) -> Optional["DeviceRowBlock"]:
        """Evaluate one expression into device result containers, left in HBM
        (a rank's Row partial travels as these blocks, parallel/mesh.py)."""
        progs, views, S = self.compile_batch([expr])
        if not S:
            return None
        counts, offs, outp = self._materialize(progs, views, S)
        return DeviceRowBlock([int(x) for x in views[0].shards], counts, offs, outp)

    @staticmethod
    def block_bitmaps(shards: Sequence[int], c: np.ndarray, o: np.ndarray, pay: np.ndarray) -> List[object]:
        """Host Bitmaps of result containers (counts ``c``, u16 offsets ``o``
        per (shard, key), u16 payload ``pay``), one per shard (None = empty)."""
        from pilosa_amd import _roaring
        from pilosa_amd import shardwidth
        cpr = shardwidth.ARENA_CPR   # device shard ids: global key = shard * cpr + slot
        result = []
        for s in range(len(shards)):
            cs = c[s * 16:(s + 1) * 16]
            nz = np.nonzero(cs)[0]
            if len(nz) == 0:
                result.append(None)
                continue
            keys = (np.uint64(shards[s]) * np.uint64(cpr) + nz.astype(np.uint64)).astype(np.uint64)
            types = np.where(cs[nz] > 4096, 2, 1).astype(np.uint8)
            result.append(_roaring.bitmap_from_containers(keys, types, cs[nz].astype(np.int32),
                                                          o[s * 16 + nz].astype(np.int64), pay))
        return result

    def materialize(self, expr) -> Tuple[List[object], List[int]]:
        """Evaluate one expression to per-shard host Bitmaps (row results)."""
        blk = self.materialize_block(expr)
        if blk is None:
            return [], []
        c, o, pay = blk.host()
        return self.block_bitmaps(blk.shards, c, o, pay), blk.shards

    @staticmethod
    def bsi_args(bsi_view: "DeviceView", depth: int, slot: int = 0) -> np.ndarray:
        """cpu int64[67]: view slot, depth, dense rows of exists / sign / bit i
        (memoised per view generation)."""
        key = (bsi_view.generation, depth, slot)
        memo = bsi_view.__dict__.setdefault("_bsi_args", {}) if hasattr(bsi_view, "__dict__") else {}
        hit = memo.get(key)
        if hit is not None:
            return hit.copy()
        args = np.full(67, -1, dtype=np.int64)
        args[0] = slot
        args[1] = depth
        args[2] = bsi_view.dense(0)
        args[3] = bsi_view.dense(1)
        for i in range(min(depth, 63)):
            args[4 + i] = bsi_view.dense(2 + i)
        memo.clear()
        memo[key] = args.copy()
        return args

    BSI_OPS = {"==": 0, "!=": 1, "<": 2, "<=": 3, ">": 4, ">=": 5, "between": 6, "notnull": 7}

    def bsi_range_view(self, bsi_view: "DeviceView", depth: int, op: str, p1: int = 0, p2: int = 0) -> "DeviceView":
        """Evaluate a BSI predicate (base-relative values) over every local
        shard into a temporary one-row device view: row 0 = matching columns,
        one bitmap container per (shard, key)."""
        torch = self.torch
        S = bsi_view.S
        payload = torch.empty(S * 16 * 4096, dtype=torch.int16, device=self.device)
        meta = torch.empty(S * 16, dtype=torch.int64, device=self.device)
        args = self.bsi_args(bsi_view, depth)
        if S and args[2] >= 0:
            tv = self._views_tensor([bsi_view])
            self.ext.bsi_range(tv, S, torch.from_numpy(args), self.BSI_OPS[op], int(p1), int(p2), payload, meta)
        else:
            payload.zero_()
            meta.copy_(torch.arange(S * 16, dtype=torch.int64, device=self.device) % 16 | (2 << 4)
                       | ((torch.arange(S * 16, dtype=torch.int64, device=self.device) * 512) << 23))
        rowptr = torch.tensor([0, 16], dtype=torch.int32, device=self.device).repeat(max(S, 0))
        sb = torch.arange(S + 1, dtype=torch.int64, device=self.device) * 16
        return DeviceView.from_device(np.zeros(1, np.uint64), rowptr, sb, meta, payload, self.device,
                                      bsi_view.shards, S * 16)

    def _one_row_view(self, payload, meta, shards) -> "DeviceView":
        """Wrap dense device results (one bitmap per (shard, key)) as a
        one-row view (row id 0) usable as an expression leaf."""
        torch = self.torch
        S = len(shards)
        rowptr = torch.tensor([0, 16], dtype=torch.int32, device=self.device).repeat(max(S, 0))
        sb = torch.arange(S + 1, dtype=torch.int64, device=self.device) * 16
        return DeviceView.from_device(np.zeros(1, np.uint64), rowptr, sb, meta, payload, self.device, shards, S * 16)

    def dense_view(self, expr) -> "DeviceView":
        """Evaluate one expression over every local shard into a dense one-row
        view (expr_dense_kernel)."""
        torch = self.torch
        progs, views, S = self.compile_batch([expr])
        payload = torch.empty(S * 16 * 4096, dtype=torch.int16, device=self.device)
        meta = torch.empty(S * 16, dtype=torch.int64, device=self.device)
        if S:
            tp, tv = self.upload_batch(progs, views)
            self.ext.expr_dense(tp, tv, S, payload, meta)
        return self._one_row_view(payload, meta, views[0].shards if views else [])

    def shift_views(self, expr, n: int) -> Tuple["DeviceView", "DeviceView"]:
        """Shift(expr, n) for 0 < n < ShardWidth (row_kernels.hip): the part
        that stays in each shard, and the spill each shard carries into the
        next shard's segment (row.go:217-239, roaring.go:944-977).  Above
        2^20 columns a shard's device sub-shards carry into each other and
        the spill of sub-shard m lands in sub-shard m of the next shard;
        below, a 2^e-column shard's bits carried past 2^e columns (not past
        its 2^20-column device shard) are its spill."""
        torch = self.torch
        src = self.dense_view(expr)
        S = src.S
        outs = [torch.empty(S * 16 * 4096, dtype=torch.int16, device=self.device) for _ in range(2)]
        metas = [torch.empty(S * 16, dtype=torch.int64, device=self.device) for _ in range(2)]
        if S:
            from pilosa_amd import shardwidth
            # a shard wider than 2^20 columns is M consecutive device sub-shards:
            # carries cross them inside the shard (row_kernels.hip)
            self.ext.shift_dense(src.t_payload, S, int(n), outs[0], metas[0], outs[1], metas[1],
                                 shardwidth.DEVICE_SUBSHARDS, shardwidth.SHARD_WIDTH // 64)
        return (self._one_row_view(outs[0], metas[0], src.shards),
                self._one_row_view(outs[1], metas[1], src.shards))

    def row_ids(self, view: "DeviceView", column: Optional[int] = None) -> np.ndarray:
        """Sorted row ids with a non-empty container on this GPU (with
        ``column``: rows holding that column's bit), rows_kernel."""
        torch = self.torch
        if view.D == 0 or view.S == 0:
            return np.zeros(0, np.uint64)
        flags = torch.zeros(view.D, dtype=torch.uint8, device=self.device)
        vd = torch.from_numpy(np.frombuffer(view.viewdev().tobytes(), dtype=np.uint8).copy())
        if column is None:
            self.ext.rows_list(vd, 0, view.S, -1, 0, flags)
        else:
            from pilosa_amd import shardwidth
            shard, off = divmod(int(column), shardwidth.ARENA_WIDTH)   # device shard
            if shard not in view.shards:
                return np.zeros(0, np.uint64)
            si = view.shards.index(shard)
            self.ext.rows_list(vd, si, 1, off >> 16, off & 0xffff, flags)
        idx = torch.nonzero(flags).reshape(-1).cpu().numpy()
        return view.rows[idx]  # the directory is sorted

    def bsi_range_count_async(self, bsi_view: "DeviceView", depth: int, op: str, p1: int = 0, p2: int = 0):
        """Count(Row(v <op> x)) without materialising the predicate view:
        device int64[1]."""
        torch = self.torch
        out = torch.zeros(1, dtype=torch.int64, device=self.device)
        args = self.bsi_args(bsi_view, depth)
        if bsi_view.S and args[2] >= 0:
            self.ext.bsi_range_count(self._views_tensor([bsi_view]), bsi_view.S, torch.from_numpy(args),
                                     self.BSI_OPS[op], int(p1), int(p2), out)
        return out

    def bsi_minmax(self, filt: Optional[object], bsi_view: "DeviceView", depth: int, which: str = "") -> np.ndarray:
        """Per (shard, key) descents -> int64[S, 16, 10] (see bsi_minmax_kernel);
        ``which`` "min" / "max" runs only that call's two descents (the other
        columns stay 0), "" all four."""
        return self.to_host(self._bsi_minmax_dev(filt, bsi_view, depth, which)).numpy().reshape(bsi_view.S, 16, 10)

    def bsi_minmax_folded(self, filt: Optional[object], bsi_view: "DeviceView", depth: int, which: str,
                          sub: int = 1) -> Tuple[int, int, bool]:
        """Min / Max of the call folded on the device (bsi_minmax_fold_kernel):
        (value, count, found) with fragments of ``sub`` arena sub-shards."""
        torch = self.torch
        o = self._bsi_minmax_dev(filt, bsi_view, depth, which)
        out = torch.zeros(3, dtype=torch.int64, device=self.device)
        S = bsi_view.S
        if S:
            self.ext.bsi_minmax_fold(o, S // sub, 16 * sub, 1 if which == "min" else 0, out)
        v, c, found = self.to_host(out).tolist()
        return int(v), int(c), bool(found)

    def _bsi_minmax_dev(self, filt: Optional[object], bsi_view: "DeviceView", depth: int, which: str = ""):
        torch = self.torch
        S = bsi_view.S
        view_index: Dict[int, int] = {id(bsi_view): 0}
        views = {id(bsi_view): bsi_view}
        if filt is not None:
            def collect(node):
                if isinstance(node, Leaf):
                    views[id(node.view)] = node.view
                elif isinstance(node, Op):
                    for a in node.args:
                        collect(a)
            collect(filt)
            progs = pack_programs([compile_expr(filt, view_index)])
        else:
            progs = pack_programs([([], [], [])])
        ordered = [None] * len(view_index)
        for vid, slot in view_index.items():
            ordered[slot] = views[vid]
        out = torch.zeros(S * 16 * 10, dtype=torch.int64, device=self.device)
        args = self.bsi_args(bsi_view, depth)
        if S and args[2] >= 0:
            tp, tv = self.upload_batch(progs, ordered)
            self.ext.bsi_minmax(tp, tv, S, torch.from_numpy(args), out, {"min": 1, "max": 2}.get(which, 0))
        return out

    def bsi_sum_async(self, filters: Sequence[Optional[object]], bsi_view: "DeviceView", depth: int,
                      matrix: Optional[bool] = None):
        """Sum/count of a BSI field for a batch of filters (None = no filter).
        Batches of BSI_MATRIX_MIN+ filters run as one bit-plane count matrix
        on the matrix cores (ops/bsi.py); ``matrix`` forces either path."""
        torch = self.torch
        if len(filters) == 1 and filters[0] is None:
            # Sum(field=v): no program to compile or upload (a constant one)
            args = self.bsi_args(bsi_view, depth)
            outs = torch.zeros(2, dtype=torch.int64, device=self.device)
            if bsi_view.S and args[2] >= 0:
                tp = self.__dict__.get("_empty_prog")
                if tp is None:   # a synchronous copy: any stream may read it afterwards
                    tp = self._empty_prog = torch.from_numpy(
                        pack_programs([([], [], [])]).view(np.uint8).copy()).to(self.device)
                    if self.device.type == "cuda":
                        torch.cuda.current_stream(self.device).synchronize()
                self.ext.bsi_sum(tp, self._views_tensor([bsi_view]), bsi_view.S, torch.from_numpy(args),
                                 outs[:1], outs[1:], 0)
            return outs[:1], outs[1:]
        if matrix is None:
            from .bsi import BSI_MATRIX_MIN
            matrix = len(filters) >= BSI_MATRIX_MIN
        if matrix:
            from .bsi import bsi_sum_matrix
            try:
                return bsi_sum_matrix(self, filters, bsi_view, depth)
            except CompileError:
                pass  # a filter the dense evaluator cannot take: per-filter kernel
        exprs = [f for f in filters if f is not None]
        view_index: Dict[int, int] = {id(bsi_view): 0}
        views = {id(bsi_view): bsi_view}

        def collect(node):
            if isinstance(node, Leaf):
                views[id(node.view)] = node.view
            elif isinstance(node, Op):
                for a in node.args:
                    collect(a)

        compiled = []
        for f in filters:
            if f is None:
                compiled.append(([], [], []))
                continue
            collect(f)
            compiled.append(compile_expr(f, view_index))
        progs = pack_programs(compiled)
        ordered = [None] * len(view_index)
        for vid, slot in view_index.items():
            ordered[slot] = views[vid]
        args = self.bsi_args(bsi_view, depth)
        outs = torch.zeros(2 * len(filters), dtype=torch.int64, device=self.device)
        out_sum, out_cnt = outs[:len(filters)], outs[len(filters):]
        if bsi_view.S and args[2] >= 0:
            tp, tv = self.upload_batch(progs, ordered)
            # filter flavour: none / flat folds (2 tiles) / any program (tile stack)
            nprog = progs["nprog"]
            if not (nprog > 0).any():
                fmode = 0
            elif bool(((nprog <= 1) | flat_mask(progs)).all()):
                fmode = 1
            else:
                fmode = 2
            self.ext.bsi_sum(tp, tv, bsi_view.S, torch.from_numpy(args), out_sum, out_cnt, fmode)
        return out_sum, out_cnt
