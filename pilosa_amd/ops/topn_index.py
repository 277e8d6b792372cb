"""Src-filtered TopN over an HBM-resident column-major slot index.

Reference: fragment.go:1568-1700 (``top``: rank-cache walk with a src row,
heap threshold, ids= re-count) and executor.go:863-930 (two phases, Pairs.Add
over shards, trim to n).

The pair-per-candidate formulation (ops/topn.py ``topn_phase1``) counts
|src ∩ row| for every cached row the walk may reach: ~10k row intersections
per (query, shard) on the Zipf headline index.  :class:`DeviceTopNIndex`
keeps, next to a view's arena, the cache slot of every set bit of every
cached row grouped by column (per shard: ``colptr[2^20+1]`` + u16 slots).
The src counts of all cached rows of a shard are then one LDS histogram over
src's columns, and the reference heap walk runs on that histogram inside the
same workgroup (pilosa_amd/kernels/topn_kernels.hip).  Phase 1 leaves one
accumulator per query over the node-wide "acc space" of row ids; across the
GPUs of a node only its non-zero entries (the candidate set) are all-gathered
and unioned, and phase 2 (the ids= re-count, the kernel with a gather instead
of the walk) sums one int64 per candidate with an all-reduce.
"""
from __future__ import annotations

import os
import threading
from contextlib import contextmanager
from typing import List, Optional, Sequence

import numpy as np

from pilosa_amd.models.cache import Pair, pair_array, pairs_from_arrays

from .device import DeviceView, GpuEngine, kernels

SHARD_WIDTH = 1 << 20   # device shard width: columns of one arena shard (16 container slots per row)
LDS_LIMIT = 160 * 1024 - 1024
# cache ranks counted row-major for the whole batch (topn_hot_kernel); the
# slot index / histogram cover the ranks after them.  Bench src mix, 16-query
# batch on the 954-shard headline index (profiles/r03_hotpart): 2048 -> hot
# 9.05 + tail histogram 3.17 ms; 4096 -> 10.03 + 1.40 ms (13.0 vs 13.9 ms per
# batch end to end); 8192 -> hot 12.7 ms, worse.  Round 4 (current kernels,
# through the executor, profiles/r04_p/): 2048 / 2560 / 3072 / 3584 / 4096 /
# 6144 -> 1,194 / 1,223 / 1,264-1,278 / 1,261 / 1,196 / 1,203 src q/s.
HOT_RANKS = int(os.environ.get("PILOSA_TOPN_HOT", "3072"))
# queries per hot-rank launch: up to 16 take topn_hot_kernel<16> (u16 query
# masks of a whole key in LDS), 17..32 topn_hot_kernel<32> (u32 masks of half
# a key per workgroup: twice the queries for the same streamed bytes).  Both
# half-key workgroups still walk every value of a container (per-value work,
# not bytes, bounds this kernel: carry-save mask counting instead of the SWAR
# adds changed nothing, 9.44 vs 9.16 ms), so the 32-query launch measured
# 30.6 ms against 2 x 9.2 ms for two 16-query launches
# (profiles/r02_topn/topn_kbench_b32.log): 16 stays the default.
HOT_Q = int(os.environ.get("PILOSA_TOPN_HOT_Q", "16"))
MAX_SLOTS = 65535
# phase-1 histograms are kept for the ids= gather up to this many bytes per batch
HIST_KEEP_BYTES = 8 << 30


class _RWLock:
    """Readers (TopN batches using an index) share it; a writer (an in-place
    refresh after writes) waits for them and holds new ones back.  A
    thread's nested read (topn over several hot-rank launches) re-enters."""

    def __init__(self):
        self._c = threading.Condition()
        self._readers = 0
        self._writer = False
        self._waiting = 0
        self._local = threading.local()

    @contextmanager
    def read(self):
        depth = getattr(self._local, "d", 0)
        if depth == 0:
            with self._c:
                while self._writer or self._waiting:
                    self._c.wait()
                self._readers += 1
        self._local.d = depth + 1
        try:
            yield
        finally:
            self._local.d = depth
            if depth == 0:
                with self._c:
                    self._readers -= 1
                    if not self._readers:
                        self._c.notify_all()

    @contextmanager
    def write(self):
        with self._c:
            self._waiting += 1
            while self._writer or self._readers:
                self._c.wait()
            self._waiting -= 1
            self._writer = True
        try:
            yield
        finally:
            with self._c:
                self._writer = False
                self._c.notify_all()


def lds_bytes(K: int, H32: int, H16: int) -> int:
    """Slot histogram bytes: u32 counters below H32, u16 below H16, u8 above
    (topn_kernels.hip HistLayout)."""
    return (H32 + (H16 - H32 + 1) // 2 + (K - H16 + 3) // 4) * 4


class DeviceTopNIndex:
    """Slot index of a view's rank caches (``cache``: a DeviceRankCache whose
    rows are ordered count desc, id asc per shard).

    ``space`` is the sorted row-id space of the phase-1/phase-2 accumulators;
    pass the union of every rank's rows on a multi-GPU node (default: this
    view's rows)."""

    def __init__(self, view: DeviceView, cache, space: Optional[np.ndarray] = None, hot: Optional[int] = None):
        import torch

        ext = kernels()
        dev = view.device
        self.view = view
        self.generation = view.generation
        space = np.asarray(view.rows if space is None else space, dtype=np.uint64)
        self.space = space
        self.A = A = int(len(space))

        def t32(a):
            return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)

        if hasattr(cache, "cache_dense"):
            # device rank caches (ops/topn_exec.DeviceRankCaches): no host pass
            S, K = int(cache.cache_dense.shape[0]), int(cache.cache_dense.shape[1])
            if (S == 0 and view.S) or (S and view.S % S):
                raise ValueError("rank cache and view disagree on the shard count")
            self.cache_dense = cache.cache_dense.contiguous()
            self.cache_cnt = cache.cache_cnt.contiguous()
            valid_t = self.cache_dense >= 0
            if A == view.D and (A == 0 or np.array_equal(space, view.rows)):
                acc_t = self.cache_dense.clamp(min=0)
                self.a2dense = torch.arange(A, dtype=torch.int32, device=dev)
            else:
                from .topn_exec import dense_dev, rows_dev
                sp = torch.from_numpy(space.view(np.int64)).to(dev)
                rid = rows_dev(view)[self.cache_dense.clamp(min=0).long()]
                acc_t = torch.searchsorted(sp, rid).clamp_(max=max(A - 1, 0))
                if bool((valid_t & (sp[acc_t] != rid)).any().item()):
                    raise ValueError("acc space misses cached rows")
                self.a2dense = dense_dev(view, sp).contiguous()
            self.cache_acc = torch.where(valid_t, acc_t, torch.zeros_like(acc_t)).to(torch.int32).contiguous()
            cnt_for_tiers = None
        else:
            S, K = cache.rows.shape
            if (S == 0 and view.S) or (S and view.S % S):
                raise ValueError("rank cache and view disagree on the shard count")
            counts = np.asarray(cache.counts, dtype=np.int64)
            valid = counts > 0
            rows = np.asarray(cache.rows, dtype=np.uint64).reshape(-1)
            dense = view.dense_many(rows).reshape(S, K)
            dense = np.where(valid, dense, -1)
            acc_i = np.searchsorted(space, rows).reshape(S, K)
            acc_i = np.minimum(acc_i, max(A - 1, 0))
            if valid.any() and not np.array_equal(space[acc_i[valid]], rows.reshape(S, K)[valid]):
                raise ValueError("acc space misses cached rows")
            acc_i = np.where(valid, acc_i, 0)
            self.cache_dense = t32(dense)
            self.cache_acc = t32(acc_i)
            self.cache_cnt = t32(np.where(valid, np.minimum(counts, 2 ** 31 - 1), 0))
            self.a2dense = t32(view.dense_many(space) if A else np.zeros(0))
            cnt_for_tiers = counts
        if K > MAX_SLOTS:
            raise ValueError(f"rank cache of {K} slots exceeds the u16 slot index ({MAX_SLOTS})")
        self.S, self.K = S, K
        # fragments wider than 2^20 columns: M arena sub-shards each.  The
        # slot index, hot-rank metadata and materialised srcs are per
        # sub-shard (Sd of them); caches, histograms and walks per fragment
        self.M = M = view.S // S if S else 1
        self.Sd = Sd = view.S
        dense_sub = self.cache_dense if M == 1 else self.cache_dense.repeat_interleave(M, dim=0).contiguous()
        # ranks [0, R): hot, counted row-major per batch; [R, K): slot index
        self.R = R = max(0, min(K, HOT_RANKS if hot is None else int(hot)))
        Kt = K - R
        # counter tiers from the cached counts (a src count never exceeds them)
        if S and Kt:
            if cnt_for_tiers is None:
                tail = self.cache_cnt[:, R:]
                n32 = int((tail >= 65536).sum(dim=1).max().item())
                n16 = int((tail >= 256).sum(dim=1).max().item())
            else:
                tail = cnt_for_tiers[:, R:]
                n32 = int((tail >= 65536).sum(axis=1).max())
                n16 = int((tail >= 256).sum(axis=1).max())
        else:
            n32 = n16 = 0
        self.H32 = min(Kt, (n32 + 63) // 64 * 64)
        self.H16 = max(self.H32, min(Kt, (n16 + 63) // 64 * 64))
        self.lds = lds_bytes(Kt, self.H32, self.H16)
        self.ok = self.lds <= LDS_LIMIT
        self._vd = torch.from_numpy(np.frombuffer(view.viewdev().tobytes(), dtype=np.uint8).copy())

        def empty(dt):
            return torch.empty(0, dtype=dt, device=dev)

        self.hot_meta = torch.full((Sd * 16 * R,), -1, dtype=torch.int32, device=dev)
        # per (sub-shard, key): [0] ranks before it are cooperative or mid-size, [1] cooperative
        self.hot_split = torch.zeros(Sd * 16 * 2, dtype=torch.int32, device=dev)
        if Sd and R:
            ext.topn_hot_meta(self._vd, Sd, K, R, dense_sub, self.hot_meta, self.hot_split)
        colcnt = torch.zeros(Sd * SHARD_WIDTH, dtype=torch.int32, device=dev)
        if Sd and Kt:
            ext.topn_index(self._vd, Sd, K, R, dense_sub, colcnt, empty(torch.int32), empty(torch.int64),
                           empty(torch.int16), False)
        self.colptr = torch.zeros((Sd, SHARD_WIDTH + 1), dtype=torch.int32, device=dev)
        if Sd:
            self.colptr[:, 1:] = torch.cumsum(colcnt.view(Sd, SHARD_WIDTH), dim=1, dtype=torch.int32)
        tot = self.colptr[:, SHARD_WIDTH].to(torch.int64)
        # each shard's slot region has 1/8 spare room, so a shard whose
        # cached rows change can be re-indexed in place (refresh)
        self.cap = tot + tot // 8 + 64
        self.entbase = torch.zeros(max(Sd, 1), dtype=torch.int64, device=dev)
        if Sd > 1:
            self.entbase[1:Sd] = torch.cumsum(self.cap, 0)[:-1]
        self.entries = int(self.cap.sum().item()) if Sd else 0
        # +16 entries: the histogram reads each slot run as aligned 16-byte words
        self.slots = torch.zeros((self.entries + 16 + 7) // 8 * 8, dtype=torch.int16, device=dev)
        if Sd and Kt:
            colcnt.zero_()
            ext.topn_index(self._vd, Sd, K, R, dense_sub, colcnt, self.colptr, self.entbase, self.slots, True)
        del colcnt, dense_sub
        self.slotmap = torch.full((S, max(A, 1)), -1, dtype=torch.int32, device=dev)
        si, ki = torch.nonzero(self.cache_dense >= 0, as_tuple=True)
        self.slotmap[si, self.cache_acc[si, ki].long()] = ki.to(torch.int32)
        if A == 0:
            self.slotmap = self.slotmap[:, :0].contiguous()
        # what this index reflects (refresh compares them with the view's)
        self.shard_gen = view.shard_gen.copy()
        self.rows_gen = view.rows_gen
        self.refreshes = 0
        self.refreshed_shards = 0
        self.rw = _RWLock()

    def refresh(self, view: DeviceView, cache, max_frac: float = 0.25) -> bool:
        """See :meth:`_refresh`; waits for the batches using this index."""
        with self.rw.write():
            return self._refresh(view, cache, max_frac)

    def _refresh(self, view: DeviceView, cache, max_frac: float = 0.25) -> bool:
        """Bring the index up to date in place after writes, re-indexing only
        the shards whose bits changed (the view's shard generations) or whose
        cached row order changed (``cache``: the rebuilt DeviceRankCaches):
        hot-rank metadata, column counts, slot region (within its spare room)
        and slot map of those shards, through the same kernels over a
        gathered sub-view.  False = the caller rebuilds the whole index (row
        directory changed, cache width changed, too many shards, a region
        overflowed)."""
        import torch

        if (view is not self.view or view.rows_gen != self.rows_gen or not hasattr(cache, "cache_dense")
                or tuple(cache.cache_dense.shape) != (self.S, self.K) or self.A != view.D
                or not (self.A == 0 or np.array_equal(self.space, view.rows))):
            return False
        S, K, R, M, Sd = self.S, self.K, self.R, self.M, self.Sd
        dev = view.device
        new_dense = cache.cache_dense.contiguous()
        # a fragment is re-indexed (all its M sub-shards) when any of its
        # sub-shards' bits or its cached row order changed
        changed = torch.from_numpy((view.shard_gen != self.shard_gen).reshape(S, M).any(axis=1)).to(dev)
        changed |= (new_dense != self.cache_dense).any(dim=1)
        C = torch.nonzero(changed).reshape(-1)
        nc = int(C.numel())
        if nc > max(1, int(S * max_frac)):
            return False
        ext = kernels()
        if nc:
            Cd = (C[:, None] * M + torch.arange(M, device=dev)[None, :]).reshape(-1) if M > 1 else C
            nd = nc * M
            D1 = view.D + 1
            sub = np.zeros((), dtype=view.viewdev().dtype)
            sub[()] = view.viewdev()
            rp_sub = view.t_rowptr.view(Sd, D1).index_select(0, Cd).contiguous()
            sb_sub = torch.cat([view.t_shard_base.index_select(0, Cd), view.t_shard_base[-1:]]).contiguous()
            sub["rowptr"] = rp_sub.data_ptr()
            sub["shard_base"] = sb_sub.data_ptr()
            sub["keymask"] = 0
            vd_sub = torch.from_numpy(np.frombuffer(sub.tobytes(), dtype=np.uint8).copy())
            cd_sub = new_dense.index_select(0, C)
            cd_sub = (cd_sub.repeat_interleave(M, dim=0) if M > 1 else cd_sub).contiguous()
            Kt = K - R
            colcnt = torch.zeros(nd * SHARD_WIDTH, dtype=torch.int32, device=dev)
            if Kt:
                ext.topn_index(vd_sub, nd, K, R, cd_sub, colcnt, torch.empty(0, dtype=torch.int32, device=dev),
                               torch.empty(0, dtype=torch.int64, device=dev),
                               torch.empty(0, dtype=torch.int16, device=dev), False)
            cp_sub = torch.zeros((nd, SHARD_WIDTH + 1), dtype=torch.int32, device=dev)
            cp_sub[:, 1:] = torch.cumsum(colcnt.view(nd, SHARD_WIDTH), dim=1, dtype=torch.int32)
            if bool((cp_sub[:, SHARD_WIDTH].to(torch.int64) > self.cap.index_select(0, Cd)).any().item()):
                return False
            eb_sub = self.entbase.index_select(0, Cd).contiguous()
            if Kt:
                colcnt.zero_()
                ext.topn_index(vd_sub, nd, K, R, cd_sub, colcnt, cp_sub, eb_sub, self.slots, True)
            del colcnt
            self.colptr.index_copy_(0, Cd, cp_sub)
            if R:
                hm_sub = torch.full((nd * 16 * R,), -1, dtype=torch.int32, device=dev)
                hs_sub = torch.zeros(nd * 16 * 2, dtype=torch.int32, device=dev)
                ext.topn_hot_meta(vd_sub, nd, K, R, cd_sub, hm_sub, hs_sub)
                self.hot_meta.view(Sd, 16 * R).index_copy_(0, Cd, hm_sub.view(nd, 16 * R))
                self.hot_split.view(Sd, 32).index_copy_(0, Cd, hs_sub.view(nd, 32))
        # the rank caches of every shard (counts of unchanged shards may move
        # too), their acc indexes, the slot map rows and the counter tiers
        self.cache_dense = new_dense
        self.cache_cnt = cache.cache_cnt.contiguous()
        valid_t = self.cache_dense >= 0
        acc_t = self.cache_dense.clamp(min=0)
        self.cache_acc = torch.where(valid_t, acc_t, torch.zeros_like(acc_t)).to(torch.int32).contiguous()
        if nc and self.A:
            self.slotmap.index_fill_(0, C, -1)
            si, ki = torch.nonzero(valid_t.index_select(0, C), as_tuple=True)
            self.slotmap[C[si], self.cache_acc[C[si], ki].long()] = ki.to(torch.int32)
        Kt = K - R
        if S and Kt:
            tail = self.cache_cnt[:, R:]
            n32 = int((tail >= 65536).sum(dim=1).max().item())
            n16 = int((tail >= 256).sum(dim=1).max().item())
        else:
            n32 = n16 = 0
        self.H32 = min(Kt, (n32 + 63) // 64 * 64)
        self.H16 = max(self.H32, min(Kt, (n16 + 63) // 64 * 64))
        self.lds = lds_bytes(Kt, self.H32, self.H16)
        self.ok = self.lds <= LDS_LIMIT
        self._vd = torch.from_numpy(np.frombuffer(view.viewdev().tobytes(), dtype=np.uint8).copy())
        self.generation = view.generation
        self.shard_gen = view.shard_gen.copy()
        self.refreshes += 1
        self.refreshed_shards += nc
        return self.ok

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.cache_dense, self.cache_acc, self.cache_cnt,
                                                          self.a2dense, self.colptr, self.entbase, self.slots,
                                                          self.slotmap, self.hot_meta))

    @property
    def stale(self) -> bool:
        return self.view.generation != self.generation

    # ------------------------------------------------------------ queries
    def _launch(self, mode: int, Q: int, src, ns_t, th_t, acc=None, pair_off=None, pair_idx=None, out=None,
                hist=None, hot_cnt=None, tail_built=None):
        import torch

        dev = self.view.device
        counts, offs, vals = src
        e32 = torch.empty(0, dtype=torch.int32, device=dev)
        e64 = torch.empty(0, dtype=torch.int64, device=dev)
        kernels().topn_src(self._vd, Q, self.S, self.K, self.H32, self.H16, self.A, counts, offs, vals, self.colptr,
                           self.entbase, self.slots, self.cache_cnt, self.cache_acc, self.slotmap, self.a2dense,
                           ns_t, th_t, mode, acc if acc is not None else e32,
                           pair_off if pair_off is not None else e64, pair_idx if pair_idx is not None else e32,
                           out if out is not None else e64, hist if hist is not None else e32,
                           self.R, self.hot_meta, hot_cnt if hot_cnt is not None else e32,
                           tail_built if tail_built is not None else e32, self.cache_dense, self.hot_split, self.M)

    def materialize(self, engine: GpuEngine, srcs: Sequence[object]):
        """Src containers of a batch: plain rows of this view are read in
        place from the arena (leaf_src, no copy); anything else (or a row
        with a run container) is materialised by the engine."""
        import torch

        from .device import Leaf

        Q = len(srcs)
        if Q and self.S and all(isinstance(x, Leaf) and x.view is self.view for x in srcs):
            dev = self.view.device
            dense = self.view.dense_many(np.array([x.row for x in srcs], dtype=np.uint64))
            rows = torch.from_numpy(np.asarray(dense, dtype=np.int64)).to(dev)
            counts = torch.zeros(Q * self.Sd * 16, dtype=torch.int32, device=dev)
            offs = torch.zeros(Q * self.Sd * 16, dtype=torch.int64, device=dev)
            has_run = torch.zeros(1, dtype=torch.int32, device=dev)
            kernels().leaf_src(self._vd, rows, self.Sd, counts, offs, has_run)
            # an arena without run containers cannot hand leaf_src one: no
            # host read of the flag (a sync between the src kernel and the
            # hot-rank launch, ~0.1 ms per batch)
            if not self._arena_has_runs() or not int(has_run.item()):
                return counts, offs, self.view.t_payload
        return engine.materialize_batch(srcs, self.Sd)

    def _arena_has_runs(self) -> bool:
        """Whether any container of the view's arena is a run container,
        checked once per view generation (writes bump it)."""
        v = self.view
        gen = getattr(v, "generation", None)
        got = self.__dict__.get("_runs_memo")
        if got is None or got[0] != gen or gen is None:
            got = (gen, bool((((v.t_meta >> 4) & 3) == 3).any().item()))
            self._runs_memo = got
        return got[1]

    def hot_counts(self, src, Q: int):
        """int32[S, Q, R]: src counts of the hot cache ranks (one row-major
        pass per HOT_Q queries, per arena sub-shard, summed per fragment),
        or None without hot ranks."""
        import torch

        if not self.R or not Q or not self.S:
            return None
        if Q > HOT_Q:
            raise ValueError(f"hot_counts: at most {HOT_Q} queries per call")
        dev = self.view.device
        hot = torch.zeros(self.Sd * Q * self.R, dtype=torch.int32, device=dev)
        z = torch.zeros(Q, dtype=torch.int32, device=dev)
        self._launch(4, Q, src, z, z, hot_cnt=hot)
        if self.M > 1:
            hot = hot.view(self.S, self.M, Q * self.R).sum(dim=1, dtype=torch.int32).reshape(-1).contiguous()
        return hot

    def hist_bytes(self, Q: int) -> int:
        return self.lds * Q * self.S

    def phase1(self, src, Q: int, ns: Sequence[int], thresholds: Sequence[int], keep_hist: bool = False,
               hot=None):
        """acc int32[Q, A]: per query the per-shard heap results summed by row.
        ``keep_hist`` also returns the (query, shard) slot histograms so the
        ids= re-count is a gather (else None).  ``hot``: hot_counts(src, Q)."""
        import torch

        dev = self.view.device
        ns_t = torch.tensor(list(ns), dtype=torch.int32).to(dev)
        th_t = torch.tensor(list(thresholds), dtype=torch.int32).to(dev)
        acc = torch.zeros((Q, self.A), dtype=torch.int32, device=dev)
        hist = torch.empty(self.hist_bytes(Q) // 4, dtype=torch.int32, device=dev) if keep_hist else None
        # which units built their tail histogram (phase 2 probes the others exactly)
        tb = torch.ones(Q * self.S, dtype=torch.int32, device=dev) if keep_hist else None
        if Q and self.S and self.A:
            self._launch(1, Q, src, ns_t, th_t, acc=acc, hist=hist, hot_cnt=hot, tail_built=tb)
        return acc, ns_t, th_t, (hist, tb) if keep_hist else None

    def phase2(self, src, Q: int, ns_t, th_t, pair_q, pair_idx, hist=None, hot=None):
        """Exact per-shard re-count of (query, acc index) pairs, summed over
        the local shards where it reaches the threshold (ids= semantics);
        from phase 1's kept histograms when given, else rebuilt."""
        import torch

        dev = self.view.device
        P = int(pair_idx.numel())
        out = torch.zeros(P, dtype=torch.int64, device=dev)
        if P and self.S:
            # pairs come sorted by query (nonzero / the union's sorted keys):
            # per-query offsets by a search, no bincount (whose output size
            # needs a host read of the max)
            off = torch.searchsorted(pair_q.to(torch.int64),
                                     torch.arange(Q + 1, device=dev, dtype=torch.int64))
            h, tb = hist if hist is not None else (None, None)
            self._launch(3 if h is not None else 2, Q, src, ns_t, th_t, pair_off=off,
                         pair_idx=pair_idx.to(torch.int32).contiguous(), out=out, hist=h, hot_cnt=hot,
                         tail_built=tb)
        return out

    def _candidates(self, acc, comm):
        """(query, acc index) of every phase-1 candidate.  Across the ranks of
        a node only the candidate SET matters (phase 2 re-counts exactly), so
        the ranks all-gather their fixed-k candidate keys and take the union
        (parallel/collectives.py) instead of all-reducing the dense
        [Q x row-space] accumulator."""
        import torch

        nz = torch.nonzero(acc > 0)
        if comm is None:
            return nz[:, 0].contiguous(), nz[:, 1].contiguous()
        A = max(self.A, 1)
        keys = comm.union(nz[:, 0].to(torch.int64) * A + nz[:, 1].to(torch.int64), tag="topn_src")
        return (keys // A).contiguous(), (keys % A).contiguous()

    def topn(self, engine: GpuEngine, srcs: Sequence[object], ns: Sequence[int], thresholds: Sequence[int],
             comm=None, defer: bool = False):
        with self.rw.read():
            return self._topn(engine, srcs, ns, thresholds, comm, defer)

    def _topn(self, engine: GpuEngine, srcs: Sequence[object], ns: Sequence[int], thresholds: Sequence[int],
             comm=None, defer: bool = False):
        """TopN(field, src_q, n=ns[q], threshold=thresholds[q]) for a batch.
        ``comm`` (parallel/collectives.Comm) spans the ranks of a node: the
        candidate union and the phase-2 sums go through it; every rank must
        call with the same batch.  ``defer``: return a pending result with
        the phase-2 all-reduce still in flight (parallel/mesh.py keeps
        several TopN batches in flight)."""
        from pilosa_amd.parallel.collectives import Pending, PendingAll
        Q = len(srcs)
        if Q == 0:
            return []
        if Q > HOT_Q:   # (the chunking depends on Q only: every rank of a node chunks alike)
            parts = [self._topn(engine, srcs[i:i + HOT_Q], ns[i:i + HOT_Q], thresholds[i:i + HOT_Q], comm, defer)
                     for i in range(0, Q, HOT_Q)]
            cat = lambda rs: [p for r in rs for p in r]   # noqa: E731
            return PendingAll(parts, cat) if defer else cat(parts)
        src = self.materialize(engine, srcs)
        hot = self.hot_counts(src, Q)
        keep = self.hist_bytes(Q) <= HIST_KEEP_BYTES
        acc, ns_t, th_t, hist = self.phase1(src, Q, ns, thresholds, keep_hist=keep, hot=hot)
        pair_q, pair_idx = self._candidates(acc, comm)
        out = self.phase2(src, Q, ns_t, th_t, pair_q, pair_idx, hist=hist, hot=hot)
        space = self.space

        def finish():
            return finish_batch_dev(space, Q, pair_q, pair_idx, out, ns)
        if comm is None:
            return finish()
        pend = Pending(comm, comm.all_reduce_async(out), finish, keep=out)
        return pend if defer else pend.result()

    def shard_pairs(self, engine: GpuEngine, src, n: int, threshold: int,
                    ids: Optional[Sequence[int]] = None) -> List[Pair]:
        with self.rw.read():
            return self._shard_pairs(engine, src, n, threshold, ids)

    def _shard_pairs(self, engine: GpuEngine, src, n: int, threshold: int,
                    ids: Optional[Sequence[int]] = None) -> List[Pair]:
        """One TopN call over the local shards as the executor's map step
        sees it (executor.go:905-930): without ``ids`` the per-shard heap
        results summed by row (phase 1, untrimmed); with ``ids`` the exact
        re-count of those rows (phase 2, summed where >= threshold)."""
        import torch

        dev = self.view.device
        src_t = self.materialize(engine, [src])
        hot = self.hot_counts(src_t, 1)
        if ids is None:
            acc, _, _, _ = self.phase1(src_t, 1, [n], [threshold], hot=hot)
            nz = torch.nonzero(acc[0] > 0).reshape(-1)
            a = nz.cpu().numpy()
            c = acc[0].index_select(0, nz).cpu().numpy()
        else:
            want = np.unique(np.asarray(list(ids), dtype=np.uint64))
            pos = np.searchsorted(self.space, want)
            pos = np.minimum(pos, max(self.A - 1, 0))
            a = pos[(self.A > 0) & (self.space[pos] == want)] if self.A else np.zeros(0, np.int64)
            ns_t = torch.zeros(1, dtype=torch.int32, device=dev)
            th_t = torch.tensor([threshold], dtype=torch.int32).to(dev)
            pa = torch.from_numpy(a.astype(np.int64)).to(dev)
            out = self.phase2(src_t, 1, ns_t, th_t, torch.zeros_like(pa), pa, hot=hot)
            c = out.cpu().numpy()
        keep = c > 0
        ids_out = self.space[a[keep]] if len(a) else np.zeros(0, np.uint64)
        return pairs_from_arrays(ids_out, c[keep])

    def topn_nosrc(self, row_counts, ns: Sequence[int], thresholds: Sequence[int], comm=None):
        with self.rw.read():
            return self._topn_nosrc(row_counts, ns, thresholds, comm)

    def _topn_nosrc(self, row_counts, ns: Sequence[int], thresholds: Sequence[int], comm=None):
        """TopN(field, n) without a src row for a batch, all on the device.
        Phase 1: per shard the first n cache entries at or above the
        threshold (fragment.top stops once its heap holds n rows), summed by
        row with one scatter-add; phase 2 (ids=): every shard's row count of
        each phase-1 id where it reaches the threshold (``row_counts``: the
        int32[S, D] per-shard row counts of the view)."""
        import torch

        Q = len(ns)
        if Q == 0:
            return []
        dev = self.view.device
        nmax = self.K if any(int(n) == 0 for n in ns) else min(self.K, max(int(n) for n in ns))
        lim = torch.tensor([int(n) if int(n) else self.K for n in ns], dtype=torch.int64).to(dev)
        mt = torch.tensor([max(1, int(t)) for t in thresholds], dtype=torch.int32).to(dev)
        # phase 1 as a dense [Q x row-space] scatter-add of the taken cache
        # entries, candidates = its nonzeros.  (Sorted unique (query, id) keys
        # of the <= Q x S x n taken entries instead measured 1.74-1.76 ms per
        # 16-query batch against 1.52-1.64 ms for this, profiles/r02_final/.)
        acc = torch.zeros((Q, max(self.A, 1)), dtype=torch.int32, device=dev)
        if self.S and self.A and nmax:
            cnt = self.cache_cnt[:, :nmax]                                       # [S, n]
            k = torch.arange(nmax, device=dev)
            take = (k[None, None, :] < lim[:, None, None]) & (cnt[None] >= mt[:, None, None])
            vals = torch.where(take, cnt[None], torch.zeros((), dtype=torch.int32, device=dev))
            idx = self.cache_acc[:, :nmax].reshape(1, -1).expand(Q, -1).to(torch.int64)
            acc.scatter_add_(1, idx, vals.reshape(Q, -1))
        pq, pa = self._candidates(acc, comm)
        out = torch.zeros(pa.numel(), dtype=torch.int64, device=dev)
        if pa.numel() and self.S:
            d = self.a2dense[pa].to(torch.int64)
            c = row_counts.index_select(1, d.clamp(min=0))                       # [S, P]
            c = torch.where((c >= mt[pq][None, :]) & (d[None, :] >= 0), c, torch.zeros_like(c))
            out = c.sum(dim=0, dtype=torch.int64)
        if comm is not None:
            comm.all_reduce(out)
        return finish_batch_dev(self.space, Q, pq, pa, out, ns)


def finish_batch_dev(space: np.ndarray, Q: int, pq, pa, cnt, ns: Sequence[int]) -> List[List[Pair]]:
    """finish_batch on the device: (query, count desc, id asc) order by three
    stable sorts (acc indexes are in id order), per-query trim to n, and only
    the kept Q x n pairs cross to the host."""
    import torch

    if pq.numel() == 0:
        return [pair_array(np.zeros(0, np.uint64), np.zeros(0, np.int64)) for _ in range(Q)]
    bq, ba = max(1, int(Q - 1).bit_length()), max(1, int(len(space) - 1).bit_length())
    if bq + 31 + ba <= 63:
        # one sort of a composite key (query, ~count, acc index): acc indexes
        # are in id order, so this is (query, count desc, id asc); zero counts
        # sort last in their query and are dropped with the trim.  The
        # (query, index, count) triples are a few thousand: ONE D2H and the
        # sort / trim on the host (the device version was ~8 small launches
        # and two syncs, 0.33 ms of a src batch -- a third of an 8-GPU
        # rank's fixed per-batch cost, profiles/r06_topn/)
        from .topn_exec import _to_host_pinned
        h = _to_host_pinned(torch.stack([pq.to(torch.int64), pa.to(torch.int64), cnt.to(torch.int64)]))
        c = np.clip(h[2], 0, (1 << 31) - 1)
        key = np.sort((h[0] << (31 + ba)) | (((1 << 31) - 1 - c) << ba) | h[1])
        q_s = key >> (31 + ba)
        c_s = ((1 << 31) - 1) - ((key >> ba) & ((1 << 31) - 1))
        bounds = np.searchsorted(q_s, np.arange(Q + 1, dtype=np.int64))
        lim = np.array([int(n) if int(n) else (1 << 62) for n in ns], dtype=np.int64)
        rank = np.arange(len(key), dtype=np.int64) - bounds[q_s]
        sel = (rank < lim[q_s]) & (c_s > 0)
        kept = key[sel]
        return _split_by_query(Q, kept >> (31 + ba), space[kept & ((1 << ba) - 1)], c_s[sel])
    keep = cnt > 0
    pq, pa, cnt = pq[keep], pa[keep], cnt[keep]
    if pq.numel() == 0:
        return [[] for _ in range(Q)]
    pa = pa.to(torch.int64)
    o = torch.sort(pa, stable=True)[1]
    pq, pa, cnt = pq[o], pa[o], cnt[o]
    o = torch.sort(cnt, descending=True, stable=True)[1]
    pq, pa, cnt = pq[o], pa[o], cnt[o]
    o = torch.sort(pq, stable=True)[1]
    pq, pa, cnt = pq[o], pa[o], cnt[o]
    dev = pq.device
    bounds = torch.searchsorted(pq, torch.arange(Q + 1, device=dev, dtype=pq.dtype))
    lim = torch.tensor([int(n) if int(n) else (1 << 62) for n in ns], dtype=torch.int64).to(dev)
    rank = torch.arange(pq.numel(), device=dev) - bounds[pq]
    sel = rank < lim[pq]
    # one device -> host copy for the kept pairs
    qac = torch.stack([pq[sel].to(torch.int64), pa[sel], cnt[sel].to(torch.int64)]).cpu().numpy()
    return _split_by_query(Q, qac[0], space[qac[1]], qac[2])


def _split_by_query(Q: int, q_h: np.ndarray, ids: np.ndarray, cnt: np.ndarray) -> List["PairArray"]:
    """Per-query columnar results from (query, id, count) rows sorted by
    query (each query's rows already in result order): a Pair object per
    kept row was ~1.7 ms of a 16-query src TopN batch."""
    b = np.searchsorted(q_h, np.arange(Q + 1))
    ids = np.asarray(ids, dtype=np.uint64)
    cnt = np.asarray(cnt, dtype=np.int64)
    return [pair_array(ids[b[q]:b[q + 1]], cnt[b[q]:b[q + 1]]) for q in range(Q)]


def finish_batch(space: np.ndarray, Q: int, pq: np.ndarray, pa: np.ndarray, cnt: np.ndarray,
                 ns: Sequence[int]) -> List[List[Pair]]:
    """Per query: pairs with a positive total, count desc then id asc, trimmed to n."""
    keep = cnt > 0
    pq, pa, cnt = pq[keep], pa[keep], cnt[keep]
    ids = space[pa] if len(pa) else np.zeros(0, np.uint64)
    order = np.lexsort((ids, -cnt, pq))
    pq, ids, cnt = pq[order], ids[order], cnt[order]
    bounds = np.searchsorted(pq, np.arange(Q + 1))
    out = []
    for q in range(Q):
        lo, hi = int(bounds[q]), int(bounds[q + 1])
        n = int(ns[q])
        if n:
            hi = min(hi, lo + n)
        out.append(pair_array(ids[lo:hi], cnt[lo:hi]))
    return out
