"""Device TopN: HBM-resident rank caches + batched two-phase TopN.

Reference semantics (executor.go:863-1000, fragment.go:1568-1700):
  phase 1, per shard: walk the ranked cache (rows by cached count desc, id
  asc); the first n candidates are counted against the src row, later ones
  only while their cached count can still beat the heap minimum; per-shard
  heaps are summed across shards by id (Pairs.Add) and sorted.
  phase 2: the coordinator re-counts src ∩ row for exactly those ids over all
  shards and trims to n.

MI355X design: the per-shard rank caches of a view live on the device
(:class:`DeviceRankCache`, built from the arena's container cardinalities with
one cumsum + gather + top-k per shard chunk); every counting step is one
batched Count(Intersect) launch over ALL local shards (pair kernels), for ALL
queries of a batch at once; the sequential heap walk per (query, shard) runs
in native code (``_roaring.topn_replay``) and asks for deeper prefixes only
where a walk ran past what was counted.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

from pilosa_amd.models.cache import Pair, sort_pairs

from .device import DeviceView, GpuEngine, Leaf, Op


class DeviceRankCache:
    """Top-``k`` (row, count) candidates of every local shard of a view,
    ordered count desc then row asc (the ranked cache order)."""

    def __init__(self, rows: np.ndarray, counts: np.ndarray, row_counts=None):
        self.rows = np.ascontiguousarray(rows, dtype=np.int64)      # [S, K]
        self.counts = np.ascontiguousarray(counts, dtype=np.int64)  # [S, K], 0 = empty slot
        # optional device int32[S, D]: every row's count per shard (ids= lookups
        # of rows outside the cache, fragment.go row count fallback)
        self.row_counts = row_counts

    @property
    def S(self) -> int:
        return self.rows.shape[0]

    @classmethod
    def from_view(cls, view: DeviceView, k: int = 50000, shard_chunk: int = 32,
                  keep_row_counts: bool = False) -> "DeviceRankCache":
        import torch

        S, D = view.S, view.D
        k = max(1, min(k, D)) if D else 1
        rows_out = np.zeros((S, k), np.int64)
        cnt_out = np.zeros((S, k), np.int64)
        if D == 0 or S == 0:
            return cls(rows_out, cnt_out)
        dev = view.device
        n = ((view.t_meta >> 6) & 0x1FFFF).to(torch.int64)
        cs = torch.zeros(n.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(n, 0, out=cs[1:])
        rp = view.t_rowptr.view(S, D + 1).to(torch.int64)  # int32 storage of u32 offsets (< 2^31 per shard)
        sb = view.t_shard_base.to(torch.int64)
        dense = torch.arange(D, dtype=torch.int64, device=dev)
        row_ids = torch.from_numpy(view.rows.astype(np.int64)).to(dev)
        all_counts = torch.empty((S, D), dtype=torch.int32, device=dev) if keep_row_counts else None
        for s0 in range(0, S, shard_chunk):
            s1 = min(S, s0 + shard_chunk)
            idx = sb[s0:s1, None] + rp[s0:s1]                       # [c, D+1] absolute container offsets
            counts = cs[idx[:, 1:]] - cs[idx[:, :-1]]               # [c, D] row cardinality per shard
            if all_counts is not None:
                all_counts[s0:s1] = counts.to(torch.int32)
            key = (counts << 32) | (0xFFFFFFFF - dense)             # count desc, then row asc
            top = torch.topk(key, k, dim=1, sorted=True).values
            c = top >> 32
            d = 0xFFFFFFFF - (top & 0xFFFFFFFF)
            rows_out[s0:s1] = row_ids[d].cpu().numpy()
            cnt_out[s0:s1] = c.cpu().numpy()
        return cls(rows_out, cnt_out, all_counts)


def _union_ids(a: np.ndarray) -> np.ndarray:
    """Sorted distinct ids; O(n) through a presence mask for small ids."""
    if not len(a):
        return a.astype(np.int64)
    mx = int(a.max())
    if 0 <= int(a.min()) and mx < (1 << 26):
        m = np.zeros(mx + 1, bool)
        m[a] = True
        return np.flatnonzero(m).astype(np.int64)
    return np.unique(a)


def topn_phase1(engine: GpuEngine, rv: DeviceView, cache: DeviceRankCache, srcs: Sequence[object], n: int = 10,
                threshold: int = 1, first_depth: int = 256, nthreads: int = 16) -> List[Dict[int, int]]:
    """Per query: {row id: summed per-shard heap count} over the local shards."""
    from pilosa_amd import _roaring

    Q, S, K = len(srcs), cache.S, cache.rows.shape[1]
    seen: List[np.ndarray] = [np.zeros(0, np.int64) for _ in range(Q)]
    blocks: List[list] = [[] for _ in range(Q)]  # per query: (rows[r], counts[S, r]) per round
    depth = np.zeros(Q, np.int64)
    pending: Dict[int, np.ndarray] = {q: np.arange(S, dtype=np.int32) for q in range(Q)}
    got_ids: List[list] = [[] for _ in range(Q)]
    got_cnt: List[list] = [[] for _ in range(Q)]
    while pending:
        qs, news = [], []
        for q, shards in pending.items():
            depth[q] = min(K, max(first_depth, max(n * 2, 1), int(depth[q]) * 4))
            c = cache.rows[shards, :depth[q]][cache.counts[shards, :depth[q]] > 0]
            cand = _union_ids(c)
            new = cand[~np.isin(cand, seen[q], assume_unique=True)] if len(seen[q]) else cand
            seen[q] = np.union1d(seen[q], new)
            qs.append(q)
            news.append(new)
        if sum(len(x) for x in news):
            mat = _count_src_rows_vec(engine, rv, srcs, qs, news)  # [S, P]
            o = 0
            for q, new in zip(qs, news):
                if len(new):
                    blocks[q].append((new, np.ascontiguousarray(mat[:, o:o + len(new)])))
                o += len(new)
        nxt: Dict[int, np.ndarray] = {}
        for q, shards in pending.items():
            need, ids, cnts = _roaring.topn_replay(cache.rows, cache.counts, shards, n, threshold, blocks[q], nthreads)
            got_ids[q].append(ids)
            got_cnt[q].append(cnts)
            if need.any():
                nxt[q] = shards[need]
        pending = nxt
    totals = []
    for q in range(Q):
        ids = np.concatenate(got_ids[q]) if got_ids[q] else np.zeros(0, np.int64)
        cnts = np.concatenate(got_cnt[q]) if got_cnt[q] else np.zeros(0, np.int64)
        u, inv = np.unique(ids, return_inverse=True)
        sums = np.zeros(len(u), np.int64)
        np.add.at(sums, inv, cnts)
        totals.append(dict(zip(u.tolist(), sums.tolist())))
    return totals


def _count_src_rows_vec(engine: GpuEngine, rv: DeviceView, srcs: Sequence[object], qs: List[int],
                        rows: List[np.ndarray]) -> np.ndarray:
    """Shard-major [S, P] counts of |src_q ∩ row| for every (q, rows[q]) block."""
    if all(type(srcs[q]) is Leaf for q in qs):
        views: List[DeviceView] = [rv]
        slot = {id(rv): 0}
        a_slot, a_dense = [], []
        for q, r in zip(qs, rows):
            src = srcs[q]
            sl = slot.get(id(src.view))
            if sl is None:
                sl = slot[id(src.view)] = len(views)
                views.append(src.view)
            a_slot.append(np.full(len(r), sl, np.int32))
            a_dense.append(np.full(len(r), src.view.dense(src.row), np.int64))
        allrows = np.concatenate(rows)
        progs = engine.pair_programs(0, np.concatenate(a_dense), 0, rv.dense_many(allrows.astype(np.uint64)))
        progs["leaf_view"][:, 0] = np.concatenate(a_slot)
        t = engine.count_per_shard_progs(progs, views, rv.S, as_tensor=True)
        # per-shard counts fit int32 (<= 2^20): halve the device->host bytes
        import torch
        return t.t().to(torch.int32).contiguous().cpu().numpy()
    owners = [(q, int(r)) for q, rr in zip(qs, rows) for r in rr.tolist()]
    return _count_src_rows(engine, rv, srcs, owners, shard_major=True).astype(np.int32)


def topn_phase2_counts(engine: GpuEngine, rv: DeviceView, srcs: Sequence[object], ids: Sequence[Sequence[int]],
                       threshold: int = 1) -> List[np.ndarray]:
    """Exact src ∩ row counts of the phase-1 ids over the local shards; per-shard
    counts below the threshold are dropped, as fragment.top() does for every
    shard of the ids= re-query."""
    owners = [(q, int(i)) for q in range(len(srcs)) for i in ids[q]]
    if not owners:
        return [np.zeros(0, np.int64) for _ in srcs]
    per_shard = _count_src_rows(engine, rv, srcs, owners)
    flat = np.where(per_shard >= max(threshold, 1), per_shard, 0).sum(axis=1)
    out, o = [], 0
    for q in range(len(srcs)):
        out.append(flat[o:o + len(ids[q])])
        o += len(ids[q])
    return out


def _count_src_rows(engine: GpuEngine, rv: DeviceView, srcs: Sequence[object], owners,
                    shard_major: bool = False) -> np.ndarray:
    """|src_q ∩ row r| per local shard for (q, r) pairs -> int64[P, S]
    (or [S, P] with ``shard_major``, transposed on the device).
    Single-row sources (the common TopN(f, Row(...)) shape) are encoded as
    pair programs directly; other trees go through the expression compiler."""
    if all(type(srcs[q]) is Leaf for q, _ in owners):
        views: List[DeviceView] = [rv]
        slot = {id(rv): 0}
        a_slot = np.empty(len(owners), np.int32)
        a_dense = np.empty(len(owners), np.int64)
        for k, (q, _) in enumerate(owners):
            src = srcs[q]
            sl = slot.get(id(src.view))
            if sl is None:
                sl = slot[id(src.view)] = len(views)
                views.append(src.view)
            a_slot[k] = sl
            a_dense[k] = src.view.dense(src.row)
        b_dense = rv.dense_many(np.array([r for _, r in owners], np.uint64))
        progs = engine.pair_programs(0, a_dense, 0, b_dense)
        progs["leaf_view"][:, 0] = a_slot
        t = engine.count_per_shard_progs(progs, views, rv.S, as_tensor=True)
    else:
        p, v, S = engine.compile_batch([Op("and", (srcs[q], Leaf(rv, int(r)))) for q, r in owners])
        t = engine.count_per_shard_progs(p, v, S, as_tensor=True)
    if shard_major:
        t = t.t()
    return t.contiguous().cpu().numpy()


def finish_topn(ids: Sequence[int], counts: np.ndarray, n: int) -> List[Pair]:
    p = sort_pairs([Pair(int(i), int(c)) for i, c in zip(ids, counts.tolist()) if c > 0])
    return p[:n] if n else p


def topn_batch(engine: GpuEngine, rv: DeviceView, cache: DeviceRankCache, srcs: Sequence[object], n: int = 10,
               threshold: int = 1, first_depth: int = 256) -> List[List[Pair]]:
    """TopN(field, <src>, n) for a batch of src expressions over the view
    ``rv`` whose rank caches are ``cache`` (single process: phase 1, then the
    ids= re-count, then trim)."""
    totals = topn_phase1(engine, rv, cache, srcs, n, threshold, first_depth)
    ids = [sorted(t) for t in totals]
    exact = topn_phase2_counts(engine, rv, srcs, ids, threshold)
    return [finish_topn(ids[q], exact[q], n) for q in range(len(srcs))]


def topn_cache_phase1(cache: DeviceRankCache, n: int, threshold: int = 1) -> Dict[int, int]:
    """TopN(field, n) without a src row: per shard the first n cache entries
    at or above the threshold (fragment.top's fill phase ends the walk as soon
    as the heap holds n rows), summed by id."""
    k = min(n, cache.rows.shape[1]) if n else cache.rows.shape[1]
    c = cache.counts[:, :k]
    m = c >= max(threshold, 1)
    ids, inv = np.unique(cache.rows[:, :k][m], return_inverse=True)
    sums = np.bincount(inv, weights=c[m], minlength=len(ids)).astype(np.int64)
    return dict(zip(ids.tolist(), sums.tolist()))


def topn_cache_phase2_counts(cache: DeviceRankCache, view: DeviceView, ids: Sequence[int], threshold: int = 1):
    """ids= re-count without a src: each shard's row count (>= threshold) of
    every id, summed over the local shards (device gather + reduce)."""
    import torch

    if cache.row_counts is None:
        raise ValueError("DeviceRankCache built without keep_row_counts")
    if not len(ids):
        return np.zeros(0, np.int64)
    dense = view.dense_many(np.asarray(ids, np.uint64))
    d = torch.from_numpy(np.maximum(dense, 0)).to(cache.row_counts.device)
    cols = cache.row_counts.index_select(1, d).to(torch.int64)          # [S, I]
    cols = torch.where(cols >= max(threshold, 1), cols, torch.zeros_like(cols))
    out = cols.sum(dim=0).cpu().numpy()
    out[dense < 0] = 0
    return out
