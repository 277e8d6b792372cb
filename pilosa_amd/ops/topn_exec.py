"""Executor-path TopN on the device: rank caches built without touching the
host fragments, and batched two-phase TopN over all local shards.

Reference: executor.go:863-1000 (executeTopN: phase 1 per-shard ``top``,
Pairs.Add over shards, phase 2 ``ids=`` re-count, trim to n),
fragment.go:1568-1712 (``top`` / ``topBitmapPairs``), fragment.go:459
(``openCache``: the persisted ``<shard>.cache`` ids with a CountRange each),
cache.go:235-281 (rank cache order).

MI355X design.  A lazily opened fragment is never read on the host for TopN:

* its rank cache is the id list of its ``.cache`` file (read natively,
  ``_roaring.read_cache_files``) with each row's count taken from the HBM arena
  metadata by ``row_counts_kernel`` -- exactly what ``openCache`` computes with
  CountRange on the mapped file;
* a fragment already warm on the host (written to since open) contributes its
  live host rank cache (``fragment.cache.top()``), as the reference would.

The per-shard lists are ranked on the device (count desc, id asc) into
``[S, K]`` tensors that feed both the cache-only TopN here and the src-TopN
slot index (ops/topn_index.py).  A batch of TopN calls is answered with both
phases on the device: phase 1 as one scatter-add of every query's per-shard
cache prefixes, phase 2 (``ids=``) as ``row_counts_sum_kernel`` over the
candidates, and only the trimmed ``Q x n`` pairs cross to the host.  On one
rank the whole batch is the three ``topn_cache_*`` kernels
(``_topn_nosrc_fused``): membership, per-threshold totals from a memoised
candidate x shard count matrix, and a per-query LDS bitonic top-n.
"""
from __future__ import annotations

import itertools
import os
import threading
from typing import List, Optional, Sequence

import numpy as np

from pilosa_amd.models.cache import Pair, pair_array, pair_arrays_split, pairs_from_arrays

from .device import DeviceView, kernels

# queries per cache-only phase-1 accumulator (Q x D int32 scratch)
NOSRC_CHUNK = 64
# largest [candidate x shard] count matrix the fused cache-only path memoises
FUSED_MAX_CELLS = 1 << 25


def prefix_bucket(n: int) -> int:
    """Cache prefix length for a batch whose largest n is ``n``: the next
    power of two (at least 16).  Candidate sets and count matrices are
    memoised per prefix, so a stream of calls with varied n builds a handful
    of them instead of one per distinct n."""
    n = max(1, int(n))
    return max(16, 1 << (n - 1).bit_length())


# cache-only TopN batches on a side stream (0: the current stream)
I32_MAX = (1 << 31) - 1


def clamp_topn_params(ns: Sequence[int], thresholds: Sequence[int]):
    """n and threshold as the int32 kernel parameters hold them.  The PQL
    grammar takes both up to 2^63-1; an n at or above 2^31 keeps every
    candidate and a threshold there admits no shard count of a 2^20..2^31
    column shard, so clamping changes no answer (an unclamped
    value overflowed the parameter array and was counted as a device fault)."""
    return ([min(int(n), I32_MAX) for n in ns], [min(max(int(t), 0), I32_MAX) for t in thresholds])


SIDE_STREAM = os.environ.get("PILOSA_TOPN_SIDE_STREAM", "1") != "0"
# cache-only batches through the native request object (binding.cpp CacheTopN);
# 0 = the Python lane path (kept for A/B runs)
NATIVE_FUSED = os.environ.get("PILOSA_TOPN_NATIVE", "1") != "0"


class _Lane:
    """A side stream and a pinned int32 parameter buffer, owned by one batch
    at a time.  The batch copies its parameters from the buffer on the
    stream and ends in a blocking D2H, so the next owner may overwrite it."""

    def __init__(self, device):
        import torch
        self.device = device
        self.stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self.run_stream = self.stream   # the stream the current batch runs on
        self.pin = None
        self._bufs = {}

    def pinned_i32(self, n: int):
        import torch
        if self.pin is None or self.pin.numel() < n:
            self.pin = torch.empty(max(n, 1024), dtype=torch.int32, pin_memory=True)
        return self.pin[:n]

    def buf(self, name: str, n: int, dtype, pinned: bool = False):
        """A reusable 1-D buffer of at least ``n`` elements (device, or pinned
        host): a batch's member / totals / answer tensors and their host copy
        cost no allocator calls once the lane is warm."""
        import torch
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            size = max(n, 1024) + (max(n, 1024) >> 1)
            b = (torch.empty(size, dtype=dtype, pin_memory=True) if pinned
                 else torch.empty(size, dtype=dtype, device=self.device))
            self._bufs[name] = b
        return b[:n]


_LANES: dict = {}
_LANES_MU = threading.Lock()


def _lane_take(device) -> "_Lane":
    """A free lane of ``device`` (a new one when all are taken): concurrent
    batches run on their own streams, and a serving thread pays no stream or
    pinned-buffer creation after the first batches."""
    with _LANES_MU:
        free = _LANES.setdefault(device, [])
        if free:
            return free.pop()
    return _Lane(device)


def _lane_give(device, lane: "_Lane") -> None:
    with _LANES_MU:
        _LANES.setdefault(device, []).append(lane)


def rows_dev(view: DeviceView):
    """int64 device copy of the view's sorted row directory (cached per view)."""
    import torch
    got = getattr(view, "_rows_dev", None)
    if got is None or got[0] != view.generation or got[1].numel() != view.D:
        t = torch.from_numpy(np.ascontiguousarray(view.rows).view(np.int64)).to(view.device)
        got = (view.generation, t)
        view._rows_dev = got
    return got[1]


def dense_dev(view: DeviceView, ids):
    """Row ids (int64 device tensor) -> dense row indexes of ``view`` (int32, -1 absent)."""
    import torch
    D = view.D
    if D == 0 or ids.numel() == 0:
        return torch.full(ids.shape, -1, dtype=torch.int32, device=ids.device)
    if int(view.rows[-1]) == D - 1:   # identity directory (rows 0..D-1)
        return torch.where((ids >= 0) & (ids < D), ids, torch.full_like(ids, -1)).to(torch.int32)
    rows = rows_dev(view)
    i = torch.searchsorted(rows, ids).clamp_(max=D - 1)
    return torch.where(rows[i] == ids, i, torch.full_like(i, -1)).to(torch.int32)


_RC_SERIAL = itertools.count(1)


class NodeCandidates:
    """One rank's view of a node candidate space (mesh cache-only TopN):
    ``space`` the sorted node-wide candidate row ids, ``nmax`` the local
    cache prefix, ``inv`` int32[S * nmax] the node index of each local rank
    slot, ``cm`` int32[U, S] each candidate's count per local fragment,
    ``ids`` arange(U) (the select kernel's tie-break ids)."""

    __slots__ = ("space", "nmax", "inv", "cm", "ids")

    def __init__(self, space, nmax, inv, cm, ids):
        self.space, self.nmax, self.inv, self.cm, self.ids = space, int(nmax), inv, cm, ids


def _select_from_buffer(buf, Q: int, T: int, U: int, q: int, t: int, lim: int) -> np.ndarray:
    """Query q's top composite keys (count << 32 | ~index) from an all-reduced
    partial buffer, with torch (the select kernel's LDS overflow case)."""
    import torch
    mw = (Q * U + 3) // 4
    member = buf[:mw].view(torch.uint8)[q * U:(q + 1) * U]
    tot = buf[mw + t * U:mw + (t + 1) * U].to(torch.int64)
    idx = torch.arange(U, device=buf.device, dtype=torch.int64)
    key = torch.where((member > 0) & (tot > 0), (tot << 32) | (0xFFFFFFFF - idx), torch.full_like(tot, -1))
    k = min(int(lim), U)
    top = torch.topk(key, k).values if k else key[:0]
    h = top.cpu().numpy()
    return h[h >= 0]


_TL = threading.local()


def _to_host_pinned(t) -> np.ndarray:
    """Device tensor -> numpy through a per-thread pinned buffer and a wait on
    the current stream only (a pageable .cpu() goes through a blit kernel and
    a device-wide wait).  The array is valid until this thread's next call."""
    import torch
    if t.device.type != "cuda":
        return t.cpu().numpy()
    n = t.numel()
    hb = getattr(_TL, "hb", None)
    if hb is None or hb.numel() < n or hb.dtype != t.dtype:
        hb = torch.empty(max(n, 4096), dtype=t.dtype, pin_memory=True)
        _TL.hb = hb
    h = hb[:n]
    h.copy_(t.reshape(-1), non_blocking=True)
    torch.cuda.current_stream(t.device).synchronize()
    return h.numpy().reshape(t.shape)


def cache_partial_ref(cnt, nmax: int, nlim: int, inv, cm, prm, Q: int, T: int, U: int, buf) -> None:
    """PyTorch reference of topn_cache_partial (kernels/topn_kernels.hip) for
    the mesh buffer [member bytes | int32 totals[T, U] | flags[2]]: the CPU
    path of mesh_cache_batch and the numerics oracle of the kernel."""
    import torch
    buf.zero_()
    mw = (Q * U + 3) // 4
    member = buf[:mw].view(torch.uint8)[:Q * U].view(Q, U)
    S = int(cnt.shape[0])
    p = prm.to(torch.int64)
    if S and nlim:
        c = cnt[:, :nlim].to(torch.int64)                                   # [S, nlim]
        j = inv.view(S, nmax)[:, :nlim].to(torch.int64)
        k = torch.arange(nlim)
        lim = torch.clamp(p[:Q], max=nlim)
        take = (k[None, None, :] < lim[:, None, None]) & (c[None] >= p[Q:2 * Q][:, None, None]) & (c[None] > 0)
        for q in range(Q):
            member[q, j[take[q]]] = 1
    th = p[4 * Q:4 * Q + T]
    cm64 = cm.to(torch.int64).view(U, S) if S else torch.zeros((U, 0), dtype=torch.int64)
    tot = torch.where(cm64[None] >= th[:, None, None], cm64[None], torch.zeros((), dtype=torch.int64)).sum(dim=2)
    buf[mw:mw + T * U] = tot.reshape(-1).to(torch.int32)


def cache_select_ref(buf, ids, prm, Q: int, T: int, KK: int):
    """PyTorch reference of topn_cache_select32: out int64[Q, KK + 1], column
    0 the rows kept (-3 / -4 when the reduced flags say stale / declined)."""
    import torch
    U = int(ids.numel())
    mw = (Q * U + 3) // 4
    out = torch.zeros((Q, KK + 1), dtype=torch.int64)
    fl = buf[mw + T * U:mw + T * U + 2].tolist()
    if fl[0] or fl[1]:
        out[:, 0] = -4 if fl[1] else -3
        return out
    member = buf[:mw].view(torch.uint8)[:Q * U].view(Q, U)
    p = prm.to(torch.int64)
    d = ids.to(torch.int64)
    for q in range(Q):
        tq = buf[mw + int(p[2 * Q + q]) * U:mw + (int(p[2 * Q + q]) + 1) * U].to(torch.int64)
        ok = (member[q] > 0) & (d >= 0) & (tq > 0)
        keys = torch.sort((tq[ok] << 32) | (0xFFFFFFFF - d[ok]), descending=True).values
        lim = min(int(keys.numel()), int(p[3 * Q + q]), KK)
        out[q, 0] = lim
        out[q, 1:1 + lim] = keys[:lim]
    return out


def mesh_cache_batch(rc: Optional["DeviceRankCaches"], ns: Sequence[int], thresholds: Sequence[int], comm,
                     cand: Optional[NodeCandidates], U: int, stale: int = 0, declined: int = 0,
                     defer: bool = False, device=None, space=None, ids=None):
    """One rank's share of a cache-only TopN batch across the ranks of a node,
    in ONE collective: every rank writes its membership bytes, int32 partial
    totals over the node candidate space and two flag words -- its vote
    [stale candidate space, declined] -- into one buffer
    (topn_cache_partial), the ranks all-reduce it, and the front end runs the
    per-query LDS top-n on the sum (topn_cache_select32).  The union of the
    per-shard candidate lists is the sum's nonzero membership, and a total
    summed per shard where it reaches the threshold is the node's ids=
    re-count (executor.go:863-903), so no candidate union or re-count round
    trip is needed, and the readiness vote needs no collective of its own:
    a rank that cannot take part (no usable candidate space: ``stale``; no
    caches or an error: ``declined``) sends zeros and its flag, and the
    select then answers nothing (the front end refreshes the space or takes
    the general path).  ``U`` comes from the command, so every rank's buffer
    has the same size whatever its local state.  The result (after the
    collective) is a list of PairArrays, or the string "stale" / "declined".
    ``space`` / ``ids`` (the node space and the select's tie-break ids)
    default to ``cand``'s; a rank with no local caches passes them alone."""
    import torch

    from pilosa_amd.parallel.collectives import Pending
    ns, thresholds = clamp_topn_params(ns, thresholds)
    Q = len(ns)
    nn = [int(n) for n in ns]
    dev = rc.view.device if rc is not None else (device if device is not None else comm.device)
    if space is None and cand is not None:
        space = cand.space
    if ids is None and cand is not None:
        ids = cand.ids
    k = kernels() if dev.type == "cuda" and NATIVE_FUSED else None
    if k is not None and hasattr(k, "mesh_cache_issue"):
        # parameters, partial and answers natively (binding.cpp mesh_cache_issue / _finish)
        part = cand is not None and not stale and not declined and rc is not None and cand.nmax > 0 and rc.S > 0
        z = _EMPTY_I32.get(dev)
        if z is None:
            z = _EMPTY_I32[dev] = torch.zeros(0, dtype=torch.int32, device=dev)
        buf, prm_d, T, KK = k.mesh_cache_issue(rc.cache_cnt if part else z, cand.nmax if part else 0,
                                               cand.inv if part else z, cand.cm if part else z, nn, thresholds,
                                               int(U), rc.K if rc is not None else 0, int(bool(stale)),
                                               int(bool(declined)), dev.index or 0)

        def finish_native():
            if ids is None or space is None:
                return "stale"
            got = k.mesh_cache_finish(buf, ids, prm_d, Q, T, KK, space)
            if isinstance(got, str):
                return got
            if got is None:   # a query overflowed the select: the torch path below
                return _finish_cache_batch(buf, prm_d, ids, space, Q, T, U, KK)
            return pair_arrays_split(*got)
        pend = Pending(comm, comm.all_reduce_async(buf), finish_native, keep=(buf, prm_d))
        return pend if defer else pend.result()
    ths = [max(1, int(t)) for t in thresholds]
    uniq_t = sorted(set(ths))
    T = len(uniq_t)
    K = rc.K if rc is not None else 0
    KK = min(U, max(nn)) if all(nn) else U
    prm = np.empty(4 * Q + T, np.int32)
    prm[:Q] = [n if n else K for n in nn]
    prm[Q:2 * Q] = ths
    tix = {t: i for i, t in enumerate(uniq_t)}
    prm[2 * Q:3 * Q] = [tix[t] for t in ths]
    prm[3 * Q:4 * Q] = [n if n else KK for n in nn]
    prm[4 * Q:] = uniq_t
    prm_d = kernels().upload_i32(torch.from_numpy(prm), dev.index or 0) if dev.type == "cuda" else \
        torch.from_numpy(prm)
    mw = (Q * U + 3) // 4
    buf = torch.empty(mw + T * U + 2, dtype=torch.int32, device=dev)
    part = cand is not None and not stale and not declined and rc is not None and cand.nmax > 0 and rc.S > 0
    if part:
        nlim = min(cand.nmax, max(int(p) for p in prm[:Q])) if Q else cand.nmax
        if dev.type == "cuda":
            kernels().topn_cache_partial(rc.cache_cnt, cand.nmax, nlim, cand.inv, cand.cm, prm_d, Q, T, U, buf, 0, 0)
        else:
            cache_partial_ref(rc.cache_cnt, cand.nmax, nlim, cand.inv, cand.cm, prm_d, Q, T, U, buf)
    else:
        z = torch.zeros(0, dtype=torch.int32, device=dev)
        if dev.type == "cuda":
            kernels().topn_cache_partial(z, 0, 0, z, z, prm_d, Q, T, U, buf, int(bool(stale)), int(bool(declined)))
        else:
            buf.zero_()
            buf[-2] = int(bool(stale))
            buf[-1] = int(bool(declined))

    def finish():
        if ids is None or space is None:
            return "stale"
        return _finish_cache_batch(buf, prm_d, ids, space, Q, T, U, KK)
    pend = Pending(comm, comm.all_reduce_async(buf), finish, keep=(buf, prm_d))
    return pend if defer else pend.result()


_EMPTY_I32: dict = {}


def _finish_cache_batch(buf, prm_d, ids, space, Q: int, T: int, U: int, KK: int):
    """The front end's end of a mesh cache-only batch in torch / numpy (the
    CPU path, and the select-overflow case of the native one): per-query
    top-n of the all-reduced buffer, decoded against the node space."""
    import torch
    if buf.device.type == "cuda":
        out = torch.empty((Q, KK + 1), dtype=torch.int64, device=buf.device)
        kernels().topn_cache_select32(buf, ids, prm_d, Q, T, out)
    else:
        out = cache_select_ref(buf, ids, prm_d, Q, T, KK)
    h = _to_host_pinned(out)
    if Q and h[0, 0] <= -3:
        return "declined" if h[0, 0] == -4 else "stale"
    prm = prm_d.cpu().numpy() if buf.device.type == "cuda" else prm_d.numpy()
    lens = h[:, 0]
    if (lens < 0).any():    # more members than one workgroup sorts: torch over the reduced buffer
        parts = [_select_from_buffer(buf, Q, T, U, q, int(prm[2 * Q + q]), int(prm[3 * Q + q]))
                 if lens[q] < 0 else h[q, 1:1 + int(lens[q])] for q in range(Q)]
        ln = [len(r) for r in parts]
    else:
        ln = lens.tolist()
        parts = [h[q, 1:1 + n] for q, n in enumerate(ln)]
    # every query's kept keys end to end, decoded in one pass, then split
    # (as the 1-GPU batch decodes: _topn_nosrc_fused_on)
    keys = np.concatenate(parts) if Q else np.zeros(0, np.int64)
    rid = space[0xFFFFFFFF - (keys & 0xFFFFFFFF)] if len(keys) else np.zeros(0, np.uint64)
    cnt = keys >> 32
    res, o = [], 0
    for n in ln:
        res.append(pair_array(rid[o:o + n], cnt[o:o + n]))
        o += n
    return res


class DeviceRankCaches:
    """Ranked caches of every local shard of one view, on the device.

    ``cache_dense`` int32[S, K] (dense row of each rank, -1 empty) and
    ``cache_cnt`` int32[S, K] (its count, 0 empty), ranks ordered count desc
    then row asc.  ``cold_shards`` counts the shards whose ranks came from
    the ``.cache`` file (fragment never loaded on the host)."""

    def __init__(self, view: DeviceView, frags: Sequence, nthreads: int = 16):
        import torch

        from pilosa_amd import _roaring
        self.view = view
        self.generation = view.generation
        self.serial = next(_RC_SERIAL)   # identity of this ranking (mesh candidate spaces key on it)
        # one rank cache per fragment; a fragment wider than 2^20 columns is
        # M device sub-shards of the arena (pilosa_amd/shardwidth.py), whose
        # row counts are summed per fragment
        S = len(frags)
        if S and view.S % S:
            raise ValueError(f"DeviceRankCaches: {view.S} arena shards for {S} fragments")
        self.M = view.S // S if S else 1
        dev = view.device
        self.S = S
        # the persisted .cache ids serve a fragment whose cache was never
        # opened; once a write opened it (mapped fragments too) the live host
        # cache is the ranking, as fragment.top would use
        cold = [f is not None and f.is_cold() and not f.cache_is_live() for f in frags]
        paths = [frags[si].cache_path() if cold[si] else "" for si in range(S)]
        offs, ids, ok = _roaring.read_cache_files(paths, nthreads)
        # a corrupt .cache file: the host fragment rebuilds its cache (openCache)
        warm = [si for si in range(S) if frags[si] is not None and (not cold[si] or not ok[si])]
        self.cold_shards = sum(1 for si in range(S) if cold[si] and ok[si])
        lens = np.diff(offs)
        for si in warm:
            lens[si] = 0
        keep = np.repeat(lens > 0, np.diff(offs)) if len(ids) else np.zeros(0, bool)
        shard_of = np.repeat(np.arange(S, dtype=np.int32), lens)
        ids = ids[keep] if len(ids) else ids
        t_shard = torch.from_numpy(shard_of).to(dev)
        t_row = torch.from_numpy(np.ascontiguousarray(ids).view(np.int64)).to(dev)
        t_dense = dense_dev(view, t_row)
        t_cnt = self._counts(t_shard, t_dense)
        if warm:
            # host rank caches of fragments loaded on the host (their live counts)
            hs, hd, hc, hr = [], [], [], []
            for si in warm:
                with frags[si].mu:
                    pairs = list(frags[si].cache.top())
                if not pairs:
                    continue
                a = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
                hs.append(np.full(len(a), si, np.int32))
                hr.append(a[:, 0])
                hd.append(view.dense_many(a[:, 0].astype(np.uint64)).astype(np.int32))
                hc.append(np.minimum(a[:, 1], 2 ** 31 - 1).astype(np.int32))
            if hs:
                t_shard = torch.cat([t_shard, torch.from_numpy(np.concatenate(hs)).to(dev)])
                t_dense = torch.cat([t_dense, torch.from_numpy(np.concatenate(hd)).to(dev)])
                t_cnt = torch.cat([t_cnt, torch.from_numpy(np.concatenate(hc)).to(dev)])
                t_row = torch.cat([t_row, torch.from_numpy(np.concatenate(hr)).to(dev)])
        N = t_dense.numel()
        if N == 0 or S == 0:
            self.K = 0
            self.cache_dense = torch.full((S, 0), -1, dtype=torch.int32, device=dev)
            self.cache_cnt = torch.zeros((S, 0), dtype=torch.int32, device=dev)
            return
        # rank per shard on the device: key = count << 32 | (~dense), sorted desc
        order = torch.argsort(t_shard.to(torch.int64) * (1 << 32) + torch.arange(N, device=dev), stable=False)
        t_shard, t_dense, t_cnt = t_shard[order], t_dense[order], t_cnt[order]
        per = torch.bincount(t_shard.to(torch.int64), minlength=S)
        start = torch.zeros(S + 1, dtype=torch.int64, device=dev)
        start[1:] = torch.cumsum(per, 0)
        pos = torch.arange(N, device=dev) - start[t_shard.to(torch.int64)]
        K = int(per.max().item())
        valid = (t_cnt > 0) & (t_dense >= 0)
        # ties order by row id as the host cache does (count desc, id asc),
        # not by dense index: a dense index follows the arena's row order of
        # first appearance, and at a cache_size cut of a tied count the two
        # orders keep different rows.  The key's low word is the row's rank
        # among the distinct row ids (order-preserving, < 2^32).
        urow, rinv = torch.unique(t_row, sorted=True, return_inverse=True)
        dense_of = torch.full((urow.numel(),), -1, dtype=torch.int64, device=dev)
        dense_of[rinv] = t_dense.to(torch.int64)
        key = torch.where(valid, (t_cnt.to(torch.int64) << 32) | (0xFFFFFFFF - rinv.to(torch.int64)),
                          torch.full_like(pos, -1))
        mat = torch.full((S, K), -1, dtype=torch.int64, device=dev)
        mat[t_shard.to(torch.int64), pos] = key
        mat = torch.sort(mat, dim=1, descending=True).values
        # a ranked cache keeps its cache_size best entries (rankCache.recalculate,
        # cache.go:245-281): a .cache file may list up to 1.1x that many ids
        sizes = [f.cache_size for f in frags if f is not None and f.cache_type == "ranked" and f.cache_size > 0]
        if sizes and K > max(sizes):
            mat = mat[:, :max(sizes)]
        live = mat >= 0
        kmax = int(live.sum(dim=1).max().item()) if K else 0
        mat, live = mat[:, :kmax], live[:, :kmax]
        self.K = kmax
        self.cache_cnt = torch.where(live, mat >> 32, torch.zeros_like(mat)).to(torch.int32).contiguous()
        rix = torch.where(live, 0xFFFFFFFF - (mat & 0xFFFFFFFF), torch.zeros_like(mat))
        self.cache_dense = torch.where(live, dense_of[rix], torch.full_like(mat, -1)).to(torch.int32).contiguous()
        if dev.type == "cuda":   # the side stream of cache-only batches starts after this point
            self._ready = torch.cuda.Event()
            self._ready.record()

    def nbytes(self) -> int:
        return 8 * self.S * self.K

    def _counts(self, t_shard, t_dense):
        """int32 count of each (fragment index, dense row) entry over the
        fragment's arena shards (row_counts_kernel)."""
        import torch
        N = int(t_dense.numel())
        dev = self.view.device
        if not N:
            return torch.zeros(0, dtype=torch.int32, device=dev)
        M = self.M
        if M > 1:
            t_shard = (t_shard.to(torch.int32)[:, None] * M +
                       torch.arange(M, dtype=torch.int32, device=dev)[None, :]).reshape(-1).contiguous()
            t_dense = t_dense.to(torch.int32).repeat_interleave(M).contiguous()
        out = torch.zeros(N * M, dtype=torch.int32, device=dev)
        kernels().row_counts(self.view.viewdev_tensor(), t_shard.contiguous(), t_dense.contiguous(), out)
        return out if M == 1 else out.view(N, M).sum(dim=1, dtype=torch.int32)

    def _count_matrix(self, u32):
        """int32[U, S]: every candidate row's count in every fragment."""
        import torch
        U = int(u32.numel())
        D = self.view.S
        cm = torch.empty((U, D), dtype=torch.int32, device=self.view.device)
        kernels().topn_cache_counts(self.view.viewdev_tensor(), D, u32, cm)
        if self.M > 1:
            cm = cm.view(U, self.S, self.M).sum(dim=2, dtype=torch.int32).contiguous()
        return cm

    def host_lists(self):
        """(rows int64[S, K], counts int64[S, K]) on the host (tests, the
        multi-rank slot index)."""
        d = self.cache_dense.cpu().numpy().astype(np.int64)
        c = self.cache_cnt.cpu().numpy().astype(np.int64)
        rows = np.where(d >= 0, self.view.rows[np.maximum(d, 0)].astype(np.int64) if self.view.D else 0, 0)
        return rows, c

    def row_counts_for(self, ids: Sequence[int]) -> np.ndarray:
        """int32[S, P]: each listed row's count in every local shard (0 absent)."""
        import torch
        P, S = len(ids), self.S
        if not P or not S:
            return np.zeros((S, P), np.int32)
        dev = self.view.device
        d = self.view.dense_many(np.asarray(ids, dtype=np.uint64)).astype(np.int32)
        t_dense = torch.from_numpy(np.tile(d, S)).to(dev)
        t_shard = torch.arange(S, dtype=torch.int32, device=dev).repeat_interleave(P)
        return self._counts(t_shard, t_dense).view(S, P).cpu().numpy()

    # ------------------------------------------------------------ cache-only TopN
    def nosrc_phase1(self, ns: Sequence[int], thresholds: Sequence[int]):
        """Per query the per-shard fill phase of fragment.top (the first n
        cache entries at or above the threshold; the walk stops once its heap
        holds n rows) summed by row -> (query, dense, count) candidate tensors."""
        import torch
        dev = self.view.device
        Q, D = len(ns), self.view.D
        qs, ds, cs = [], [], []
        for q0 in range(0, Q, NOSRC_CHUNK):
            q1 = min(Q, q0 + NOSRC_CHUNK)
            nn = [int(n) for n in ns[q0:q1]]
            nmax = self.K if any(n == 0 for n in nn) else min(self.K, max(nn))
            if not nmax or not D:
                continue
            lim = torch.tensor([n if n else self.K for n in nn], dtype=torch.int64).to(dev)
            mt = torch.tensor([max(1, int(t)) for t in thresholds[q0:q1]], dtype=torch.int32).to(dev)
            cnt = self.cache_cnt[:, :nmax]
            dn = self.cache_dense[:, :nmax]
            # accumulate over the candidate rows only (the union of the shards'
            # first nmax cache entries), not a dense [queries x D] row space
            u, inv = torch.unique(dn.clamp(min=-1), return_inverse=True)
            U = int(u.numel())
            k = torch.arange(nmax, device=dev)
            take = (k[None, None, :] < lim[:, None, None]) & (cnt[None] >= mt[:, None, None]) & (dn[None] >= 0)
            vals = torch.where(take, cnt[None], torch.zeros((), dtype=torch.int32, device=dev))
            acc = torch.zeros((q1 - q0, U), dtype=torch.int32, device=dev)
            acc.scatter_add_(1, inv.reshape(1, -1).expand(q1 - q0, -1), vals.reshape(q1 - q0, -1))
            nz = torch.nonzero(acc > 0)
            qs.append(nz[:, 0] + q0)
            ds.append(u[nz[:, 1]].to(torch.int64))
            cs.append(acc[nz[:, 0], nz[:, 1]].to(torch.int64))
        if not qs:
            z = torch.zeros(0, dtype=torch.int64, device=dev)
            return z, z, z
        return torch.cat(qs), torch.cat(ds), torch.cat(cs)

    def recount(self, pq, pdense, thresholds: Sequence[int]):
        """ids= re-count without src: per (query, dense row) the sum over the
        local shards of the row's count where it reaches the query's threshold.
        A row asked for by several queries of the batch with one threshold is
        counted once (the per-shard counts do not depend on the query)."""
        import torch
        dev = self.view.device
        P = int(pdense.numel())
        out = torch.zeros(P, dtype=torch.int64, device=dev)
        if P and self.S:
            th = torch.tensor([max(1, int(t)) for t in thresholds], dtype=torch.int64).to(dev)[pq]
            key = (pdense.to(torch.int64) << 32) | th
            uk, inv = torch.unique(key, return_inverse=True)
            ud = (uk >> 32).to(torch.int32).contiguous()
            ut = (uk & 0xFFFFFFFF).to(torch.int32).contiguous()
            if self.M == 1:
                res = torch.zeros(int(uk.numel()), dtype=torch.int64, device=dev)
                kernels().row_counts_sum(self.view.viewdev_tensor(), self.S, ud, ut, res)
            else:   # the threshold applies to a fragment's count, summed over its sub-shards
                cm = self._count_matrix(ud)
                res = torch.where(cm >= ut.clamp(min=1)[:, None], cm, torch.zeros_like(cm)).sum(dim=1)
            out = res[inv]
        return out

    def topn_nosrc(self, ns: Sequence[int], thresholds: Sequence[int], comm=None,
                   space: Optional[np.ndarray] = None, defer: bool = False):
        """Whole TopN(field, n) calls (both phases, trimmed) for a batch.
        ``comm`` (parallel/collectives.Comm) spans the ranks of a node; the
        candidates then travel in ``space``, the sorted union of every rank's
        row ids (identical on all ranks): each rank's phase-1 keys are
        all-gathered and unioned, the ids= re-count is all-reduced (left in
        flight with ``defer``: a pending result, parallel/collectives.Pending)."""
        import torch

        from pilosa_amd.parallel.collectives import Pending

        from .topn_index import finish_batch_dev
        Q = len(ns)
        if Q == 0:
            return []
        ns, thresholds = clamp_topn_params(ns, thresholds)
        # the fused kernels total int32 counts: the node's columns (every device
        # sub-shard of every fragment, 2^20 each) must stay below 2^31
        if comm is None and self.view.D and self.view.S < 2048:
            got = self._topn_nosrc_fused(ns, thresholds)
            return got if got is not None else self._topn_nosrc_dense(ns, thresholds)
        pq, pd, _ = self.nosrc_phase1(ns, thresholds)
        if comm is None:
            out = self.recount(pq, pd, thresholds)
            return finish_batch_dev(self.view.rows, Q, pq, pd, out, ns)
        dev = self.view.device
        sp = torch.from_numpy(np.ascontiguousarray(space, dtype=np.uint64).view(np.int64)).to(dev)
        A = max(int(sp.numel()), 1)
        acc = torch.searchsorted(sp, rows_dev(self.view)[pd]) if pd.numel() else pd
        keys = comm.union(pq * A + acc, tag="topn_nosrc")
        pq, pa = keys // A, keys % A
        local = dense_dev(self.view, sp[pa]) if pa.numel() else pa.to(torch.int32)
        out = self.recount(pq, local.clamp(min=-1), thresholds)
        sp_h = np.asarray(space, dtype=np.uint64)
        pend = Pending(comm, comm.all_reduce_async(out), lambda: finish_batch_dev(sp_h, Q, pq, pa, out, ns), keep=out)
        return pend if defer else pend.result()

    def _candidates(self, nmax: int):
        """(u, inv) = torch.unique of the first ``nmax`` ranks of every shard:
        the candidate rows of a cache-only phase 1 (dense ids, -1 = empty) and
        each rank's candidate index.  A property of the rank caches, memoised
        per prefix length (this object is rebuilt when the caches change)."""
        import torch
        memo = self.__dict__.setdefault("_cand", {})
        got = memo.get(nmax)
        if got is None:
            u, inv = torch.unique(self.cache_dense[:, :nmax].clamp(min=-1), return_inverse=True)
            got = (u, inv.reshape(-1))
            memo[nmax] = got
        return got

    def _fused_memo(self, nmax: int):
        """(u int32[U], inv int32[S*nmax], cm int32[U, S]) for a prefix length:
        the candidate rows, each rank's candidate index and every candidate's
        count in every shard.  Fixed for this object (rebuilt when the view's
        generation moves), so a batch pays none of it after the first."""
        import torch
        memo = self.__dict__.setdefault("_fused", {})
        got = memo.get(nmax)
        if got is None:
            # a longer prefix's memo serves too (its candidates are a superset;
            # the member kernel stops at this batch's ranks)
            longer = [k for k, v in memo.items() if k > nmax and v is not False]
            if longer:
                return memo[min(longer)]
            u, inv = self._candidates(nmax)
            U = int(u.numel())
            if U * self.view.S > FUSED_MAX_CELLS:
                got = False
            else:
                u32 = u.to(torch.int32).contiguous()
                got = (u32, inv.to(torch.int32).contiguous(), self._count_matrix(u32))
                if self.view.device.type == "cuda":
                    # built on this batch's stream; other batches' streams read it
                    torch.cuda.current_stream(self.view.device).synchronize()
            memo[nmax] = got
        return got

    def _native_fused(self, memo):
        """The native request object (kernels/binding.cpp CacheTopN) over a
        fused memo, made once per memo: it owns its streams and pinned
        buffers and runs a batch without the interpreter between the H2D and
        the decoded answers.  None off the GPU or without the extension."""
        import torch
        if self.view.device.type != "cuda":
            return None
        u32, inv32, cm = memo
        stride = int(inv32.numel()) // max(self.S, 1)
        nat = self.__dict__.setdefault("_nat", {})
        got = nat.get(stride)
        if got is None:
            k = kernels()
            if not hasattr(k, "CacheTopN"):
                return None
            self._ready.synchronize()   # the rank caches' build, once
            rows = torch.from_numpy(np.ascontiguousarray(self.view.rows, dtype=np.uint64).view(np.int64))
            got = nat[stride] = k.CacheTopN(self.cache_cnt, inv32, u32, cm, stride, rows)
        return got

    # ------------------------------------------------------------ mesh (node-wide) cache-only batches
    def local_nmax(self, nreq: int) -> int:
        """This rank's cache prefix for a batch whose largest n is ``nreq``
        (0: some call takes every cached row)."""
        return self.K if nreq == 0 else min(self.K, int(nreq))

    def local_candidate_rows(self, nreq: int) -> np.ndarray:
        """Sorted row ids of every row in the first local_nmax(nreq) ranks of
        any local shard: this rank's share of the node candidate space."""
        nmax = self.local_nmax(nreq)
        if not nmax or not self.S:
            return np.zeros(0, np.uint64)
        u, _ = self._candidates(nmax)
        d = u[u >= 0].cpu().numpy().astype(np.int64)
        return np.asarray(self.view.rows[d], dtype=np.uint64) if len(d) else np.zeros(0, np.uint64)

    def node_candidates(self, nreq: int, space: np.ndarray) -> "NodeCandidates":
        """The local tensors of a mesh cache-only batch over the node
        candidate space ``space`` (sorted union of every rank's
        local_candidate_rows(nmax), identical on all ranks): each local rank
        slot's node index and each node candidate's count per local fragment
        (0 where this rank does not hold the row)."""
        import torch
        dev = self.view.device
        U = len(space)
        nmax = self.local_nmax(nreq)
        if not nmax or not self.S:
            return NodeCandidates(space, 0, torch.zeros(0, dtype=torch.int32, device=dev),
                                  torch.zeros((U, self.S), dtype=torch.int32, device=dev),
                                  torch.arange(U, dtype=torch.int32, device=dev))
        u, inv = self._candidates(nmax)
        u_h = u.cpu().numpy().astype(np.int64)
        present = u_h >= 0
        node_of_u = np.zeros(len(u_h), np.int64)
        if present.any():
            node_of_u[present] = np.searchsorted(space, self.view.rows[u_h[present]])
        inv_node = torch.from_numpy(node_of_u).to(dev)[inv].to(torch.int32).contiguous()
        cm = torch.zeros((U, self.S), dtype=torch.int32, device=dev)
        if present.any() and self.S:
            loc = self._count_matrix(torch.from_numpy(u_h[present].astype(np.int32)).to(dev))
            cm[torch.from_numpy(node_of_u[present]).to(dev)] = loc
        return NodeCandidates(space, nmax, inv_node, cm, torch.arange(U, dtype=torch.int32, device=dev))

    def topn_nosrc_mesh(self, ns: Sequence[int], thresholds: Sequence[int], comm, cand: "NodeCandidates",
                        defer: bool = False):
        """Cache-only TopN batch across the ranks of a node in ONE collective
        (:func:`mesh_cache_batch` with this rank's caches)."""
        return mesh_cache_batch(self, ns, thresholds, comm, cand, len(cand.space), defer=defer)

    def _topn_nosrc_fused(self, ns: Sequence[int], thresholds: Sequence[int]) -> Optional[List[List[Pair]]]:
        """Cache-only TopN batch in three hand-written kernels
        (kernels/topn_kernels.hip topn_cache_*): membership of every query's
        cache prefixes, one total per (distinct threshold, candidate) from the
        memoised count matrix, and a per-query LDS bitonic top-n.  One H2D of
        the batch parameters, one D2H of the Q x n keys.  None when the
        candidate set is too large for it (the torch path then runs)."""
        import torch
        Q = len(ns)
        nn = [int(n) for n in ns]
        nmax = self.K if any(n == 0 for n in nn) else min(self.K, prefix_bucket(max(nn)))
        if not nmax:
            return [[] for _ in range(Q)]
        dev = self.view.device
        if dev.type != "cuda":
            return self._topn_nosrc_fused_on(ns, nn, nmax, thresholds, None)
        # the memo (candidate x shard count matrix) reads the arena: build it on
        # the arena's own stream, where in-place arena writes (update_rows,
        # apply_deltas_multi, grow_segment) are ordered, and wait for it before
        # any side stream reads it.  Later batches find it built.
        memo = self._fused_memo(nmax)
        if memo is False:
            return None
        nat = self._native_fused(memo) if NATIVE_FUSED else None
        if nat is not None:
            got = nat.run(nn, thresholds, nmax)
            return None if got is None else pair_arrays_split(*got)
        lane = _lane_take(dev)
        if not SIDE_STREAM:
            lane.run_stream = torch.cuda.current_stream(dev)
            res = self._topn_nosrc_fused_on(ns, nn, nmax, thresholds, lane)
        else:
            lane.run_stream = lane.stream
            # a serving mix's TopN batch does not queue behind the Count batches
            # of other requests on the default stream, nor behind another
            # request's TopN batch
            lane.stream.wait_event(self._ready)
            with torch.cuda.stream(lane.stream):
                res = self._topn_nosrc_fused_on(ns, nn, nmax, thresholds, lane)
        _lane_give(dev, lane)   # not after an error: its copies may still be in flight
        return res

    def _topn_nosrc_fused_on(self, ns, nn, nmax, thresholds, lane):
        import torch
        Q = len(ns)
        memo = self._fused_memo(nmax)
        if memo is False:
            return None
        u32, inv32, cm = memo
        stride = int(inv32.numel()) // max(self.S, 1)   # the memo's prefix length (>= nmax)
        U = int(u32.numel())
        dev = self.view.device
        ths = [max(1, int(t)) for t in thresholds]
        uniq_t = sorted(set(ths))
        KK = min(U, max(nn)) if all(nn) else U
        pin = lane.pinned_i32(4 * Q + len(uniq_t)) if lane is not None else None
        prm = pin.numpy() if pin is not None else np.empty(4 * Q + len(uniq_t), np.int32)
        prm[:Q] = [n if n else self.K for n in nn]
        prm[Q:2 * Q] = ths
        tix = {t: i for i, t in enumerate(uniq_t)}
        prm[2 * Q:3 * Q] = [tix[t] for t in ths]
        prm[3 * Q:4 * Q] = [n if n else KK for n in nn]
        prm[4 * Q:] = uniq_t
        T = len(uniq_t)
        if lane is not None:
            prm_d = lane.buf("prm", len(prm), torch.int32)
            prm_d.copy_(pin, non_blocking=True)
            member = lane.buf("member", Q * U, torch.uint8).view(Q, U)   # cleared by the launcher
            tot = lane.buf("tot", T * U, torch.int64).view(T, U)
            out = lane.buf("out", Q * (KK + 1), torch.int64).view(Q, KK + 1)
        else:
            prm_d = torch.from_numpy(prm).to(dev)
            member = torch.empty((Q, U), dtype=torch.uint8, device=dev)   # cleared by the launcher
            tot = torch.empty((T, U), dtype=torch.int64, device=dev)
            out = torch.empty((Q, KK + 1), dtype=torch.int64, device=dev)
        kernels().topn_cache_batch(self.cache_cnt, stride, inv32, u32, cm, prm_d, Q, T, member, tot, out, nmax)
        if lane is not None:
            # answers to the lane's pinned buffer, then wait for this stream only
            hb = lane.buf("out_h", out.numel(), torch.int64, pinned=True)
            hb.copy_(out.view(-1), non_blocking=True)
            lane.run_stream.synchronize()   # the stream this batch ran on (no current-stream lookup)
            h = hb.numpy().reshape(Q, KK + 1)
        else:
            h = out.cpu().numpy()
        lens = h[:, 0]
        if (lens < 0).any():     # a query with more members than one workgroup sorts
            return None
        # every query's kept keys end to end, decoded in one pass (keys ->
        # dense rows -> ids, counts), then split into per-query views: fewer
        # numpy calls than decoding query by query, and no work on the
        # padding of short answers (a [Q, max n] decode measured slower)
        ln = lens.tolist()
        keys = np.concatenate([h[q, 1:1 + n] for q, n in enumerate(ln)]) if Q else np.zeros(0, np.int64)
        ids = np.asarray(self.view.rows, dtype=np.uint64)[0xFFFFFFFF - (keys & 0xFFFFFFFF)] if len(keys) else \
            np.zeros(0, np.uint64)
        cnt = keys >> 32
        res, o = [], 0
        for n in ln:
            res.append(pair_array(ids[o:o + n], cnt[o:o + n]))
            o += n
        return res

    def _topn_nosrc_dense(self, ns: Sequence[int], thresholds: Sequence[int]) -> List[List[Pair]]:
        """Single-rank cache-only TopN batch without a host round trip until
        the end: phase 1 accumulates every query's cache prefixes into a
        [Q, candidates] matrix, phase 2 re-counts each candidate row once per
        distinct threshold (row_counts_sum), and one top-k over the composite
        key (count desc, id asc) trims each query to n; only the Q x n pairs
        are copied to the host.  Same answers as nosrc_phase1 + recount +
        finish_batch_dev, with no data-dependent shapes (no syncs) on the way."""
        import torch
        dev = self.view.device
        Q = len(ns)
        nn = [int(n) for n in ns]
        nmax = self.K if any(n == 0 for n in nn) else min(self.K, max(nn))
        if not nmax:
            return [[] for _ in range(Q)]
        u, inv = self._candidates(nmax)
        U = int(u.numel())
        ths = [max(1, int(t)) for t in thresholds]
        uniq_t = sorted(set(ths))
        lim_mt = torch.tensor([[n if n else self.K for n in nn], ths], dtype=torch.int64).to(dev, non_blocking=True)
        lim, mt = lim_mt[0], lim_mt[1].to(torch.int32)
        cnt = self.cache_cnt[:, :nmax]
        dn = self.cache_dense[:, :nmax]
        k = torch.arange(nmax, device=dev)
        take = (k[None, None, :] < lim[:, None, None]) & (cnt[None] >= mt[:, None, None]) & (dn[None] >= 0)
        vals = torch.where(take, cnt[None], torch.zeros((), dtype=torch.int32, device=dev))
        acc = torch.zeros((Q, U), dtype=torch.int32, device=dev)
        acc.scatter_add_(1, inv.reshape(1, -1).expand(Q, -1), vals.reshape(Q, -1))
        # phase 2: every candidate row re-counted once per distinct threshold
        ud = u.clamp(min=0).to(torch.int32).contiguous()
        res = torch.zeros((len(uniq_t), U), dtype=torch.int64, device=dev)
        cm = self._count_matrix(ud) if self.M > 1 else None   # per fragment over its sub-shards
        for ti, t in enumerate(uniq_t):
            if cm is not None:
                res[ti] = torch.where(cm >= t, cm, torch.zeros_like(cm)).sum(dim=1)
                continue
            kernels().row_counts_sum(self.view.viewdev_tensor(), self.S, ud,
                                     torch.full((U,), t, dtype=torch.int32, device=dev), res[ti])
        if len(uniq_t) == 1:
            tot = res[0][None, :].expand(Q, -1)
        else:
            tsel = torch.tensor([uniq_t.index(t) for t in ths], dtype=torch.int64).to(dev)
            tot = res[tsel]
        live = (acc > 0) & (u >= 0)[None, :]
        score = torch.where(live, tot, torch.zeros((), dtype=torch.int64, device=dev))
        # composite key: count desc, then dense (= row id) asc
        key = (score << 32) | (0xFFFFFFFF - u.clamp(min=0).to(torch.int64))[None, :]
        key = torch.where(score > 0, key, torch.full((), -1, dtype=torch.int64, device=dev))
        kk = min(U, max(nn)) if all(nn) else U   # a query keeps up to n rows (n may exceed the cache width)
        top = torch.topk(key, kk, dim=1, sorted=True).values
        h = top.cpu().numpy()
        rows = self.view.rows
        out: List[List[Pair]] = []
        for q in range(Q):
            r = h[q]
            r = r[r >= 0]
            if nn[q]:
                r = r[:nn[q]]
            d = (0xFFFFFFFF - (r & 0xFFFFFFFF)).astype(np.int64)
            ids = rows[d] if len(d) else np.zeros(0, np.uint64)
            out.append(pair_array(ids, r >> 32))
        return out

    def shard_pairs_nosrc(self, n: int, threshold: int, ids: Optional[Sequence[int]] = None) -> List[Pair]:
        """One cache-only TopN call as the executor's map step sees it: phase 1
        (untrimmed per-shard results summed by row) or the ids= re-count."""
        import torch
        dev = self.view.device
        if ids is None:
            pq, pd, pc = self.nosrc_phase1([n], [threshold])
        else:
            want = np.unique(np.asarray(list(ids), dtype=np.uint64))
            d = self.view.dense_many(want)
            d = d[d >= 0]
            pd = torch.from_numpy(d.astype(np.int64)).to(dev)
            pq = torch.zeros_like(pd)
            pc = self.recount(pq, pd, [threshold])
        keep = pc > 0
        d_h = pd[keep].cpu().numpy()
        c_h = pc[keep].cpu().numpy()
        rows = self.view.rows[d_h] if len(d_h) else np.zeros(0, np.uint64)
        return pairs_from_arrays(rows, c_h)
