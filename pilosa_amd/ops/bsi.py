"""Batched BSI Sum as a bit-plane matrix product on the matrix cores.

Reference: fragment.go:1109-1141 (``sum``): per shard, for a filter F,

    count = |F & exists|
    sum   = sum_i 2^i (|F & exists & ~sign & bit_i| - |F & exists & sign & bit_i|)

The per-filter kernel (bitmap_kernels.hip bsi_sum) streams every bit plane
once per filter.  For a batch of Q filters the same numbers are one count
matrix C = F x P^T over all 2^20 * S bit positions, where the rows of P are the
filter-independent planes

    P_i = exists & ~sign & bit_i,   N_i = exists & sign & bit_i,   exists

(2*depth + 1 rows, built once per view generation and cached) and the rows of
F are the filters evaluated densely (expr_dense, one launch for the batch).
The product runs on ``bitgemm`` (kernels/bitgemm.hip) in MODE_MFMA_KSLICE:
a 32x64 output tile per workgroup whose 4 waves split the k-steps, every
32-bit k-step one ``v_mfma_i32_32x32x32_i8`` per 32x32 half, so the planes are
read once for the whole batch instead of once per filter.  32 Row() filters
over 1B columns (profiles/r02_bsi/): per-filter kernel 6.75 ms; matrix path
densify 1.2 ms + bitgemm 4.1 ms (64x64-tile MFMA 5.3 ms, 128x128 15.4 ms,
VALU tiles 8.4 ms).  Below BSI_MATRIX_MIN filters the per-filter kernel wins
(the GEMM streams all 2*depth+1 planes regardless of Q).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .device import CompileError, DeviceView, GpuEngine, Leaf, Op, compile_expr, kernels, pack_programs
from .groupby import MODE_MFMA, MODE_MFMA_KSLICE, MODE_MFMA_SKINNY, MODE_VALU, WORDS_PER_SHARD, _vd

# batches of at least this many filters take the matrix path
BSI_MATRIX_MIN = 32


class BsiPlanes:
    """Filter-independent planes [P_0..P_{d-1}, N_0..N_{d-1}, exists] of one
    BSI view, int64[2d+1, S*16384], cached per (view, generation, depth)."""

    def __init__(self):
        self._cache: Dict[Tuple[int, int, int], Tuple[object, object]] = {}

    def get(self, bv: DeviceView, depth: int):
        import torch

        key = (id(bv), bv.generation, depth)
        hit = self._cache.get(key)
        if hit is not None and hit[0] is bv:
            return hit[1]
        ext = kernels()
        S = bv.S
        kw = S * WORDS_PER_SHARD
        dense = np.full(depth + 2, -1, np.int64)
        dense[0], dense[1] = bv.dense(0), bv.dense(1)
        for i in range(depth):
            dense[2 + i] = bv.dense(2 + i)
        rows = torch.from_numpy(dense).to(bv.device)
        raw = torch.empty((depth + 2) * kw, dtype=torch.int64, device=bv.device)
        if S:
            ext.densify(_vd(bv), rows, 0, S, raw)
        raw = raw.view(depth + 2, kw)
        ex, sg = raw[0], raw[1]
        planes = torch.empty((2 * depth + 1, kw), dtype=torch.int64, device=bv.device)
        pos = ex & ~sg
        neg = ex & sg
        torch.bitwise_and(raw[2:], pos.unsqueeze(0), out=planes[:depth])
        torch.bitwise_and(raw[2:], neg.unsqueeze(0), out=planes[depth:2 * depth])
        planes[2 * depth].copy_(ex)
        del raw, pos, neg
        self._cache.clear()  # one BSI view's planes at a time (several GB at 1B columns)
        self._cache[key] = (bv, planes)
        return planes


_PLANES = BsiPlanes()


def bsi_sum_matrix(engine: GpuEngine, filters: Sequence[Optional[object]], bv: DeviceView, depth: int,
                   mode: Optional[int] = None, splits: int = 2048):
    """(sum int64[Q], count int64[Q]) for a batch of filters (None = all
    columns), base-relative like bsi_sum_async."""
    import torch

    ext = kernels()
    Q = len(filters)
    dev = bv.device
    out_s = torch.zeros(Q, dtype=torch.int64, device=dev)
    out_c = torch.zeros(Q, dtype=torch.int64, device=dev)
    S = bv.S
    if not Q or not S or bv.dense(0) < 0:
        return out_s, out_c
    kw = S * WORDS_PER_SHARD
    planes = _PLANES.get(bv, depth)
    # dense filters: one expr_dense launch for the batch, rows of F in place
    F = torch.empty(Q * kw, dtype=torch.int64, device=dev)
    live = [q for q, f in enumerate(filters) if f is not None]
    leaf_view = filters[live[0]].view if live and isinstance(filters[live[0]], Leaf) else None
    if live and leaf_view is not None and leaf_view.S == S and \
            all(isinstance(filters[q], Leaf) and filters[q].view is leaf_view for q in live):
        # plain Row() filters of one view: densify the rows directly (one launch)
        dense = np.full(Q, -1, np.int64)
        for q in live:
            dense[q] = leaf_view.dense(filters[q].row)
        ext.densify(_vd(leaf_view), torch.from_numpy(dense).to(dev), 0, S, F)
        live = []
    if live:
        view_index: Dict[int, int] = {}
        views: Dict[int, DeviceView] = {}

        def collect(node):
            if isinstance(node, Leaf):
                views[id(node.view)] = node.view
            elif isinstance(node, Op):
                for a in node.args:
                    collect(a)
        comp = []
        for q in live:
            collect(filters[q])
            comp.append(compile_expr(filters[q], view_index))
        ordered = [None] * len(view_index)
        for vid, slot in view_index.items():
            ordered[slot] = views[vid]
        for v in ordered:
            if v.S != S:
                raise CompileError("filter views must share the BSI view's shards")
        progs = pack_programs(comp)
        tp, tv = engine.upload_batch(progs, ordered)
        Fl = torch.empty(len(live) * kw, dtype=torch.int64, device=dev)
        meta = torch.empty(len(live) * S * 16, dtype=torch.int64, device=dev)
        ext.expr_dense(tp, tv, S, Fl.view(torch.int16), meta)
        if len(live) == Q:
            F = Fl
        else:
            F.view(Q, kw)[torch.tensor(live, device=dev)] = Fl.view(len(live), kw)
    for q, f in enumerate(filters):
        if f is None:
            F.view(Q, kw)[q].copy_(planes[2 * depth])  # all columns: the exists plane
    N = 2 * depth + 1
    if mode is None:
        mode = MODE_MFMA_KSLICE
    C = torch.zeros(Q * N, dtype=torch.int32, device=dev)
    if mode == MODE_MFMA_KSLICE:
        tiles = math.ceil(Q / 32) * math.ceil(N / 64)
    else:
        bt = 128 if mode == MODE_MFMA else 64
        tiles = math.ceil(Q / bt) * math.ceil(N / bt)
    sp = max(1, min(kw // 32, math.ceil(splits / tiles)))
    ext.bitgemm(F, planes.reshape(-1), Q, N, kw, sp, mode, C)
    C = C.view(Q, N).to(torch.int64)
    w = torch.pow(torch.full((depth,), 2, dtype=torch.int64, device=dev), torch.arange(depth, device=dev))
    out_s = ((C[:, :depth] - C[:, depth:2 * depth]) * w).sum(dim=1)
    out_c = C[:, 2 * depth]
    return out_s, out_c
