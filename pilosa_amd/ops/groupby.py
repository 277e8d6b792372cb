"""GroupBy count matrices on the device (kernels/bitgemm.hip).

Reference: executor.go:3060-3230 (``groupByIterator``) walks row combinations
per shard and intersects them one pair at a time.  For two grouped fields the
whole result is the count matrix C[ra][rb] = |A_ra ∩ B_rb| summed over the
shards -- a GEMM over bit positions.  Rows are densified per shard chunk into
u64 bit rows (``densify``) and multiplied on the matrix cores with
``v_mfma_i32_32x32x32_i8``: mode 2 gives every wave a 64x64 tile and expands
bits to bytes with 24-bit multiplies (826-846 T bit-ops/s at 128-256 rows vs
469-490 for the VALU AND+popcount mode 0; mode 1, a byte-table expansion
through LDS, is kept as the measured negative result at ~216).  The emitting
of (ra, rb, count) groups in lexicographic order with ``previous``/``limit``
stays on the host.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import numpy as np

from .device import DeviceView, kernels

WORDS_PER_SHARD = 1 << 14        # 2^20 bits
MODE_VALU, MODE_MFMA_TABLE, MODE_MFMA, MODE_MFMA_SKINNY, MODE_MFMA_KSLICE = 0, 1, 2, 3, 4
# below this many rows on either side the 128x128 MFMA tiles run mostly empty
# and the VALU kernel is faster (profiles/r01_groupby/bitgemm_bench.log)
MFMA_MIN_ROWS = 96


def _vd(view: DeviceView):
    import torch
    return torch.from_numpy(np.frombuffer(view.viewdev().tobytes(), dtype=np.uint8).copy())


def pair_count_matrix(va: DeviceView, rows_a: Sequence[int], vb: DeviceView, rows_b: Sequence[int],
                      mode: Optional[int] = None, chunk_bytes: int = 1 << 30, blocks: int = 2048,
                      filt: Optional[Tuple[DeviceView, int]] = None) -> np.ndarray:
    """int64[len(rows_a), len(rows_b)]: |row_a ∩ row_b (∩ filter row)| over
    all local shards.  ``filt`` = (view, row id) intersected into A."""
    import torch

    ext = kernels()
    Ra, Rb = len(rows_a), len(rows_b)
    if mode is None:
        mode = MODE_MFMA if min(Ra, Rb) >= MFMA_MIN_ROWS else MODE_VALU
    out = np.zeros((Ra, Rb), np.int64)
    if Ra == 0 or Rb == 0 or va.S == 0:
        return out
    if va.S != vb.S:
        raise ValueError("views must share the local shard list")
    dev = va.device
    da = torch.from_numpy(va.dense_many(np.asarray(rows_a, np.uint64))).to(dev)
    db = torch.from_numpy(vb.dense_many(np.asarray(rows_b, np.uint64))).to(dev)
    row_bytes = WORDS_PER_SHARD * 8
    chunk = max(1, min(va.S, 2047, chunk_bytes // ((Ra + Rb) * row_bytes)))
    acc = torch.zeros((Ra, Rb), dtype=torch.int64, device=dev)
    vda, vdb = _vd(va), _vd(vb)
    bt = 128 if mode == MODE_MFMA else 64
    tiles = math.ceil(Ra / bt) * math.ceil(Rb / bt)
    fv = fd = None
    if filt is not None:
        fv = _vd(filt[0])
        fd = torch.from_numpy(filt[0].dense_many(np.asarray([filt[1]], np.uint64))).to(dev)
    for s0 in range(0, va.S, chunk):
        s1 = min(va.S, s0 + chunk)
        kw = (s1 - s0) * WORDS_PER_SHARD
        A = torch.empty(Ra * kw, dtype=torch.int64, device=dev)
        B = torch.empty(Rb * kw, dtype=torch.int64, device=dev)
        ext.densify(vda, da, s0, s1, A)
        ext.densify(vdb, db, s0, s1, B)
        if fv is not None:
            F = torch.empty(kw, dtype=torch.int64, device=dev)
            ext.densify(fv, fd, s0, s1, F)
            A.view(Ra, kw).bitwise_and_(F.view(1, kw))
            del F
        C = torch.zeros(Ra * Rb, dtype=torch.int32, device=dev)
        splits = max(1, min(kw // 8, math.ceil(blocks / tiles)))
        ext.bitgemm(A, B, Ra, Rb, kw, splits, mode, C)
        acc += C.view(Ra, Rb).to(torch.int64)
        del A, B
    return acc.cpu().numpy()


def emit_groups(cand_a: Sequence[int], cand_b: Sequence[int], counts: np.ndarray, prev: Optional[Tuple[int, ...]],
                limit: int):
    """(ra, rb, count) with count > 0 in lexicographic (ra, rb) order, keys
    strictly after ``prev``, at most ``limit`` (executor.go:1241-1442 paging)."""
    out = []
    a = np.asarray(cand_a, dtype=np.int64)
    b = np.asarray(cand_b, dtype=np.int64)
    for i in range(len(a)):
        ra = int(a[i])
        if prev is not None and ra < prev[0]:
            continue
        nz = np.flatnonzero(counts[i] > 0)
        if prev is not None and ra == prev[0]:
            nz = nz[b[nz] > prev[1]]
        for k in nz.tolist():
            out.append((ra, int(b[k]), int(counts[i, k])))
            if len(out) >= limit:
                return out
    return out
