"""Fragment files -> HBM container arena (resume path).

The reference opens every fragment by mmap + header walk + op-log replay
(fragment.go:311-456, roaring/roaring.go:1562-1653) and serves reads from
containers that alias the mapping.  Here the device arena is the read replica,
so a view's fragment files are parsed natively (native/arena_io.cpp
``FragmentLoader``) straight into the arena layout: the row directory, CSR
rowptr and packed container metadata are built on host threads, and the
payload is streamed shard-chunk by shard-chunk through two pinned staging
buffers on a copy stream (fill of chunk k+1 overlaps the H2D of chunk k).
No host ``Bitmap`` is created for any fragment without an op log.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from .device import DeviceView

# per-shard metadata slack and payload slack of patchable arenas (same as
# DeviceView.patchable)
META_SLACK, META_MIN_SLACK = 0.125, 16
PAYLOAD_SLACK, PAYLOAD_MIN_SLACK_U16 = 0.25, 8 << 20


def load_view(paths: Sequence[str], shards: Sequence[int], device, patchable: bool = True,
              nthreads: Optional[int] = None, chunk_bytes: int = 256 << 20,
              stats: Optional[Dict] = None, subs: Optional[Sequence[int]] = None) -> DeviceView:
    """Build a :class:`DeviceView` over ``shards`` from their fragment files
    (``""`` or a missing path = empty shard).  Above 2^20 columns per shard
    ``shards`` are device shard ids and ``subs[i]`` the sub-shard of
    ``paths[i]`` that arena shard i holds (pilosa_amd/shardwidth.py)."""
    import torch

    from pilosa_amd import _roaring

    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 8)
    device = torch.device(device)
    t0 = time.perf_counter()
    from pilosa_amd import shardwidth
    if shardwidth.WIDE and subs is None:
        raise ValueError(f"load_view: shard width 2^{shardwidth.EXPONENT} needs the sub-shard of every path")
    ld = _roaring.FragmentLoader([p or "" for p in paths], int(nthreads), shardwidth.KEY_SHIFT,
                                 [int(x) for x in subs] if shardwidth.WIDE else [])
    info = ld.scan()
    rows = ld.rows()
    t_scan = time.perf_counter()
    rowptr, sb, meta, cap, pb = ld.fill_index(META_SLACK if patchable else 0.0,
                                              META_MIN_SLACK if patchable else 0)
    t_index = time.perf_counter()
    S = len(paths)
    P = int(pb[-1])
    total = P + (max(PAYLOAD_MIN_SLACK_U16, int(P * PAYLOAD_SLACK)) if patchable else 0)
    total = max(total, 8)
    if device.type == "cuda":
        t_payload = torch.empty(total, dtype=torch.int16, device=device)
        if total > P:
            t_payload[P:].zero_()
        _stream_payload(ld, pb, t_payload, device, chunk_bytes)
    else:
        t_payload = torch.zeros(total, dtype=torch.int16)
        if S:
            ld.fill_payload(0, S, t_payload.numpy().view(np.uint16))
    t_pay = time.perf_counter()
    dv = DeviceView.from_host_index(rows, rowptr, sb, meta, t_payload, P, device, list(shards),
                                    cap=cap if patchable else None)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t_end = time.perf_counter()
    if stats is not None:
        stats.update({"files": S, "file_bytes": int(info["file_bytes"]), "containers": int(info["containers"]),
                      "replayed_shards": int(info["replayed"]), "payload_bytes": 2 * P, "rows": int(len(rows)),
                      "scan_s": round(t_scan - t0, 3), "index_s": round(t_index - t_scan, 3),
                      "payload_s": round(t_pay - t_index, 3), "upload_index_s": round(t_end - t_pay, 3),
                      "total_s": round(t_end - t0, 3)})
    return dv


def _stream_payload(ld, pb: np.ndarray, t_payload, device, chunk_bytes: int):
    """Chunked H2D of the payload through two pinned buffers."""
    import torch

    S = len(pb) - 1
    chunk = max(int(chunk_bytes) // 2, 4096)
    stream = torch.cuda.Stream(device)
    bufs = [None, None]
    events = [None, None]
    s, k = 0, 0
    while s < S:
        e = s + 1
        while e < S and int(pb[e + 1] - pb[s]) <= chunk:
            e += 1
        n = int(pb[e] - pb[s])
        if n == 0:
            ld.fill_payload(s, e, np.zeros(8, np.uint16))  # releases the (empty) mappings
            s = e
            continue
        slot = k & 1
        if events[slot] is not None:
            events[slot].synchronize()
        buf = bufs[slot]
        if buf is None or buf.numel() < n:
            buf = bufs[slot] = torch.empty(max(n, chunk), dtype=torch.int16, pin_memory=True)
        ld.fill_payload(s, e, buf.numpy().view(np.uint16))
        with torch.cuda.stream(stream):
            t_payload[int(pb[s]):int(pb[e])].copy_(buf[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        events[slot] = ev
        s, k = e, k + 1
    stream.synchronize()


def fragment_paths(view, shards: Sequence[int]) -> Tuple[list, list]:
    """(paths, fragments) of a holder view for ``shards`` ('' where absent)."""
    frags = [view.fragment(s) if view is not None else None for s in shards]
    return [f.path if f is not None else "" for f in frags], frags
