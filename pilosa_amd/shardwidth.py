"""Shard width knob (reference: shardwidth/16.go .. 32.go build tags selected
by ``make SHARD_WIDTH=n``, Makefile:9-19; default exponent 20).

The exponent comes from ``PILOSA_SHARD_WIDTH`` (16..32) when the package is
first imported -- the equivalent of the reference's build tag: every process
of a cluster (and every tool that reads its data) must use the same value.
Fragments, rows, imports, placement and the file formats follow it.

Device arenas (``ops/device.py``, ``kernels/``) keep 16 container slots per
row and 2^20-column device shards.  A narrower shard (exponent 16..19, 2^(e-16)
containers per row) maps onto them one to one: its containers fill the first
2^(e-16) slots of each row, container keys are translated at the host/device
boundary (``device_key`` / ``host_key``: the loader, build_arena, the write
replay, row results) and a shard's columns stay ``shard * ShardWidth + x``.
Wider shards (21..32) would need several device shards per shard; a node
with such a width answers from the host roaring path (server.Server disables
the GPU executor and says so in its log).
"""
from __future__ import annotations

import os

DEFAULT_EXPONENT = 20
MIN_EXPONENT, MAX_EXPONENT = 16, 32
DEVICE_EXPONENT = 20   # device shard width (16 container slots per row)


def _exponent() -> int:
    raw = os.environ.get("PILOSA_SHARD_WIDTH", str(DEFAULT_EXPONENT))
    try:
        e = int(raw)
    except ValueError:
        raise ValueError(f"PILOSA_SHARD_WIDTH must be an exponent in [{MIN_EXPONENT}, {MAX_EXPONENT}], got {raw!r}")
    if not MIN_EXPONENT <= e <= MAX_EXPONENT:
        raise ValueError(f"PILOSA_SHARD_WIDTH must be an exponent in [{MIN_EXPONENT}, {MAX_EXPONENT}], got {e}")
    return e


EXPONENT = _exponent()
SHARD_WIDTH = 1 << EXPONENT
CONTAINERS_PER_ROW = SHARD_WIDTH >> 16


KEY_SHIFT = EXPONENT - 16   # log2(containers per row)


def device_supported() -> bool:
    """True when the GPU arenas can hold this shard width (2^16..2^20)."""
    return MIN_EXPONENT <= EXPONENT <= DEVICE_EXPONENT


def device_key(k):
    """Host container key (row << KEY_SHIFT | j) -> arena key (row * 16 + j).
    Works on ints and uint64 numpy arrays."""
    if KEY_SHIFT == 4:
        return k
    return ((k >> KEY_SHIFT) << 4) | (k & (CONTAINERS_PER_ROW - 1))


def host_key(k):
    """Arena key (row * 16 + j, j < CONTAINERS_PER_ROW) -> host container key."""
    if KEY_SHIFT == 4:
        return k
    return ((k >> 4) << KEY_SHIFT) | (k & 15)
