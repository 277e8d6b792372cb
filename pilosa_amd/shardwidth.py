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
A wider shard (exponent 21..32) is split into ``DEVICE_SUBSHARDS`` =
2^(e-20) device sub-shards of 2^20 columns: host shard s becomes device
shards s*M .. s*M + M-1 (``device_shards``), container c of a row goes to
sub-shard c >> 4, arena slot c & 15.  Global columns then stay
``device_shard * 2^20 + x``, so every kernel, row result and per-shard count
works unchanged on device shard ids; the GPU executor maps host shards to
device shards at the arena boundary (ops/gpu_executor.py ``SubFragment``) and
the native file loader reads one sub-shard of a file per arena shard.
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

# device shards per shard (2^(e-20) above 2^20 columns, else 1), the arena's
# columns per device shard and its containers per row
DEVICE_SUBSHARDS = 1 << max(0, EXPONENT - DEVICE_EXPONENT)
WIDE = DEVICE_SUBSHARDS > 1
ARENA_WIDTH = min(SHARD_WIDTH, 1 << DEVICE_EXPONENT)
ARENA_CPR = ARENA_WIDTH >> 16


def device_supported() -> bool:
    """True when the GPU arenas can hold this shard width: 2^16..2^20 map one
    to one, wider shards as 2^(e-20) device sub-shards each."""
    return MIN_EXPONENT <= EXPONENT <= MAX_EXPONENT


def device_shards(shards):
    """Host shard ids -> the device shard ids of the arena (identity up to 2^20)."""
    if not WIDE:
        return [int(s) for s in shards]
    M = DEVICE_SUBSHARDS
    return [int(s) * M + i for s in shards for i in range(M)]


def device_key(k):
    """Host container key (row << KEY_SHIFT | j) -> arena key (row * 16 + j;
    above 2^20 columns j is the slot within the key's sub-shard, c & 15).
    Works on ints and uint64 numpy arrays."""
    if KEY_SHIFT == 4:
        return k
    return ((k >> KEY_SHIFT) << 4) | (k & (ARENA_CPR - 1))


def sub_of_key(k):
    """Device sub-shard of a host container key (0 up to 2^20 columns)."""
    return (k >> 4) & (DEVICE_SUBSHARDS - 1) if WIDE else 0 * k


def host_key(k, sub: int = 0):
    """Arena key (row * 16 + j, j < ARENA_CPR) of sub-shard ``sub`` -> host
    container key."""
    if KEY_SHIFT == 4:
        return k
    if WIDE:
        return ((k >> 4) << KEY_SHIFT) | (sub << 4) | (k & 15)
    return ((k >> 4) << KEY_SHIFT) | (k & 15)
