"""Shard width knob (reference: shardwidth/16.go .. 32.go build tags selected
by ``make SHARD_WIDTH=n``, Makefile:9-19; default exponent 20).

The exponent comes from ``PILOSA_SHARD_WIDTH`` (16..32) when the package is
first imported -- the equivalent of the reference's build tag: every process
of a cluster (and every tool that reads its data) must use the same value.
Fragments, rows, imports, placement and the file formats follow it.

The GPU kernels are specialised for 2^20-column device shards (16 containers
per row in the arena, ``kernels/``), so a node with another width answers
from the host roaring path (server.Server disables the GPU executor and says
so in its log).
"""
from __future__ import annotations

import os

DEFAULT_EXPONENT = 20
MIN_EXPONENT, MAX_EXPONENT = 16, 32
DEVICE_EXPONENT = 20


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


def device_supported() -> bool:
    """True when the GPU arena layout matches the shard width."""
    return EXPONENT == DEVICE_EXPONENT
