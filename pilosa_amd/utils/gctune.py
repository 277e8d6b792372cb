"""Cyclic-GC policy for a long-running index process.

A node holds millions of long-lived Python objects (fragments, views, rank
caches, translate maps) and every query allocates short-lived ones (a
16-call TopN request builds thousands of Pair objects).  With CPython's
default thresholds (700, 10, 10) the allocation churn triggers a collection
every 700 objects and, now and then, a full one that walks the whole heap:
on the 954-shard bench index the collector took 0.51 s of a 0.65 s run of
cache-only TopN requests (706 collections, profiles/r04_k/).

The policy here (what the Go runtime gets for free from a non-moving,
concurrent collector):
  * objects that are alive after start-up or a warm-up are moved out of the
    collector's generations (``gc.freeze``), so collections walk only what
    was allocated since;
  * gen-0 collections run every ``THRESHOLD0`` net allocations instead of 700
    (10k: a collection of that many young objects stays well under a
    millisecond, so it does not show in request tail latency);
  * :class:`Refreezer` re-freezes survivors periodically (after a young
    collection, so short-lived cycles are reclaimed first) and runs one full
    unfrozen collection every ``full_every`` seconds, so cyclic garbage that
    was frozen is still reclaimed eventually.
"""
from __future__ import annotations

import gc
import os
import time

THRESHOLD0 = 10_000


def enabled() -> bool:
    """``PILOSA_GC_FREEZE=0`` turns the policy off (the test suite does: its
    process opens and drops hundreds of servers)."""
    return os.environ.get("PILOSA_GC_FREEZE", "1") != "0"


def configure(threshold0: int = THRESHOLD0) -> None:
    g0, g1, g2 = gc.get_threshold()
    if g0 < threshold0:
        gc.set_threshold(threshold0, max(g1, 10), max(g2, 10))


def freeze_long_lived() -> int:
    """Collect, then move every surviving object to the permanent generation.
    Returns how many objects are frozen."""
    gc.collect()
    gc.freeze()
    return gc.get_freeze_count()


class Refreezer:
    """Call :meth:`tick` from a periodic loop (the server's runtime loop)."""

    def __init__(self, every: float = 60.0, full_every: float = 1800.0):
        self.every = every
        self.full_every = full_every
        self._last = time.monotonic()
        self._last_full = self._last

    def tick(self, now: float = None) -> str:
        now = time.monotonic() if now is None else now
        if now - self._last_full >= self.full_every:
            gc.unfreeze()
            gc.collect()
            gc.freeze()
            self._last = self._last_full = now
            return "full"
        if now - self._last >= self.every:
            gc.collect(1)   # young generations only: short-lived cycles go first
            gc.freeze()
            self._last = now
            return "freeze"
        return ""
