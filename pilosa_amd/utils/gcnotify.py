"""Garbage-collection notifications -> stats (reference: gcnotify/gcnotify.go,
gc.go: a counter per completed GC cycle).

The gc callback runs inside whatever allocation triggered the collection --
possibly while that thread holds the stats registry lock -- so it only bumps
plain integers; :meth:`GCNotifier.flush` moves them into the stats client from
an ordinary context (the server's runtime loop, or on demand)."""
from __future__ import annotations

import gc


class GCNotifier:
    def __init__(self, stats):
        self.stats = stats
        self.collections = 0
        self._flushed = 0
        self._cb = None

    def start(self):
        def cb(phase, info):
            if phase == "stop":
                self.collections += 1   # no locks, no allocation-heavy work here
        self._cb = cb
        gc.callbacks.append(cb)
        return self

    def flush(self) -> int:
        """Report the collections since the last flush as the
        ``garbage_collection`` counter; returns how many."""
        n = self.collections - self._flushed
        if n > 0:
            self._flushed += n
            try:
                self.stats.count("garbage_collection", n)
            except Exception:  # noqa: BLE001
                pass
        return n

    def stop(self):
        if self._cb is not None and self._cb in gc.callbacks:
            gc.callbacks.remove(self._cb)
        self._cb = None
        self.flush()
