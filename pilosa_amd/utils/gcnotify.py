"""Garbage-collection notifications -> stats (reference: gcnotify/gcnotify.go,
gc.go: a counter per completed GC cycle)."""
from __future__ import annotations

import gc


class GCNotifier:
    def __init__(self, stats):
        self.stats = stats
        self.collections = 0
        self._cb = None

    def start(self):
        def cb(phase, info):
            if phase == "stop":
                self.collections += 1
                try:
                    self.stats.count("garbage_collection", 1)
                except Exception:  # noqa: BLE001
                    pass
        self._cb = cb
        gc.callbacks.append(cb)
        return self

    def stop(self):
        if self._cb is not None and self._cb in gc.callbacks:
            gc.callbacks.remove(self._cb)
        self._cb = None
