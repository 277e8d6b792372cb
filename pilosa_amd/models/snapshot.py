"""Background fragment snapshotting (reference: fragment.go:187-239
snapshotQueue, holder.go:160 newSnapshotQueue(100, 2)).

When a fragment's op log grows past MaxOpN the write path enqueues the
fragment instead of rewriting the file inline; a small pool of workers
performs the write -> fsync -> rename.  A full queue falls back to an inline
snapshot (back-pressure, as in the reference)."""
from __future__ import annotations

import queue
import threading


class SnapshotQueue:
    def __init__(self, depth: int = 100, workers: int = 2, logger=None):
        self.q: "queue.Queue" = queue.Queue(maxsize=depth)
        self.pending = set()
        self.mu = threading.Lock()
        self.logger = logger
        self.done = 0
        self._threads = [threading.Thread(target=self._run, name=f"snapshot-{i}", daemon=True)
                         for i in range(workers)]
        for t in self._threads:
            t.start()

    def enqueue(self, frag) -> bool:
        """Queue ``frag`` for snapshotting; False when it ran inline."""
        with self.mu:
            if id(frag) in self.pending:
                return True
            try:
                self.q.put_nowait(frag)
            except queue.Full:
                frag.snapshot()
                return False
            self.pending.add(id(frag))
        return True

    def _run(self):
        while True:
            frag = self.q.get()
            if frag is None:
                return
            with self.mu:
                self.pending.discard(id(frag))
            try:
                if frag.opn > 0 and getattr(frag, "_fh", None) is not None:
                    frag.snapshot()
                    self.done += 1
            except Exception as e:  # noqa: BLE001 - a failed snapshot keeps the op log valid
                if self.logger is not None:
                    self.logger.printf("snapshot %s: %s", getattr(frag, "path", "?"), e)
            finally:
                self.q.task_done()

    def drain(self):
        self.q.join()

    def close(self):
        self.drain()
        for _ in self._threads:
            self.q.put(None)
