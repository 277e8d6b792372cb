"""Cross-request batching of Count() queries for the GPU path.

The reference executes every HTTP query on its own (executor.go:116-209): a
Count is one map/reduce over the shards.  On a GPU a single query leaves the
device almost idle -- the headline kernels reach their throughput only with
thousands of queries per launch (bench.py, batch 4096).  ``CountCoalescer``
turns independent concurrent requests into such batches without adding a
timer: the first request for a (index, shard set) key becomes the *leader*
and launches everything pending for that key; requests that arrive while a
batch runs queue up and the leader hands leadership to one of them when its
own batch is done ("group commit").  An idle server therefore answers a lone
query with no added latency, and a loaded one batches automatically.

``run_batch(key, calls)`` returns one result per call, or None when the
batch cannot run on the device (each caller then executes its own query on
the regular path); an exception also falls back per call, so every request
gets exactly the result or error it would have had alone.
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Dict, List, Optional, Sequence

_FALLBACK = object()


class _Slot:
    __slots__ = ("call", "event", "result", "lead")

    def __init__(self, call):
        self.call = call
        self.event = threading.Event()
        self.result: Any = None
        self.lead = False


class CountCoalescer:
    def __init__(self, run_batch: Callable[[Any, Sequence[Any]], Optional[List[Any]]], max_batch: int = 4096):
        self.run_batch = run_batch
        self.max_batch = max(1, int(max_batch))
        self._lock = threading.Lock()
        self._pending: Dict[Any, List[_Slot]] = {}
        self._busy: set = set()
        self.batches = 0       # launched batches
        self.batched = 0       # calls that went through a batch
        self.fallbacks = 0     # calls sent back to the regular path
        self.last_error: Optional[BaseException] = None   # why the last batch fell back (diagnostics)

    def submit(self, key, call, fallback: Callable[[], Any]):
        """Result of ``call`` (via a batch, or ``fallback()``)."""
        slot = _Slot(call)
        with self._lock:
            self._pending.setdefault(key, []).append(slot)
            if key not in self._busy:
                self._busy.add(key)
                slot.lead = True
        while True:
            if slot.lead:
                slot.lead = False
                self._lead(key, slot)
            slot.event.wait()
            if slot.lead:           # handed leadership before our batch ran
                slot.event.clear()
                continue
            break
        if slot.result is _FALLBACK:
            return fallback()
        return slot.result

    def _lead(self, key, mine: _Slot):
        """Run batches for ``key`` until ``mine`` is answered, then pass the
        lead to a waiting request (or release the key)."""
        while True:
            with self._lock:
                q = self._pending.get(key) or []
                batch, rest = q[:self.max_batch], q[self.max_batch:]
                self._pending[key] = rest
            if batch:
                self._run(key, batch)
            with self._lock:
                rest = self._pending.get(key) or []
                if mine.event.is_set() or not rest:
                    if rest:
                        nxt = rest[0]
                        nxt.lead = True
                        nxt.event.set()
                    else:
                        self._busy.discard(key)
                        self._pending.pop(key, None)
                    return

    def _run(self, key, batch: List[_Slot]):
        try:
            res = self.run_batch(key, [s.call for s in batch]) if len(batch) > 0 else []
        except Exception as err:  # noqa: BLE001 - every call retries alone and gets its own error
            self.last_error = err
            res = None
        self.batches += 1
        if res is None or len(res) != len(batch):
            self.fallbacks += len(batch)
            for s in batch:
                s.result = _FALLBACK
                s.event.set()
            return
        self.batched += len(batch)
        for s, r in zip(batch, res):
            s.result = r
            s.event.set()
