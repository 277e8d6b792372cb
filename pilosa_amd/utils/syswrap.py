"""Process-wide cap on memory-mapped fragment files (reference syswrap/mmap.go:
a counter of live mmaps against ``max-map-count``; past the cap a mapping is
refused with ErrMaxMapCountReached and the caller falls back to reading the
file into heap).  Cold fragments map their files through
_roaring.MappedBitmap (models/fragment.py ``_cold``); each live view holds one
slot."""
from __future__ import annotations

import threading

_lock = threading.Lock()
_count = 0
_max = 1_000_000


class ErrMaxMapCountReached(RuntimeError):
    def __init__(self):
        super().__init__("maximum map count reached")


def set_max_map_count(n: int) -> None:
    global _max
    with _lock:
        _max = max(0, int(n))


def max_map_count() -> int:
    return _max


def try_acquire() -> bool:
    """Take one map slot; False when the cap is reached."""
    global _count
    with _lock:
        if _count >= _max:
            return False
        _count += 1
        return True


def release() -> None:
    global _count
    with _lock:
        if _count > 0:
            _count -= 1


def map_count() -> int:
    return _count
