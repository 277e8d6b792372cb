"""Metrics (reference: stats/stats.go, statsd/, prometheus/).

``StatsClient`` API: count / count_with_tags / gauge / histogram / set /
timing / with_tags.  Backends: Nop, Expvar (in-memory map served at
/debug/vars), Prometheus (text exposition at /metrics), StatsD (UDP, DataDog
tag syntax) and Multi.  GPU gauges (HBM bytes, kernel launches) are fed by the
server's runtime monitor.
"""
from __future__ import annotations

import socket
import threading
import time
from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Tuple


class NopStatsClient:
    def with_tags(self, *tags):
        return self

    def tags(self):
        return []

    def count(self, name, value=1, rate=1.0):
        pass

    def count_with_tags(self, name, value, tags, rate=1.0):
        pass

    def gauge(self, name, value, rate=1.0):
        pass

    def histogram(self, name, value, rate=1.0):
        pass

    def set(self, name, value, rate=1.0):
        pass

    def timing(self, name, seconds, rate=1.0):
        pass


class _Registry:
    def __init__(self):
        # reentrant: a finalizer or gc callback that records a stat while its
        # thread is inside one of these updates must not deadlock the process
        self.mu = threading.RLock()
        self.counters: Dict[Tuple[str, Tuple[str, ...]], float] = defaultdict(float)
        self.gauges: Dict[Tuple[str, Tuple[str, ...]], float] = {}
        self.hist: Dict[Tuple[str, Tuple[str, ...]], List[float]] = defaultdict(list)
        self.sets: Dict[Tuple[str, Tuple[str, ...]], set] = defaultdict(set)


class ExpvarStatsClient(NopStatsClient):
    def __init__(self, registry: Optional[_Registry] = None, tags: Sequence[str] = ()):
        self.reg = registry or _Registry()
        self._tags = tuple(sorted(tags))

    def with_tags(self, *tags):
        return type(self)(self.reg, tuple(sorted(set(self._tags) | set(tags))))

    def tags(self):
        return list(self._tags)

    def count(self, name, value=1, rate=1.0):
        with self.reg.mu:
            self.reg.counters[(name, self._tags)] += value

    def count_with_tags(self, name, value, tags, rate=1.0):
        with self.reg.mu:
            self.reg.counters[(name, tuple(sorted(set(self._tags) | set(tags))))] += value

    def gauge(self, name, value, rate=1.0):
        with self.reg.mu:
            self.reg.gauges[(name, self._tags)] = value

    def histogram(self, name, value, rate=1.0):
        with self.reg.mu:
            h = self.reg.hist[(name, self._tags)]
            h.append(value)
            if len(h) > 4096:
                del h[:2048]

    def set(self, name, value, rate=1.0):
        with self.reg.mu:
            self.reg.sets[(name, self._tags)].add(value)

    def timing(self, name, seconds, rate=1.0):
        self.histogram(name, seconds, rate)

    # ---- exposition
    def expvar(self) -> dict:
        out = {}
        with self.reg.mu:
            for (n, t), v in self.reg.counters.items():
                out[_key(n, t)] = v
            for (n, t), v in self.reg.gauges.items():
                out[_key(n, t)] = v
            for (n, t), v in self.reg.hist.items():
                if v:
                    s = sorted(v)
                    out[_key(n, t)] = {"count": len(s), "p50": s[len(s) // 2], "p99": s[int(len(s) * .99)]}
        return out

    def prometheus(self) -> str:
        lines = []
        with self.reg.mu:
            for (n, t), v in sorted(self.reg.counters.items()):
                lines.append(f"pilosa_{_prom(n)}_total{_labels(t)} {v}")
            for (n, t), v in sorted(self.reg.gauges.items()):
                lines.append(f"pilosa_{_prom(n)}{_labels(t)} {v}")
            for (n, t), v in sorted(self.reg.hist.items()):
                lines.append(f"pilosa_{_prom(n)}_count{_labels(t)} {len(v)}")
                lines.append(f"pilosa_{_prom(n)}_sum{_labels(t)} {sum(v)}")
        return "\n".join(lines) + "\n"


PrometheusStatsClient = ExpvarStatsClient


class StatsDClient(NopStatsClient):
    """DataDog-flavoured statsd over UDP (reference statsd/statsd.go)."""

    def __init__(self, host="127.0.0.1:8125", prefix="pilosa.", tags: Sequence[str] = ()):
        h, _, p = host.partition(":")
        self.addr = (h, int(p or 8125))
        self.prefix = prefix
        self._tags = tuple(tags)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)

    def with_tags(self, *tags):
        c = StatsDClient.__new__(StatsDClient)
        c.addr, c.prefix, c.sock = self.addr, self.prefix, self.sock
        c._tags = tuple(sorted(set(self._tags) | set(tags)))
        return c

    def tags(self):
        return list(self._tags)

    def _send(self, name, value, typ, tags=()):
        t = tuple(self._tags) + tuple(tags)
        msg = f"{self.prefix}{name}:{value}|{typ}" + (f"|#{','.join(t)}" if t else "")
        try:
            self.sock.sendto(msg.encode(), self.addr)
        except OSError:
            pass

    def count(self, name, value=1, rate=1.0):
        self._send(name, value, "c")

    def count_with_tags(self, name, value, tags, rate=1.0):
        self._send(name, value, "c", tags)

    def gauge(self, name, value, rate=1.0):
        self._send(name, value, "g")

    def histogram(self, name, value, rate=1.0):
        self._send(name, value, "h")

    def set(self, name, value, rate=1.0):
        self._send(name, value, "s")

    def timing(self, name, seconds, rate=1.0):
        self._send(name, int(seconds * 1000), "ms")


class MultiStatsClient(NopStatsClient):
    def __init__(self, *clients):
        self.clients = list(clients)

    def with_tags(self, *tags):
        return MultiStatsClient(*[c.with_tags(*tags) for c in self.clients])

    def tags(self):
        return self.clients[0].tags() if self.clients else []

    def count(self, *a, **k):
        for c in self.clients:
            c.count(*a, **k)

    def count_with_tags(self, *a, **k):
        for c in self.clients:
            c.count_with_tags(*a, **k)

    def gauge(self, *a, **k):
        for c in self.clients:
            c.gauge(*a, **k)

    def histogram(self, *a, **k):
        for c in self.clients:
            c.histogram(*a, **k)

    def set(self, *a, **k):
        for c in self.clients:
            c.set(*a, **k)

    def timing(self, *a, **k):
        for c in self.clients:
            c.timing(*a, **k)


def _key(n, t):
    return n if not t else n + "{" + ",".join(t) + "}"


def _prom(n):
    return "".join(ch if ch.isalnum() else "_" for ch in n)


def _labels(t):
    if not t:
        return ""
    parts = []
    for tag in t:
        k, _, v = tag.partition(":")
        parts.append(f'{_prom(k)}="{v}"')
    return "{" + ",".join(parts) + "}"


def new_stats_client(kind: str, host: str = "") -> NopStatsClient:
    kind = (kind or "none").lower()
    if kind in ("expvar", "prometheus"):
        return ExpvarStatsClient()
    if kind == "statsd":
        return StatsDClient(host or "127.0.0.1:8125")
    if kind == "none" or kind == "nop":
        return NopStatsClient()
    raise ValueError(f"'{kind}' not a valid stats client, choose from [expvar, statsd, prometheus, none].")


class Timer:
    def __init__(self, stats, name):
        self.stats, self.name = stats, name

    def __enter__(self):
        self.t = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.stats.timing(self.name, time.perf_counter() - self.t)
