"""Tracing (reference: tracing/tracing.go, tracing/opentracing).

A global tracer (no-op by default) wraps executor/API/fragment work in spans.
``RecordingTracer`` keeps finished spans in memory (tests, /debug/traces) and
``HipEventTracer`` additionally brackets GPU work with torch/HIP events so the
span durations reflect device time.  Cross-node propagation uses the
``X-Pilosa-Trace`` HTTP header (inject/extract like http/client.go:1043 and
http/handler.go:229-236).
"""
from __future__ import annotations

import contextlib
import threading
import time
import uuid
from typing import Dict, List, Optional

TRACE_HEADER = "X-Pilosa-Trace"


class Span:
    __slots__ = ("name", "trace_id", "span_id", "parent_id", "start", "end", "tags", "events")

    def __init__(self, name, trace_id, parent_id=None):
        self.name = name
        self.trace_id = trace_id
        self.span_id = uuid.uuid4().hex[:16]
        self.parent_id = parent_id
        self.start = time.perf_counter()
        self.end = None
        self.tags: Dict[str, object] = {}
        self.events = None   # [start, end] HIP events of a GPU span (HipEventTracer)

    def set_tag(self, k, v):
        self.tags[k] = v

    @property
    def duration(self) -> float:
        return (self.end or time.perf_counter()) - self.start

    def device_ms(self, wait: bool = True) -> Optional[float]:
        """Device time between the span's start and end events on its stream
        (the kernels / copies / collectives it enqueued, plus anything other
        threads queued on that stream in between); None for a host span, or
        when ``wait`` is False and the device has not reached the end yet."""
        ev = self.events
        if not ev or ev[1] is None:
            return None
        if not ev[1].query():
            if not wait:
                return None
            ev[1].synchronize()
        return float(ev[0].elapsed_time(ev[1]))

    def to_dict(self, wait: bool = False) -> dict:
        d = {"name": self.name, "trace": self.trace_id, "span": self.span_id, "parent": self.parent_id,
             "ms": round(self.duration * 1000, 3), "tags": {k: str(v) for k, v in self.tags.items()}}
        dm = self.device_ms(wait)
        if dm is not None:
            d["device_ms"] = round(dm, 4)
        return d


class NopTracer:
    def start_span(self, name, parent=None, gpu=False):
        return None

    def finish(self, span):
        pass


class RecordingTracer:
    def __init__(self, limit: int = 10000):
        self.spans: List[Span] = []
        self.limit = limit
        self.mu = threading.Lock()

    def start_span(self, name, parent: Optional[Span] = None, gpu: bool = False):
        tid = parent.trace_id if parent is not None else uuid.uuid4().hex
        return Span(name, tid, parent.span_id if parent is not None else None)

    def finish(self, span: Span):
        span.end = time.perf_counter()
        with self.mu:
            self.spans.append(span)
            if len(self.spans) > self.limit:
                del self.spans[: len(self.spans) - self.limit]

    def trace(self, trace_id: str) -> List[Span]:
        with self.mu:
            return [s for s in self.spans if s.trace_id == trace_id]

    def tree(self, trace_id: str, wait: bool = True) -> List[dict]:
        """The spans of one trace as nested dicts (children under
        ``children``, in start order); GPU spans carry ``device_ms``."""
        spans = sorted(self.trace(trace_id), key=lambda s: s.start)
        nodes = {s.span_id: dict(s.to_dict(wait), children=[]) for s in spans}
        roots = []
        for s in spans:
            n = nodes[s.span_id]
            if s.parent_id in nodes:
                nodes[s.parent_id]["children"].append(n)
            else:
                roots.append(n)
        return roots


class HipEventTracer(RecordingTracer):
    """RecordingTracer whose GPU spans (``span(name, gpu=True)``: kernel
    launches, device-to-host copies, collectives) also record HIP events on
    the current stream at start and end, so the span tree shows device time
    next to host time (HIP-event timing per kernel and per RCCL
    op).  Events are read lazily (``Span.device_ms``), so tracing adds no
    synchronisation to the query path."""

    def __init__(self, limit: int = 10000):
        super().__init__(limit)
        try:
            import torch
            self._torch = torch if torch.cuda.is_available() else None
        except Exception:  # noqa: BLE001 - no torch: host spans only
            self._torch = None

    def start_span(self, name, parent: Optional[Span] = None, gpu: bool = False):
        s = super().start_span(name, parent)
        if gpu and self._torch is not None:
            e = self._torch.cuda.Event(enable_timing=True)
            e.record()
            s.events = [e, None]
        return s

    def finish(self, span: Span):
        if span.events is not None:
            e = self._torch.cuda.Event(enable_timing=True)
            e.record()
            span.events[1] = e
        super().finish(span)


_tracer = NopTracer()
_local = threading.local()


def set_global_tracer(t):
    global _tracer
    _tracer = t


def global_tracer():
    return _tracer


def current_span() -> Optional[Span]:
    return getattr(_local, "span", None)


def enabled() -> bool:
    return not isinstance(_tracer, NopTracer)


@contextlib.contextmanager
def span(name: str, gpu: bool = False, **tags):
    """A child span of the thread's current span (a new trace at the top);
    ``gpu``: bracket it with HIP events too (HipEventTracer)."""
    t = _tracer
    if isinstance(t, NopTracer):
        yield None
        return
    parent = current_span()
    s = t.start_span(name, parent, gpu=gpu)
    for k, v in tags.items():
        s.set_tag(k, v)
    _local.span = s
    try:
        yield s
    finally:
        _local.span = parent
        t.finish(s)


def bind(fn):
    """``fn`` wrapped to run under the caller's current span in whatever
    thread calls it (map/reduce fan-out pools, executor shard workers): the
    span context is thread-local, as Go's is carried in a context.Context."""
    parent = current_span()
    if parent is None or isinstance(_tracer, NopTracer):
        return fn

    def run(*a, **kw):
        prev = current_span()
        _local.span = parent
        try:
            return fn(*a, **kw)
        finally:
            _local.span = prev
    return run


def context() -> str:
    """The current span as the propagation string (header value / mesh command field)."""
    s = current_span()
    return f"{s.trace_id}:{s.span_id}" if s is not None else ""


def inject_headers(headers: dict):
    s = current_span()
    if s is not None:
        headers[TRACE_HEADER] = f"{s.trace_id}:{s.span_id}"


def extract_headers(headers) -> Optional[Span]:
    v = headers.get(TRACE_HEADER) if headers is not None else None
    if not v or ":" not in v:
        return None
    tid, sid = v.split(":", 1)
    s = Span("remote", tid)
    s.span_id = sid
    return s


@contextlib.contextmanager
def remote_parent(headers):
    """Run the block under the span named by a propagated context (an HTTP
    header dict, or a ``context()`` string from a mesh command)."""
    if isinstance(headers, str):
        headers = {TRACE_HEADER: headers} if headers else None
    p = extract_headers(headers)
    prev = current_span()
    if p is not None:
        _local.span = p
    try:
        yield
    finally:
        _local.span = prev
