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
    __slots__ = ("name", "trace_id", "span_id", "parent_id", "start", "end", "tags")

    def __init__(self, name, trace_id, parent_id=None):
        self.name = name
        self.trace_id = trace_id
        self.span_id = uuid.uuid4().hex[:16]
        self.parent_id = parent_id
        self.start = time.perf_counter()
        self.end = None
        self.tags: Dict[str, object] = {}

    def set_tag(self, k, v):
        self.tags[k] = v

    @property
    def duration(self) -> float:
        return (self.end or time.perf_counter()) - self.start


class NopTracer:
    def start_span(self, name, parent=None):
        return None

    def finish(self, span):
        pass


class RecordingTracer:
    def __init__(self, limit: int = 10000):
        self.spans: List[Span] = []
        self.limit = limit
        self.mu = threading.Lock()

    def start_span(self, name, parent: Optional[Span] = None):
        tid = parent.trace_id if parent is not None else uuid.uuid4().hex
        return Span(name, tid, parent.span_id if parent is not None else None)

    def finish(self, span: Span):
        span.end = time.perf_counter()
        with self.mu:
            self.spans.append(span)
            if len(self.spans) > self.limit:
                del self.spans[: len(self.spans) - self.limit]


_tracer = NopTracer()
_local = threading.local()


def set_global_tracer(t):
    global _tracer
    _tracer = t


def global_tracer():
    return _tracer


def current_span() -> Optional[Span]:
    return getattr(_local, "span", None)


@contextlib.contextmanager
def span(name: str, **tags):
    t = _tracer
    if isinstance(t, NopTracer):
        yield None
        return
    parent = current_span()
    s = t.start_span(name, parent)
    for k, v in tags.items():
        s.set_tag(k, v)
    _local.span = s
    try:
        yield s
    finally:
        _local.span = parent
        t.finish(s)


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
    p = extract_headers(headers)
    prev = current_span()
    if p is not None:
        _local.span = p
    try:
        yield
    finally:
        _local.span = prev
