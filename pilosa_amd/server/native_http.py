"""Native HTTP front end (pilosa_amd/native/httpd.cpp) behind the same route
table as the stdlib server (http_handler.Handler).

Reference: the Go net/http server of http/handler.go; the query route
(:293, handlePostQuery :495) keeps the JSON response shape of :977-1052.

Threads:
  * native epoll workers (C++) accept, parse and write;
  * ``count batchers`` take every queued Count-only JSON query request at
    once, grouped by index, and answer each group with ONE native compile +
    device launch over the concatenated PQL text (Executor._count_text_fast);
    the response bodies are formatted natively.  A group that cannot be
    answered that way (unknown field, keys, no GPU, cluster not ready, ...)
    goes back to the general queue so every error matches the Python path;
  * ``generic workers`` run every other request through Handler.dispatch.
"""
from __future__ import annotations

import os
import threading
import time
import traceback
from typing import Dict, List, Optional
from urllib.parse import parse_qs

from pilosa_amd.utils import gojson
from pilosa_amd.server.http_handler import Handler, HTTPError


def available() -> bool:
    try:
        from pilosa_amd import _httpd  # noqa: F401
        return True
    except ImportError:
        return False


class _Headers:
    """Case-insensitive header lookup (the subset of email.message.Message the
    handlers use)."""
    __slots__ = ("_d", "_items")

    def __init__(self, items):
        self._items = items
        self._d: Dict[str, str] = {}
        for k, v in items:
            self._d.setdefault(k.lower(), v)

    def get(self, name: str, default=None):
        return self._d.get(name.lower(), default)

    def __contains__(self, name):
        return name.lower() in self._d

    def __getitem__(self, name):
        return self._d.get(name.lower())

    def items(self):
        return list(self._items)


class NativeRequest:
    __slots__ = ("method", "path", "query", "headers", "body", "vars", "sent", "_srv", "_id")

    def __init__(self, srv, rid: int, method: str, path: str, query: str, headers, body: bytes):
        self._srv = srv
        self._id = rid
        self.method = method
        self.path = path.rstrip("/") or "/"
        self.query = {k: v[-1] for k, v in parse_qs(query, keep_blank_values=True).items()}
        self.headers = _Headers(headers)
        self.body = body
        self.vars = {}
        self.sent = False

    def send(self, status: int, body, ctype: str):
        if isinstance(body, str):
            body = body.encode()
        self._srv.respond(self._id, int(status), ctype, body or b"")
        self.sent = True

    def send_json(self, obj, status: int = 200):
        import json
        self.send(status, gojson.encode_line(obj), "application/json")


class NativeHTTPServer:
    """Drop-in for the ThreadingHTTPServer returned by make_http_server:
    ``server_address``, ``serve_forever()``, ``shutdown()``, ``server_close()``."""

    def __init__(self, handler: Handler, bind: str, io_threads: int = 4, workers: int = 16,
                 batchers: Optional[int] = None, max_batch: int = 1 << 16, topn_batchers: Optional[int] = None):
        from pilosa_amd import _httpd

        if batchers is None:
            batchers = int(os.environ.get("PILOSA_HTTP_COUNT_BATCHERS", "2"))
        if topn_batchers is None:
            topn_batchers = int(os.environ.get("PILOSA_HTTP_TOPN_BATCHERS", "2"))

        host, _, port = bind.rpartition(":")
        host = host or "0.0.0.0"
        if host == "localhost":
            host = "127.0.0.1"
        self.handler = handler
        self.srv = _httpd.Server(host, int(port), io_threads)
        self.server_address = (host, self.srv.port())
        self.srv.set_cors(list(getattr(handler, "allowed_origins", None) or []))
        self.n_workers, self.n_batchers, self.max_batch = workers, batchers, max_batch
        self.n_topn_batchers = topn_batchers
        # adaptive group commit (off with min 0): while another Count batch is
        # on the device, a batcher waits up to hold_us for hold_min requests
        # so the next batch is fuller; with the device idle it takes what is queued
        self.hold_min = int(os.environ.get("PILOSA_HTTP_HOLD_MIN", "0"))
        self.hold_us = int(os.environ.get("PILOSA_HTTP_HOLD_US", "300"))
        self._in_flight = 0
        self._if_mu = threading.Lock()
        self.held_batches = 0
        self.topn_batches = 0
        self.topn_batched_requests = 0
        self.topn_requeued = 0
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self.batches = 0
        self.batched_requests = 0
        self.requeued = 0
        self.count_s = 0.0
        self._gen = 0

    # ------------------------------------------------------------ lifecycle
    def serve_forever(self):
        # Count batching only pays with a device behind the executor
        server = self.handler.server
        self.srv.set_count_batching(server is None or getattr(server, "gpu", None) is not None)
        # cache-only TopN requests too: one device batch per group of them
        self.srv.set_topn_batching(server is not None and getattr(server, "gpu", None) is not None)
        # the liveness probe (GET /version, cluster membership) is answered by
        # the epoll workers: a saturated worker pool cannot fail it
        import json
        try:
            ver = self.handler.api.version()
            self.srv.set_static("GET", "/version", "application/json", (gojson.encode_line({"version": ver})).encode())
        except Exception:  # noqa: BLE001 - the Python route still answers
            pass
        self.srv.start()
        for i in range(self.n_workers):
            self._spawn(self._generic_loop, f"http-worker-{i}")
        self.set_batchers(self.n_batchers, self.n_topn_batchers)
        self._stop.wait()

    def set_batchers(self, count: Optional[int] = None, topn: Optional[int] = None):
        """Change the number of Count / TopN group-commit threads of a running
        server: a new generation of loops starts and the old ones exit after
        their current group."""
        self.n_batchers = self.n_batchers if count is None else count
        self.n_topn_batchers = self.n_topn_batchers if topn is None else topn
        self._gen += 1
        for i in range(self.n_batchers):
            self._spawn(self._count_loop, f"http-count-{i}", self._gen)
        for i in range(self.n_topn_batchers):
            self._spawn(self._topn_loop, f"http-topn-{i}", self._gen)

    def _spawn(self, fn, name, *args):
        t = threading.Thread(target=fn, name=name, args=args, daemon=True)
        t.start()
        self._threads.append(t)

    def shutdown(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)
        self.srv.stop()

    def server_close(self):
        pass

    def stats(self) -> dict:
        d = dict(self.srv.stats())
        d.update(batches=self.batches, batched_requests=self.batched_requests, requeued=self.requeued,
                 count_ms_per_batch=round(1000 * self.count_s / max(self.batches, 1), 3),
                 topn_batches=self.topn_batches, topn_batched_requests=self.topn_batched_requests,
                 topn_requeued=self.topn_requeued, count_batchers=self.n_batchers,
                 topn_batchers=self.n_topn_batchers, hold_min=self.hold_min, hold_us=self.hold_us,
                 held_batches=self.held_batches)
        server = self.handler.server
        gpu = getattr(getattr(server, "executor", None), "gpu", None)
        nb = getattr(gpu, "text_batches", 0)
        if nb:
            d.update(text_prep_ms_per_batch=round(1000 * gpu.text_prep_s / nb, 3),
                     text_wait_ms_per_batch=round(1000 * gpu.text_wait_s / nb, 3))
        return d

    # ------------------------------------------------------------ loops
    def _generic_loop(self):
        srv, handler = self.srv, self.handler
        while not self._stop.is_set():
            for rid, method, path, query, headers, body in srv.take(1, 500):
                req = NativeRequest(srv, rid, method, path, query, headers, body)
                try:
                    handler.dispatch(req)
                    if not req.sent:
                        req.send(200, b"", "text/plain; charset=utf-8")
                except HTTPError as e:
                    if not req.sent:
                        req.send(e.status, str(e) + "\n", "text/plain; charset=utf-8")
                except Exception as e:  # noqa: BLE001 - panic recovery (handler.go:323)
                    msg = f"PANIC: {e}\n{traceback.format_exc()}"
                    if handler.logger is not None:
                        handler.logger.printf("%s", msg)
                    if not req.sent:
                        req.send(500, msg, "text/plain; charset=utf-8")

    def _count_loop(self, gen: int = 0):
        srv = self.srv
        while not self._stop.is_set() and gen == self._gen:
            hold = self.hold_min > 1 and self._in_flight > 0
            if hold:
                self.held_batches += 1
            groups = srv.take_counts(self.max_batch, 500, self.hold_min if hold else 1, self.hold_us if hold else 0)
            if not groups:
                continue
            with self._if_mu:
                self._in_flight += 1
            try:
                self._count_groups(srv, groups)
            finally:
                with self._if_mu:
                    self._in_flight -= 1

    def _count_groups(self, srv, groups):
        for index, ids, ncalls, text in groups:
            t0 = time.perf_counter()
            counts = self._count_group(index, text, sum(ncalls))
            self.count_s += time.perf_counter() - t0
            if counts is None:
                self.requeued += len(ids)
                srv.requeue(ids)
                continue
            self.batches += 1
            self.batched_requests += len(ids)
            srv.respond_counts(ids, ncalls, counts)

    def _topn_loop(self, gen: int = 0):
        """Concurrent flat-TopN requests of an index, answered as ONE device
        batch (Executor._topn_text_fast: the calls of every request in one
        fused cache-only launch); bodies are formatted from the columnar
        results without building Pair objects.  A group the fast path cannot
        answer goes back to the general queue."""
        srv = self.srv
        from pilosa_amd.server.encoding import result_json_bytes
        while not self._stop.is_set() and gen == self._gen:
            for index, ids, ncalls, text in srv.take_topn(self.max_batch, 500):
                res = self._topn_group(index, text, sum(ncalls))
                if res is None:
                    self.topn_requeued += len(ids)
                    srv.requeue(ids)
                    continue
                self.topn_batches += 1
                self.topn_batched_requests += len(ids)
                k = 0
                for rid, nc in zip(ids, ncalls):
                    body = b'{"results":[' + b",".join(result_json_bytes(r) for r in res[k:k + nc]) + b"]}\n"
                    k += nc
                    srv.respond(rid, 200, "application/json", body)

    def _topn_group(self, index: str, text: str, ncalls: int):
        server = self.handler.server
        api = self.handler.api
        ex = getattr(server, "executor", None) if server is not None else None
        if ex is None or api is None:
            return None
        try:
            api.validate("Query")
            res = ex._topn_plain_fast(index, text)
            if res is None:
                res = ex._topn_text_fast(index, text)
        except Exception:  # noqa: BLE001 - the general path reports it
            return None
        if res is None or len(res) != ncalls:
            return None
        return res

    def _count_group(self, index: str, text: str, ncalls: int) -> Optional[List[int]]:
        server = self.handler.server
        api = self.handler.api
        ex = getattr(server, "executor", None) if server is not None else None
        if ex is None or api is None:
            return None
        try:
            api.validate("Query")
            res = ex._count_text_fast(index, text, None, None, min_calls=1)
        except Exception:  # noqa: BLE001 - the general path reports it
            return None
        if res is None or len(res) != ncalls:
            return None
        return [int(x) for x in res]


def make_native_http_server(handler: Handler, bind: str, **kw) -> NativeHTTPServer:
    return NativeHTTPServer(handler, bind, **kw)
