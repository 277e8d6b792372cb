"""Native HTTP front end (native/httpd.cpp, server/native_http.py): same
answers as the stdlib server on the reference's routes (http/handler.go
:276-314, query responses :977-1052), HTTP/1.1 details (keep-alive,
pipelining, chunked bodies, Connection: close, Expect: 100-continue,
OPTIONS), and the Count group commit -- concurrent Count-only requests
answered as one batch, with a fallback to the general path that keeps every
answer and error identical."""
import json
import socket
import tempfile
import threading

import pytest

from pilosa_amd.server import native_http

pytestmark = [pytest.mark.skipif(not native_http.available(), reason="_httpd not built"), pytest.mark.timeout(90)]


def _server(native: bool):
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger
    return Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger(),
                  native_http=native).open()


def _raw(port, data: bytes) -> bytes:
    # generous: right after a load phase the server may still be draining the
    # load generator's backlog on a busy (xdist) machine
    s = socket.create_connection(("127.0.0.1", port), timeout=60)
    s.sendall(data)
    out = b""
    while True:
        x = s.recv(65536)
        if not x:
            break
        out += x
    s.close()
    return out


def _responses(raw: bytes):
    """[(status, body)] of a stream of HTTP/1.1 responses."""
    out = []
    while raw:
        he = raw.index(b"\r\n\r\n")
        head = raw[:he].decode()
        status = int(head.split(" ", 2)[1])
        n = 0
        for line in head.split("\r\n")[1:]:
            k, _, v = line.partition(":")
            if k.lower() == "content-length":
                n = int(v)
        if status == 100:
            raw = raw[he + 4:]
            continue
        out.append((status, raw[he + 4:he + 4 + n]))
        raw = raw[he + 4 + n:]
    return out


def _req(method, path, body=b"", headers=(), close=False):
    h = [f"{method} {path} HTTP/1.1", "Host: x", f"Content-Length: {len(body)}", *headers]
    if close:
        h.append("Connection: close")
    return ("\r\n".join(h) + "\r\n\r\n").encode() + body


SCRIPT = [
    ("POST", "/index/i", b""),
    ("POST", "/index/i/field/f", b""),
    ("POST", "/index/i/field/g", b'{"options": {"type": "int", "min": 0, "max": 1000}}'),
    ("POST", "/index/i/query", b"Set(1, f=2) Set(5, f=2) Set(3, f=7) Set(2, g=40)"),
    ("POST", "/index/i/query", b"Count(Row(f=2))"),
    ("POST", "/index/i/query", b"Count(Row(f=2)) Count(Union(Row(f=2), Row(f=7)))"),
    ("POST", "/index/i/query", b"Row(f=2)"),
    ("POST", "/index/i/query", b"Sum(field=g)"),
    ("POST", "/index/i/query", b"Count(Row(nope=2))"),
    ("POST", "/index/missing/query", b"Count(Row(f=2))"),
    ("POST", "/index/i/query", b"Count(Row(f=2)"),
    ("POST", "/index/i/query?shards=0", b"Count(Row(f=2))"),
    ("POST", "/index/i/query?bogus=1", b"Count(Row(f=2))"),
    ("GET", "/index/i", b""),
    ("GET", "/schema", b""),
    ("GET", "/nope", b""),
    ("DELETE", "/index/i/query", b""),
    ("GET", "/version", b""),
]


def test_native_matches_stdlib_server():
    got = {}
    for native in (True, False):
        srv = _server(native)
        try:
            assert type(srv.httpd).__name__ == ("NativeHTTPServer" if native else "_Srv")
            port = srv.httpd.server_address[1]
            got[native] = [_responses(_raw(port, _req(m, p, b, close=True)))[0] for m, p, b in SCRIPT]
        finally:
            srv.close()
    for (m, p, b), a, c in zip(SCRIPT, got[True], got[False]):
        assert a == c, (m, p, b, a, c)
    statuses = [s for s, _ in got[True]]
    assert statuses[4] == 200 and json.loads(got[True][4][1]) == {"results": [2]}
    assert 404 in statuses and 400 in statuses and 405 in statuses


def test_pipelining_chunked_close_options_continue():
    srv = _server(True)
    try:
        port = srv.httpd.server_address[1]
        _raw(port, _req("POST", "/index/i", close=True))
        _raw(port, _req("POST", "/index/i/field/f", close=True))
        _raw(port, _req("POST", "/index/i/query", b"Set(10, f=1) Set(11, f=1)", close=True))
        chunked = (b"POST /index/i/query HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
                   b"6\r\nCount(\r\n9\r\nRow(f=1))\r\n0\r\nX-Trailer: 1\r\n\r\n")
        stream = (_req("POST", "/index/i/query", b"Count(Row(f=1))") + chunked
                  + _req("OPTIONS", "/index/i/query") + _req("GET", "/version")
                  + _req("POST", "/index/i/query", b"Count(Row(f=9))", close=True)
                  + _req("GET", "/version"))  # after Connection: close: never answered
        rs = _responses(_raw(port, stream))
        # OPTIONS without configured CORS origins: the route table's 405, as
        # the reference's router answers (server/handler_test.go "CORS" :830)
        assert [s for s, _ in rs] == [200, 200, 405, 200, 200]
        assert json.loads(rs[0][1]) == {"results": [2]} and json.loads(rs[1][1]) == {"results": [2]}
        assert b"version" in rs[3][1]
        assert json.loads(rs[4][1]) == {"results": [0]}
        # Expect: 100-continue: the interim response arrives before the body is sent
        s = socket.create_connection(("127.0.0.1", port), timeout=10)
        body = b"Count(Row(f=1))"
        s.sendall(f"POST /index/i/query HTTP/1.1\r\nHost: x\r\nExpect: 100-continue\r\n"
                  f"Content-Length: {len(body)}\r\nConnection: close\r\n\r\n".encode())
        assert s.recv(100).startswith(b"HTTP/1.1 100 Continue")
        s.sendall(body)
        out = b""
        while True:
            x = s.recv(65536)
            if not x:
                break
            out += x
        assert _responses(out) == [(200, b'{"results":[2]}\n')]
        # malformed request line
        assert _responses(_raw(port, b"BROKEN\r\n\r\n"))[0][0] == 400
    finally:
        srv.close()


def _host_fast(ex, calls):
    """A stand-in device fast path: the concatenated group text answered by
    the host executor (records each call)."""
    from pilosa_amd.pql import parse_string

    def fast(index, text, shards, opt, min_calls=None):
        calls.append(text)
        q = parse_string(text)
        gpu = ex.gpu
        return [int(r) for r in ex.execute(index, q).results] if gpu is None else None
    return fast


def test_count_group_commit_and_fallback():
    from pilosa_amd import _httpd
    srv = _server(True)
    try:
        port = srv.httpd.server_address[1]
        for m, p, b in SCRIPT[:4]:
            _raw(port, _req(m, p, b, close=True))
        ex = srv.executor
        calls = []
        ex._count_text_fast = _host_fast(ex, calls)
        srv.httpd.srv.set_count_batching(True)
        bodies = [b"Count(Row(f=2))", b"Count(Row(f=7)) Count(Row(f=2))", b"Count(Intersect(Row(f=2), Row(f=7)))",
                  b"Count(Row(f=99))"]
        want = [[2], [1, 2], [0], [0]]
        res = _httpd.load("127.0.0.1", port, "/index/i/query", bodies, 32, 4, 1.0, 400)
        # a loaded machine completes fewer requests in the 1 s window
        assert res["errors"] == 0 and res["requests"] >= 8
        assert len(res["samples"]) == min(400, res["requests"])
        for k, body in res["samples"]:
            assert json.loads(body)["results"] == want[k]
        st = srv.httpd.stats()
        assert st["count_requests"] >= res["requests"] and st["batched_requests"] > 0
        assert any(t.count("Count(") > 2 for t in calls), "no multi-request group was formed"
        # a group the fast path declines (unknown field) goes to the general
        # path: same error as the stdlib server, other groups unaffected
        rs = _responses(_raw(port, _req("POST", "/index/i/query", b"Count(Row(nope=1))", close=True)))
        assert rs[0] == (400, b"{\"error\":\"executing: field not found\"}\n")
        assert srv.httpd.stats()["requeued"] >= 1
    finally:
        srv.close()


def test_count_group_commit_with_adaptive_hold():
    """Adaptive group commit (take_counts min_n / hold_us): while another
    batch is in flight a batcher waits briefly for a fuller batch; every
    answer is unchanged and the held takes are counted."""
    from pilosa_amd import _httpd
    srv = _server(True)
    try:
        port = srv.httpd.server_address[1]
        for m, p, b in SCRIPT[:4]:
            _raw(port, _req(m, p, b, close=True))
        ex = srv.executor
        calls = []
        ex._count_text_fast = _host_fast(ex, calls)
        srv.httpd.hold_min, srv.httpd.hold_us = 8, 2000
        srv.httpd.set_batchers(2)
        srv.httpd.srv.set_count_batching(True)
        bodies = [b"Count(Row(f=2))", b"Count(Row(f=7)) Count(Row(f=2))"]
        want = [[2], [1, 2]]
        res = _httpd.load("127.0.0.1", port, "/index/i/query", bodies, 32, 4, 1.0, 200)
        assert res["errors"] == 0 and res["requests"] >= 8
        for k, body in res["samples"]:
            assert json.loads(body)["results"] == want[k]
        st = srv.httpd.stats()
        assert st["hold_min"] == 8 and st["batched_requests"] > 0
        assert st["held_batches"] > 0, "no batcher ever held for a fuller batch"
    finally:
        srv.close()


def test_concurrent_generic_requests():
    srv = _server(True)
    try:
        port = srv.httpd.server_address[1]
        _raw(port, _req("POST", "/index/i", close=True))
        _raw(port, _req("POST", "/index/i/field/f", close=True))
        errs = []

        def writer(k):
            try:
                for j in range(20):
                    rs = _responses(_raw(port, _req("POST", "/index/i/query", f"Set({k * 100 + j}, f=3)".encode(),
                                                    close=True)))
                    assert rs[0][0] == 200
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=writer, args=(k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs
        rs = _responses(_raw(port, _req("POST", "/index/i/query", b"Count(Row(f=3))", close=True)))
        assert json.loads(rs[0][1]) == {"results": [160]}
    finally:
        srv.close()


def test_chunk_size_and_framing_attacks_rejected():
    """Chunk sizes are hex digits only and bounded before any arithmetic; a
    request carrying both Content-Length and Transfer-Encoding, or a
    non-numeric Content-Length, is refused (ADVICE r02 httpd.cpp:637)."""
    srv = _server(True)
    try:
        port = srv.httpd.server_address[1]
        head = b"POST /index/i/query HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
        for body in (b"ffffffffffffff9c\r\nCount(Row(f=1))\r\n0\r\n\r\n",   # wraps size_t arithmetic
                     b"zz\r\nabc\r\n0\r\n\r\n",                              # not hex
                     b"\r\nabc\r\n0\r\n\r\n",                                # empty size line
                     b"3\r\nabcXY0\r\n\r\n"):                                # chunk not CRLF-terminated
            rs = _responses(_raw(port, head + body))
            assert rs and rs[0][0] in (400, 413), (body, rs)
        rs = _responses(_raw(port, b"POST /index/i/query HTTP/1.1\r\nHost: x\r\nContent-Length: 3\r\n"
                                   b"Transfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n0\r\n\r\n"))
        assert rs[0][0] == 400
        rs = _responses(_raw(port, b"POST /index/i/query HTTP/1.1\r\nHost: x\r\nContent-Length: 1x\r\n\r\nx"))
        assert rs[0][0] == 400
        # the server still answers normally afterwards
        assert _responses(_raw(port, _req("GET", "/version", close=True)))[0][0] == 200
    finally:
        srv.close()


def test_pipelined_requests_run_in_order():
    """A pipelined Set followed by Count/Row on one keep-alive connection sees
    the write: a connection's requests execute one at a time, in order, even
    though Count-only requests go to the batcher (ADVICE r02 httpd.cpp:709)."""
    srv = _server(True)
    try:
        port = srv.httpd.server_address[1]
        _raw(port, _req("POST", "/index/i", close=True))
        _raw(port, _req("POST", "/index/i/field/f", close=True))
        stream = b""
        for k in range(40):
            stream += _req("POST", "/index/i/query", f"Set({k}, f=3)".encode())
            stream += _req("POST", "/index/i/query", b"Count(Row(f=3))")
        stream += _req("POST", "/index/i/query", b"Row(f=3)", close=True)
        rs = _responses(_raw(port, stream))
        assert len(rs) == 81
        counts = [json.loads(b)["results"][0] for s, b in rs[1:80:2]]
        assert counts == list(range(1, 41))
        assert json.loads(rs[80][1])["results"][0]["columns"] == list(range(40))
    finally:
        srv.close()


def test_topn_group_commit_and_fallback():
    """Concurrent flat-TopN requests are taken as one group per index
    (native/httpd.cpp kind 2) and answered by ONE fast-path call; a group
    the fast path declines goes to the general path with identical answers."""
    from pilosa_amd import _httpd
    from pilosa_amd.pql import parse_string
    srv = _server(True)
    try:
        port = srv.httpd.server_address[1]
        for m, p, b in SCRIPT[:4]:
            _raw(port, _req(m, p, b, close=True))
        ex = srv.executor
        texts = []

        def fast(index, text, shards=None):
            texts.append(text)
            return ex.execute(index, parse_string(text)).results
        ex._topn_text_fast = fast
        srv.httpd.srv.set_topn_batching(True)
        bodies = [b"TopN(f, n=2)", b"TopN(f, n=1) TopN(f)", b"TopN(f, n=5, threshold=2)"]
        # the general path's answers (stdlib JSON encoding of the same results)
        want = [json.loads(_responses(_raw(port, _req("POST", "/index/i/query", b, close=True)))[0][1])["results"]
                for b in bodies]
        assert want[0] and want[0][0], want
        res = _httpd.load("127.0.0.1", port, "/index/i/query", bodies, 24, 4, 1.0, 300)
        assert res["errors"] == 0 and res["requests"] >= 6
        for k, body in res["samples"]:
            assert json.loads(body)["results"] == want[k], (k, body)
        st = srv.httpd.stats()
        assert st["topn_requests"] >= res["requests"] and st["topn_batched_requests"] > 0
        assert any(t.count("TopN(") > 3 for t in texts), "no multi-request TopN group was formed"
        # nested calls (a src row) are not batched; a declined group falls back
        rs = _responses(_raw(port, _req("POST", "/index/i/query", b"TopN(f, Row(f=2), n=1)", close=True)))
        assert rs[0][0] == 200 and len(json.loads(rs[0][1])["results"]) == 1
        ex._topn_text_fast = lambda index, text, shards=None: None
        rs = _responses(_raw(port, _req("POST", "/index/i/query", b"TopN(nope, n=1)", close=True)))
        assert rs[0][0] == 400 and srv.httpd.stats()["topn_requeued"] >= 1
    finally:
        srv.close()
