"""Drives one sanitizer-built host module (the reference runs its
whole suite under ``go test -race`` and fuzzes the roaring decoder,
roaring/fuzzer.go:28-323).

    python san_driver.py <module-dir> <httpd|translate|arena|pql> [seed]

``<module-dir>`` holds the module built by ``native/build.py:build_sanitized``
(ASan+UBSan or TSan); the sanitizer runtime is preloaded by the caller
(tests/test_native_sanitizers.py).  Each mode mixes concurrent well-formed use
with malformed / truncated / mutated input and exits 0 only when every check
holds; a sanitizer report aborts the process with its own exit status.
Prints ``<mode>: ok`` on success.
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import random
import shutil
import socket
import sys
import tempfile
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))


def load(moddir: str, name: str):
    path = next(os.path.join(moddir, f) for f in os.listdir(moddir) if f.startswith(name + ".") and f.endswith(".so"))
    loader = importlib.machinery.ExtensionFileLoader(name, path)
    spec = importlib.util.spec_from_file_location(name, path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


def mutate(rng: random.Random, b: bytes, n: int = 4) -> bytes:
    b = bytearray(b)
    for _ in range(rng.randint(1, n)):
        op = rng.randrange(4)
        if op == 0 and b:
            b[rng.randrange(len(b))] = rng.randrange(256)
        elif op == 1:
            b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        elif op == 2 and b:
            del b[rng.randrange(len(b))]
        elif b:
            del b[rng.randrange(len(b)):]
    return bytes(b)


def run_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


# --------------------------------------------------------------------- httpd
def drive_httpd(m, rng: random.Random):
    """Concurrent keep-alive load (both the batched Count queue and the
    general queue), pipelined requests, chunked bodies and malformed framing
    against the epoll workers."""
    srv = m.Server("127.0.0.1", 0, 4, 1 << 20)
    srv.start()
    srv.set_count_batching(True)
    port = srv.port()
    stop = threading.Event()

    def general():
        while not stop.is_set():
            for rid, method, path, query, headers, body in srv.take(8, 50):
                srv.respond(rid, 200, "application/json", b'{"len": %d}' % len(body))

    def counts():
        while not stop.is_set():
            for index, ids, ncalls, text in srv.take_counts(1 << 12, 50):
                if rng.random() < 0.1:
                    srv.requeue(ids)      # the general path answers these
                    continue
                srv.respond_counts(ids, ncalls, [7] * sum(ncalls))
    responders = [threading.Thread(target=general), threading.Thread(target=general), threading.Thread(target=counts)]
    for t in responders:
        t.start()

    def ok_request(path=b"/index/i/query", body=b"Count(Row(f=1))"):
        s = socket.create_connection(("127.0.0.1", port), timeout=5)
        s.sendall(b"POST " + path + b" HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % len(body) + body)
        data = b""
        while b"\r\n\r\n" not in data:
            chunk = s.recv(65536)
            if not chunk:
                break
            data += chunk
        s.close()
        return data

    def fuzz_client(seed):
        r = random.Random(seed)
        good = [b"POST /index/i/query HTTP/1.1\r\nHost: x\r\nContent-Length: 15\r\n\r\nCount(Row(f=1))",
                b"GET /status HTTP/1.1\r\nHost: x\r\n\r\n",
                b"POST /index/i/query HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nCount\r\na\r\n(Row(f=1))\r\n0\r\n\r\n",
                b"POST /index/i/field/f/import HTTP/1.1\r\nContent-Length: 4\r\n\r\nabcd"]
        bad = [b"POST / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n",
               b"POST / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nffffffffffffffffff\r\n",
               b"POST / HTTP/1.1\r\nContent-Length: -5\r\n\r\n",
               b"POST / HTTP/1.1\r\nContent-Length: 99999999999999999999\r\n\r\n",
               b"POST / HTTP/1.1\r\nContent-Length: 5000000\r\n\r\nxx",
               b"GET / HTTP/1.1\r\n" + b"X-Long: " + b"a" * 70000 + b"\r\n\r\n",
               b"\r\n\r\n\r\n", b"GARBAGE\x00\xff\r\n\r\n", b"GET\r\n\r\n"]
        for _ in range(40):
            k = r.randrange(4)
            if k == 0:      # pipelined well-formed requests in one write
                payload = b"".join(r.choice(good) for _ in range(r.randint(2, 6)))
            elif k == 1:
                payload = r.choice(bad)
            elif k == 2:
                payload = mutate(r, r.choice(good), 6)
            else:           # a request split over several writes
                payload = r.choice(good)
            try:
                s = socket.create_connection(("127.0.0.1", port), timeout=2)
                if k == 3:
                    cut = sorted(r.sample(range(1, len(payload)), 2))
                    for a, b_ in zip([0] + cut, cut + [len(payload)]):
                        s.sendall(payload[a:b_])
                        time.sleep(0.001)
                else:
                    s.sendall(payload)
                if r.random() < 0.3:
                    s.shutdown(socket.SHUT_WR)
                s.settimeout(0.3)
                try:
                    while s.recv(65536):
                        pass
                except OSError:
                    pass
                s.close()
            except OSError:
                pass

    load_out = {}

    def loadgen():
        load_out.update(m.load("127.0.0.1", port, "/index/i/query",
                               ["Count(Row(f=1))", "Count(Row(f=1)) Count(Row(f=2))", "Row(f=3)"],
                               32, 4, 1.5, 16))
    base = rng.randrange(1 << 30)
    run_threads([loadgen] + [lambda s=s: fuzz_client(s) for s in range(base, base + 6)])
    assert load_out["requests"] > 0, load_out
    assert load_out["errors"] == 0, load_out
    assert b" 200 " in ok_request(), "server stopped answering after the fuzz clients"
    assert b" 200 " in ok_request(b"/index/i/field/f/import", b"\x00" * 1000)
    stop.set()
    for t in responders:
        t.join()
    srv.stop()
    st = srv.stats()
    assert st["requests"] > 0, st


# ----------------------------------------------------------------- translate
def drive_translate(m, rng: random.Random):
    """Concurrent create/lookup/reverse lookups and log streaming on one
    store, reopen consistency, then replay of mutated and truncated logs."""
    d = tempfile.mkdtemp()
    try:
        path = os.path.join(d, "keys")
        st = m.Store(path, False, 0)
        st.open()
        keys = [f"k{i}" for i in range(3000)]

        def writer(seed):
            r = random.Random(seed)
            for _ in range(60):
                ks = r.sample(keys, r.randint(1, 40))
                t = r.choice([m.T_COLUMN, m.T_ROW])
                ids = st.translate(t, "i", "f" if t == m.T_ROW else "", ks, True)
                assert all(ids), "created keys must get ids"
                back = st.keys_of(t, "i", "f" if t == m.T_ROW else "", ids)
                assert back == ks, (back[:3], ks[:3])

        def reader(seed):
            r = random.Random(seed)
            for _ in range(60):
                st.translate(m.T_COLUMN, "i", "", r.sample(keys, 10), False)
                off = r.randrange(st.size() + 1)
                try:
                    st.read_from(off)
                except Exception:  # noqa: BLE001 -- an offset inside an entry
                    pass
                st.entries(0)
                st.seq(m.T_COLUMN, "i", "")
        run_threads([lambda s=s: writer(s) for s in range(4)] + [lambda s=s: reader(s + 10) for s in range(3)])
        cols = st.translate(m.T_COLUMN, "i", "", keys, False)
        log = st.read_from(0)
        st.close()
        st2 = m.Store(path, True, 0)
        st2.open()
        assert st2.translate(m.T_COLUMN, "i", "", keys, False) == cols
        st2.close()
        for k in range(120):
            bad = mutate(rng, log, 8) if k % 3 else log[:rng.randrange(len(log) + 1)]
            s3 = m.Store(os.path.join(d, f"fuzz{k}"), False, 0)
            s3.open()
            try:
                s3.apply_log(bad)
            except Exception:  # noqa: BLE001 -- corrupt input is refused, not fatal
                pass
            s3.entries(0)
            s3.close()
            with open(os.path.join(d, f"file{k}"), "wb") as fh:
                fh.write(bad)
            s4 = m.Store(os.path.join(d, f"file{k}"), False, 0)
            try:
                s4.open()
                s4.translate(m.T_COLUMN, "i", "", ["zz"], True)
                s4.close()
            except Exception:  # noqa: BLE001
                pass
    finally:
        shutil.rmtree(d, ignore_errors=True)


# --------------------------------------------------------------------- arena
def drive_arena(m, rng: random.Random):
    """The parallel fragment loader and the cache-file reader over valid,
    truncated, bit-flipped and empty fragment files (8 loader threads)."""
    import numpy as np
    d = tempfile.mkdtemp()
    try:
        sw = 1 << 20
        m.write_zipf_fragments(d, 0, 3, 3 * sw, 3000, 2.0, 1.6, 50.0, rng.randrange(1 << 20), 4, 1, 200)
        good = [os.path.join(d, str(s)) for s in range(3)]
        blobs = [open(p, "rb").read() for p in good]
        paths = list(good)
        for k in range(24):
            b = rng.choice(blobs)
            if k % 3 == 0:
                b = b[:rng.randrange(len(b))]
            elif k % 3 == 1:
                b = mutate(rng, b[:4096], 6) + b[4096:]
            else:
                b = mutate(rng, b, 3)
            p = os.path.join(d, f"bad{k}")
            with open(p, "wb") as fh:
                fh.write(b)
            paths.append(p)
        open(os.path.join(d, "empty"), "wb").close()
        paths.append(os.path.join(d, "empty"))

        def load_set(ps, must_ok):
            try:
                ld = m.FragmentLoader(ps, 8)
                ld.scan()
                ld.rows()
                rowptr, sb, meta, cap, pb = ld.fill_index(0.0, 0)
                buf = np.zeros(int(pb[-1]) + 8, np.uint16)
                ld.fill_payload(0, len(ps), buf)
                return int(pb[-1])
            except Exception:  # noqa: BLE001
                if must_ok:
                    raise
                return -1
        total = load_set(good, True)
        assert total > 0
        for k in range(len(paths) - 3):
            load_set(good + [paths[3 + k]], False)
        run_threads([lambda: load_set(good, True) for _ in range(3)])
        caches = [p + ".cache" for p in good]
        cblobs = [open(p, "rb").read() for p in caches]
        for k in range(30):
            p = os.path.join(d, f"c{k}.cache")
            with open(p, "wb") as fh:
                fh.write(mutate(rng, rng.choice(cblobs), 4))
            caches.append(p)
        offs, ids, ok = m.read_cache_files(caches, 8)
        assert all(ok[:3])
        for b in blobs[:1] + [mutate(rng, blobs[0][:8192], 5) for _ in range(40)]:
            try:
                bm = m.Bitmap.from_bytes(b)
                bm.count()
            except Exception:  # noqa: BLE001
                pass
        # the import-request decoder over valid, truncated and mutated bodies
        # (hand-encoded ImportRequest: packed and unpacked ids, keys, unknown fields)
        def varint(v):
            out = bytearray()
            while True:
                b7 = v & 0x7F
                v >>= 7
                out.append(b7 | (0x80 if v else 0))
                if not v:
                    return bytes(out)

        def field(fn, wt, payload):
            return varint(fn << 3 | wt) + (varint(len(payload)) + payload if wt == 2 else payload)
        ids = b"".join(varint(rng.randrange(1 << 40)) for _ in range(500))
        body = (field(1, 2, b"i") + field(2, 2, b"f") + field(3, 0, varint(7)) + field(4, 2, ids) +
                field(5, 2, ids) + field(5, 0, varint(3)) + field(7, 2, b"key") + field(9, 0, varint(1)) +
                field(6, 2, b"".join(varint((1 << 64) - 5) for _ in range(3))))
        got = m.decode_import_request(body)
        assert got["Shard"] == 7 and len(got["RowIDs"]) == 500 and len(got["ColumnIDs"]) == 501
        for k in range(300):
            b = body[:rng.randrange(len(body))] if k % 2 else mutate(rng, body, 4)
            for vals in (False, True):
                try:
                    m.decode_import_request(b, vals)
                except Exception:  # noqa: BLE001 - RuntimeError is the contract
                    pass
    finally:
        shutil.rmtree(d, ignore_errors=True)


# ----------------------------------------------------------------------- pql
def drive_pql(m, rng: random.Random):
    """Parser + native Count planner over valid, mutated and deeply nested
    PQL, with the planner's worker threads and concurrent callers."""
    import numpy as np
    sys.path.insert(0, REPO)
    corpus = ["Count(Row(f=1))", "Count(Intersect(Row(f=1), Row(g=2)))",
              "Count(Union(Row(f=1), Row(f=2), Row(g=7))) Count(Difference(Row(f=3), Row(g=1)))",
              "Count(Xor(Row(f=1), Row(g=2)))", "TopN(f, Row(g=1), n=5)", 'Set(1, f="a\\"b")',
              "Count(Row(f > 10))", "Count(Row(-5 < f < 10))", "Row(f=1, from='2018-01-01T00:00', to='2019-01-01T00:00')",
              "Rows(f, previous=10, limit=5)", "GroupBy(Rows(f), Rows(g), limit=3)", "Options(Count(Row(f=1)), shards=[0,1])",
              "Count(Intersect(Row(f=1), Row(f=1)))", "Sum(Row(f=1), field=v)", "Count(Shift(Row(f=1), n=2))"]
    corpus += ["Count(Row(t=3, from='2020-01-01T00:00', to='2020-01-03T05:00')) Count(Row(t=4, to=2020-01-02))",
               "Count(Intersect(Row(f=2), Row(t=9, from=\"2020-01-01T00:00\")))"]
    fields = {"f": 0, "g": 1}
    dirs = [np.array(sorted(rng.sample(range(1000), 300)), np.uint64),
            np.array(sorted(rng.sample(range(1000), 200)), np.uint64)]
    ranges = {"t\x1f2020-01-01T00:00\x1f2020-01-03T05:00": [0, 1], "t\x1f\x01\x1f2020-01-02": [1],
              "t\x1f2020-01-01T00:00\x1f\x01": [0]}
    texts = list(corpus)
    for _ in range(600):
        texts.append(mutate(rng, rng.choice(corpus).encode(), 5).decode("latin-1"))
    for depth in (50, 500, 5000):
        texts.append("Count(" + "Intersect(" * depth + "Row(f=1)" + ")" * depth + ")")
        texts.append("Count(" + "Union(" * depth + "Row(f=1)" + ")" * (depth // 2))
    texts.append("Count(Row(f=" + "9" * 400 + "))")
    texts.append(" ".join(f"Count(Intersect(Row(f={rng.randrange(1200)}), Row(g={rng.randrange(1200)})))"
                          for _ in range(3000)))

    def one(t):
        for fn in (lambda: m.parse_calls(t), lambda: m.count_text_fields(t), lambda: m.count_text_ranges(t),
                   lambda: m.plan_count_text(t, fields, dirs, True, True, 4),
                   lambda: m.plan_count_text(t, fields, dirs, True, True, 4, ranges),
                   lambda: m.compile_counts([t, t], fields, dirs),
                   lambda: m.compile_count_text(t, fields, dirs)):
            try:
                fn()
            except Exception:  # noqa: BLE001 -- ParseError / ValueError are the contract
                pass
    for t in texts:
        one(t)
    big = texts[-1]
    got = m.plan_count_text(big, fields, dirs, True, True, 8)
    assert got is not None and got[0] == 3000
    run_threads([lambda: [m.plan_count_text(big, fields, dirs, True, True, 4) for _ in range(5)] for _ in range(4)])


def main():
    import faulthandler
    faulthandler.dump_traceback_later(float(os.environ.get("SAN_DRIVER_TIMEOUT", "400")), exit=True)
    moddir, mode = sys.argv[1], sys.argv[2]
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rng = random.Random(seed)
    name = {"httpd": "_httpd", "translate": "_translate", "arena": "_roaring", "pql": "_pql"}[mode]
    if mode == "pql":
        sys.path.insert(0, REPO)
    m = load(moddir, name)
    {"httpd": drive_httpd, "translate": drive_translate, "arena": drive_arena, "pql": drive_pql}[mode](m, rng)
    print(f"{mode}: ok", file=sys.stderr)


if __name__ == "__main__":
    main()
