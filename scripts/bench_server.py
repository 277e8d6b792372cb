#!/usr/bin/env python3
"""End-to-end serving throughput through the full HTTP server: concurrent
keep-alive clients each POST one `Count(Intersect(Row(f=a), Row(f=b)))` per
request to /index/i/query (HTTP parse, executor, group commit, GPU).

Index:
  --index disk    (default) the config-2 Zipf index written as Pilosa-format
                  fragment files (native/arena_io.cpp write_zipf_fragments),
                  opened by the server like any data dir (lazy holder, file
                  loader -> HBM); --cols / --rows size it (1B x 1M = config 2)
  --index import  a small index built through Field.import_bits (--shards)
Client:
  --client native (default) closed-loop C++ load generator (_httpd.load,
                  the role wrk plays), --conns connections
  --client python http.client in --procs processes x --threads threads
Every run checks a sample of HTTP responses against Executor.execute on the
same server.  Prints one JSON line; PILOSA_NATIVE_HTTP=0 serves through the
stdlib ThreadingHTTPServer instead of native/httpd.cpp."""
import argparse
import http.client
import json
import math
import multiprocessing as mp
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def client(port, queries, seconds, out):
    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    n, lat, i = 0, 0.0, 0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        q = queries[i % len(queries)]
        i += 1
        t0 = time.perf_counter()
        try:
            conn.request("POST", "/index/i/query", body=q.encode())
            r = conn.getresponse()
            body = r.read()
        except (http.client.HTTPException, OSError):
            conn.close()
            conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
            continue
        if r.status != 200:
            out.put(("err", body[:200]))
            return
        lat += time.perf_counter() - t0
        n += 1
    out.put(("ok", n, lat))


def worker(port, queries, seconds, threads, out):
    import threading
    ts = [threading.Thread(target=client, args=(port, queries[k::threads], seconds, out)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


def python_clients(port, queries, args):
    out = mp.Queue()
    ps = [mp.Process(target=worker, args=(port, queries[k::args.procs], args.seconds, args.threads, out))
          for k in range(args.procs)]
    for p in ps:
        p.start()
    res = [out.get() for _ in range(args.procs * args.threads)]
    for p in ps:
        p.join()
    errs = [r for r in res if r[0] != "ok"]
    n = sum(r[1] for r in res if r[0] == "ok")
    lat = sum(r[2] for r in res if r[0] == "ok")
    return {"requests": n, "errors": len(errs), "first_error": errs[0][1] if errs else b"",
            "mean_ms": 1000 * lat / max(n, 1), "clients": args.procs * args.threads}


def write_disk_index(base, args):
    tag = f"{args.cols}:{args.rows}:zipf1.6/50:8:seed1"
    marker = os.path.join(base, ".serve_data")
    if os.path.exists(marker) and open(marker).read() == tag:
        return {"reused": True}
    shutil.rmtree(base, ignore_errors=True)
    os.makedirs(base, exist_ok=True)
    from pilosa_amd import _roaring
    from pilosa_amd.models.field import FieldOptions
    from pilosa_amd.models.holder import Holder
    nshards = math.ceil(args.cols / (1 << 20))
    h = Holder(base).open()
    h.create_index("i", keys=False, track_existence=True)
    h.index("i").create_field("f", FieldOptions())
    h.close()
    fdir = os.path.join(base, "i", "f", "views", "standard", "fragments")
    os.makedirs(fdir, exist_ok=True)
    w = _roaring.write_zipf_fragments(fdir, 0, nshards, args.cols, args.rows, 8.0, 1.6, 50.0, 1, 16)
    with open(marker, "w") as fh:
        fh.write(tag)
    return {"files": int(w["shards"]), "bytes": int(w["bytes"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--index", choices=("disk", "import"), default="disk")
    ap.add_argument("--cols", type=int, default=1_000_000_000)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--shards", type=int, default=64, help="--index import: shards")
    ap.add_argument("--bits-per-col", type=float, default=2.0, help="--index import")
    ap.add_argument("--client", choices=("native", "python"), default="native")
    ap.add_argument("--conns", type=int, default=128)
    ap.add_argument("--client-threads", type=int, default=4)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--threads", type=int, default=16, help="python client threads per process")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--verify", type=int, default=256, help="HTTP responses checked against Executor.execute")
    ap.add_argument("--gpu", default="on")
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--batchers", default="",
                    help="comma list: one load run per Count group-commit thread count (native server)")
    args = ap.parse_args()
    import numpy as np

    from bench import zipf_rows
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger

    d = args.data_dir or tempfile.mkdtemp(prefix="pilosa_serve_", dir=os.environ.get("TMPDIR") or "/tmp")
    info = {}
    t0 = time.time()
    if args.index == "disk":
        info["write"] = write_disk_index(d, args)
        nrows = args.rows
    info["write_s"] = round(time.time() - t0, 1)
    t0 = time.time()
    srv = Server(d, bind="127.0.0.1:0", gpu=args.gpu, logger=CaptureLogger()).open()
    info["open_s"] = round(time.time() - t0, 1)
    try:
        if args.index == "import":
            idx = srv.holder.create_index("i")
            f = idx.create_field("f")
            rng = np.random.default_rng(7)
            ncols = args.shards << 20
            nbits = int(ncols * args.bits_per_col)
            t0 = time.time()
            f.import_bits(zipf_rows(rng, nbits, args.rows).astype(np.uint64),
                          rng.integers(0, ncols, size=nbits).astype(np.uint64))
            info["import_s"] = round(time.time() - t0, 1)
            nrows = args.rows
        qrng = np.random.default_rng(11)
        a, b = zipf_rows(qrng, 20000, nrows), zipf_rows(qrng, 20000, nrows)
        queries = [f"Count(Intersect(Row(f={x}), Row(f={y})))" for x, y in zip(a, b)]
        gpu = srv.executor.gpu
        # first query loads the index into HBM
        t0 = time.time()
        srv.executor.execute("i", queries[0])
        info["first_query_s"] = round(time.time() - t0, 1)
        if args.index == "import":
            for q in queries[:8]:
                got = srv.executor.execute("i", q).results[0]
                srv.executor.gpu = None
                want = srv.executor.execute("i", q).results[0]
                srv.executor.gpu = gpu
                assert got == want, (q, got, want)
        port = srv.uri.port
        sweep = [int(x) for x in args.batchers.split(",") if x] or [None]
        for nb in sweep:
            if nb is not None:
                srv.httpd.set_batchers(nb)
                time.sleep(0.5)
            run_load(srv, port, queries, args, info, nrows, gpu)
    finally:
        srv.close()
        if not args.data_dir:
            shutil.rmtree(d, ignore_errors=True)


def run_load(srv, port, queries, args, info, nrows, gpu):
    h = srv.httpd
    if hasattr(h, "count_s"):   # per-run group-commit stats
        h.batches = h.batched_requests = 0
        h.count_s = 0.0
    if gpu is not None:
        gpu.text_batches, gpu.text_prep_s, gpu.text_wait_s = 0, 0.0, 0.0
    t0 = time.perf_counter()
    if args.client == "native":
        from pilosa_amd import _httpd
        res = _httpd.load("127.0.0.1", port, "/index/i/query", [q.encode() for q in queries], args.conns,
                          args.client_threads, args.seconds, args.verify)
        res["clients"] = args.conns
    else:
        res = python_clients(port, queries, args)
    el = time.perf_counter() - t0
    # the sampled HTTP answers against the executor's own
    mism = 0
    samples = res.pop("samples", [])
    for k, body in samples:
        want = srv.executor.execute("i", queries[k]).results
        if json.loads(body)["results"] != want:
            mism += 1
    st = srv.httpd.stats() if hasattr(srv.httpd, "stats") else None
    co = srv.executor._coalescer
    fe = res.pop("first_error", b"")
    print(json.dumps({
        "metric": "HTTP Count(Intersect) requests/s", "value": round(res["requests"] / args.seconds, 1),
        "clients": res["clients"], "client": args.client, "seconds": args.seconds,
        "mean_latency_ms": round(res["mean_ms"], 3),
        "p50_ms": round(res.get("p50_ms", 0), 3), "p99_ms": round(res.get("p99_ms", 0), 3),
        "errors": res["errors"], "first_error": fe[:300].decode(errors="replace") if fe else "",
        "verified": len(samples), "mismatches": mism,
        "server": type(srv.httpd).__name__, "server_stats": st,
        "gpu": gpu is not None, "coalescer": {"batches": co.batches, "batched": co.batched,
                                              "fallbacks": co.fallbacks} if co else None,
        "index": args.index, "cols": args.cols if args.index == "disk" else args.shards << 20, "rows": nrows,
        "setup": info, "wall_s": round(el, 1)}), flush=True)


if __name__ == "__main__":
    main()
