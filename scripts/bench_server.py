#!/usr/bin/env python3
"""End-to-end serving throughput through the full HTTP server: concurrent
clients each POST one `Count(Intersect(Row(f=a), Row(f=b)))` per request to
/index/i/query (PQL parse, executor, cross-request coalescing, GPU).

Clients run in separate processes (keep-alive HTTP/1.1 connections) so they
do not share the server's interpreter.  Prints one JSON line; run with
PILOSA_COALESCE=0 for the one-launch-per-request baseline."""
import argparse
import http.client
import json
import multiprocessing as mp
import os
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=64)
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--bits-per-col", type=float, default=2.0)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--threads", type=int, default=16, help="client threads per process")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--gpu", default="on")
    args = ap.parse_args()
    import numpy as np

    from bench import zipf_rows
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger

    d = tempfile.mkdtemp()
    srv = Server(d, bind="127.0.0.1:0", gpu=args.gpu, logger=CaptureLogger()).open()
    try:
        idx = srv.holder.create_index("i")
        f = idx.create_field("f")
        rng = np.random.default_rng(7)
        ncols = args.shards << 20
        nbits = int(ncols * args.bits_per_col)
        t0 = time.time()
        f.import_bits(zipf_rows(rng, nbits, args.rows).astype(np.uint64),
                      rng.integers(0, ncols, size=nbits).astype(np.uint64))
        t_import = time.time() - t0
        qrng = np.random.default_rng(11)
        a, b = zipf_rows(qrng, 20000, args.rows), zipf_rows(qrng, 20000, args.rows)
        queries = [f"Count(Intersect(Row(f={x}), Row(f={y})))" for x, y in zip(a, b)]
        # correctness spot check against the host path, and warm-up
        gpu = srv.executor.gpu
        for q in queries[:8]:
            got = srv.executor.execute("i", q).results[0]
            srv.executor.gpu = None
            want = srv.executor.execute("i", q).results[0]
            srv.executor.gpu = gpu
            assert got == want, (q, got, want)
        # single-thread costs: one request through the executor (parse + plan +
        # launch), and one 256-call batch through the coalescer's batch path
        from pilosa_amd.pql import parse_string
        t0 = time.perf_counter()
        for q in queries[:200]:
            srv.executor.execute("i", q)
        micro = {"execute_ms": round((time.perf_counter() - t0) / 200 * 1000, 3)}
        t0 = time.perf_counter()
        for q in queries[:200]:
            parse_string(q)
        micro["parse_ms"] = round((time.perf_counter() - t0) / 200 * 1000, 3)
        calls = [parse_string(q).calls[0] for q in queries[:256]]
        shards = srv.holder.index("i").available_shards()
        if gpu is not None:
            gpu.try_count_batch("i", calls, shards)
            t0 = time.perf_counter()
            for _ in range(5):
                gpu.try_count_batch("i", calls, shards)
            micro["batch256_ms"] = round((time.perf_counter() - t0) / 5 * 1000, 3)
        port = srv.uri.port
        out = mp.Queue()
        ps = [mp.Process(target=worker, args=(port, queries[k::args.procs], args.seconds, args.threads, out))
              for k in range(args.procs)]
        t0 = time.perf_counter()
        for p in ps:
            p.start()
        res = [out.get() for _ in range(args.procs * args.threads)]
        el = time.perf_counter() - t0
        for p in ps:
            p.join()
        errs = [r for r in res if r[0] != "ok"]
        n = sum(r[1] for r in res if r[0] == "ok")
        lat = sum(r[2] for r in res if r[0] == "ok")
        co = srv.executor._coalescer
        print(json.dumps({"metric": "HTTP Count(Intersect) requests/s", "value": round(n / args.seconds, 1),
                          "clients": args.procs * args.threads, "seconds": args.seconds,
                          "mean_latency_ms": round(1000 * lat / max(n, 1), 2), "errors": errs[:3],
                          "gpu": gpu is not None, "coalesce": srv.executor.coalesce,
                          "coalescer": {"batches": co.batches, "batched": co.batched,
                                        "fallbacks": co.fallbacks} if co else None,
                          "micro": micro, "shards": args.shards, "bits": nbits, "import_s": round(t_import, 1),
                          "wall_s": round(el, 1)}), flush=True)
    finally:
        srv.close()


if __name__ == "__main__":
    main()
