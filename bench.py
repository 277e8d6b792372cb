#!/usr/bin/env python3
"""Headline benchmark: PQL queries/sec on a 1M-row x 1B-column set field.

Config (BASELINE.json config 2/3): index ``i`` with one set field ``f``;
1,000,000 rows x 1,000,000,000 columns (954 shards of 2^20 columns); every
column holds 8 bits whose rows follow the reference's Zipf(s=1.6, v=50) row
generator (fragment_internal_test.go:2377-2460) -> ~8e9 set bits, random-init
synthetic data generated deterministically per shard (no dataset download).

A *step* is one batch of B concurrent PQL queries
``Count(Intersect(Row(f=a), Row(f=b)))`` with a, b drawn from the same Zipf
law (hot rows are queried most, as in production).  Two modes:

* ``--mode disk`` (default): the product path.  The index is written as 954
  Pilosa-format fragment files (one per shard) into a data dir, opened by a
  ``Holder`` (lazy fragments), and its view is loaded from the files straight
  into HBM (native/arena_io.cpp, ops/loader.py).  Every step is one request
  ``Executor.execute("i", "<B Count calls>")`` through the same entry point the
  HTTP handler uses (PQL text -> native compile -> batched HIP kernel ->
  results); ``--clients`` request threads keep the GPU busy while the next
  request is prepared.
* ``--mode synthetic``: the kernel harness.  The arena is generated in memory
  and batches go to the engine directly (no holder, no executor).

Both modes re-derive a sample of the counts (64 queries x 8 shards) on the host
roaring core and report ``verified`` in ``extra``.  With N GPUs each rank owns a
contiguous 1/N of the shards (strong scaling: the index size is fixed) and the
per-batch counts are summed with an RCCL all-reduce.  ``value`` = total
queries/sec.

Run: python bench.py [--gpus N --steps K --warmup W --batch B --mode disk|synthetic]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

TOTAL_COLS = 1_000_000_000
NROWS = 1_000_000
SHARD_WIDTH = 1 << 20


_COMM = None  # parallel/collectives.Comm when WORLD_SIZE > 1


def all_reduce(t, op=None):
    """Sum (or ``op``) a device tensor over the ranks (RCCL; the gloo rehearsal
    mode goes through host copies)."""
    return _COMM.all_reduce(t, op)


_T0 = time.time()


def log(msg):
    """Progress line on stderr (long GPU runs must keep writing)."""
    print(f"[bench {time.time() - _T0:7.1f}s r{os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def zipf_rows(rng, n, nrows=NROWS, s=1.6, v=50.0):
    # inverse-CDF sampling of P(k) ~ (v+k)^-s, k in [0, nrows)
    k = np.arange(nrows, dtype=np.float64)
    w = (v + k) ** (-s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.searchsorted(cdf, rng.random(n)).astype(np.int64)


def bench_topn(args, view, eng, rng, world, rank, dev):
    """TopN batches on the device rank caches (pilosa_amd/ops/topn.py):
      cache:  TopN(f, n=100)            -- ranked-cache TopN (BASELINE config 3)
      src:    TopN(f, Row(f=a), n=100)  -- src-filtered, a from the 1000 hottest rows
    Multi-GPU: phase-1 pairs are all-gathered and summed by id, the ids=
    re-count is all-reduced (RCCL), as the reference coordinator does over HTTP."""
    import torch
    import torch.distributed as dist

    from pilosa_amd.ops.planner import BenchPlanner
    from pilosa_amd.ops.topn import (DeviceRankCache, finish_topn, topn_cache_phase1, topn_cache_phase2_counts,
                                     topn_phase1, topn_phase2_counts)
    from pilosa_amd.pql import parse_string

    from pilosa_amd.ops.topn_index import DeviceTopNIndex

    n = 100
    t0 = time.perf_counter()
    cache = DeviceRankCache.from_view(view, k=args.topn_cache, keep_row_counts=True)
    torch.cuda.synchronize(dev)
    t_cache = time.perf_counter() - t0
    planner = BenchPlanner({"f": view})
    # node-wide row-id space of the TopN accumulators (identical on every rank)
    space = np.asarray(view.rows, dtype=np.uint64)
    if world > 1:
        import torch as _t
        parts = _COMM.all_gather_var(_t.from_numpy(space.view(np.int64).copy()).to(dev))
        space = np.unique(np.concatenate([p.cpu().numpy().view(np.uint64) for p in parts]))
    t0 = time.perf_counter()
    tindex = DeviceTopNIndex(view, cache, space=space)
    torch.cuda.synchronize(dev)
    t_index = time.perf_counter() - t0

    def merge(totals):
        # phase-1 pairs summed by (query, id) over ranks: (q, id, count)
        # triples all-gathered as int64 tensors
        if world == 1:
            return totals
        from pilosa_amd.parallel.collectives import pairs_to_arrays
        q, ids, cnt = pairs_to_arrays(totals)
        flat = torch.from_numpy(np.stack([q, ids, cnt], axis=1).reshape(-1)).to(dev)
        parts = [p.cpu().numpy().reshape(-1, 3) for p in _COMM.all_gather_var(flat)]
        allp = np.concatenate(parts) if parts else np.zeros((0, 3), np.int64)
        out = [dict() for _ in totals]
        for qq, i, c in allp.tolist():
            out[qq][i] = out[qq].get(i, 0) + c
        return out

    def allreduce(exact, ids):
        if world == 1:
            return exact
        flat = torch.from_numpy(np.concatenate(exact) if exact else np.zeros(0, np.int64)).to(dev)
        all_reduce(flat)
        flat = flat.cpu().numpy()
        o, out = 0, []
        for q in range(len(ids)):
            out.append(flat[o:o + len(ids[q])])
            o += len(ids[q])
        return out

    def run_cache(qs):
        # device phase 1 (scatter-add of cache prefixes) + device ids= re-count
        calls = [parse_string(q).calls[0] for q in qs]
        return tindex.topn_nosrc(cache.row_counts, [c.uint_arg("n")[0] for c in calls], [1] * len(calls),
                                 comm=_COMM if world > 1 else None)

    def run_cache_host(qs):
        calls = [parse_string(q).calls[0] for q in qs]
        totals = merge([topn_cache_phase1(cache, c.uint_arg("n")[0]) for c in calls])
        ids = [sorted(t) for t in totals]
        exact = allreduce([topn_cache_phase2_counts(cache, view, i) for i in ids], ids)
        return [finish_topn(ids[q], exact[q], n) for q in range(len(qs))]

    def run_src(qs):
        # slot-index path: LDS histogram + in-kernel heap walk (ops/topn_index.py)
        calls = [parse_string(q).calls[0] for q in qs]
        srcs = [planner.plan(c.children[0]) for c in calls]
        ns = [c.uint_arg("n")[0] for c in calls]
        return tindex.topn(eng, srcs, ns, [1] * len(srcs), comm=_COMM if world > 1 else None)

    def run_src_pairs(qs):
        # pair-count path with the native heap replay (ops/topn.py), for comparison
        calls = [parse_string(q).calls[0] for q in qs]
        srcs = [planner.plan(c.children[0]) for c in calls]
        totals = merge(topn_phase1(eng, view, cache, srcs, n=n))
        ids = [sorted(t) for t in totals]
        exact = allreduce(topn_phase2_counts(eng, view, srcs, ids), ids)
        return [finish_topn(ids[q], exact[q], n) for q in range(len(qs))]

    def timed(fn, queries, B, batches):
        fn(queries[:B])  # warmup
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        res = None
        for b in range(1, batches + 1):
            res = fn(queries[b * B:(b + 1) * B])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        elt = torch.tensor([el], dtype=torch.float64, device=dev)
        if world > 1:
            all_reduce(elt, op=dist.ReduceOp.MAX)
        el = float(elt.item())
        return {"qps": round(B * batches / el, 2), "ms_per_batch": round(el / batches * 1000, 2), "batch": B,
                "sample_top3": [(p.id, p.count) for p in res[0][:3]] if res and res[0] else []}

    B, nb = args.topn_batch, args.topn_batches
    out = {"n": n, "cache_k": args.topn_cache, "cache_build_s": round(t_cache, 2),
           "slot_index_build_s": round(t_index, 2), "slot_index_bytes": tindex.nbytes()}
    cq = [f"TopN(f, n={n})"] * (B * (nb + 1))
    out["cache"] = timed(run_cache, cq, B, nb)
    out["cache_paths_agree"] = [[(p.id, p.count) for p in r] for r in run_cache(cq[:B])] == \
        [[(p.id, p.count) for p in r] for r in run_cache_host(cq[:B])]
    hot = zipf_rows(rng, B * (nb + 1), 1000)
    src_q = [f"TopN(f, Row(f={a}), n={n})" for a in hot]
    out["src"] = timed(run_src, src_q, B, nb)
    if args.topn_pairs_batches > 0:
        nbp = min(nb, args.topn_pairs_batches)
        res_idx = run_src(src_q[B:2 * B])
        res_pairs = run_src_pairs(src_q[B:2 * B])
        out["src_pairs"] = timed(run_src_pairs, src_q, B, nbp)
        out["src_paths_agree"] = [[(p.id, p.count) for p in r] for r in res_idx] == \
            [[(p.id, p.count) for p in r] for r in res_pairs]
    return out


def bench_topn_exec(args, holder, ex, gpu, shards, fdir, world, rank, dev):
    """BASELINE config 3 through the product path: TopN requests go through
    ``Executor.execute`` on the lazily opened index (PQL text -> device rank
    caches from the fragments' .cache files + HBM arena -> both TopN phases on
    the device, ops/topn_exec.py).  ``cache``: TopN(f, n=100); ``src``:
    TopN(f, Row(f=a), n=100) with a from the 1000 hottest rows; every request
    carries ``--topn-batch`` calls, ``--clients`` request threads.  With N
    GPUs every rank runs the same requests over its shard range and the
    candidates / re-counts merge over RCCL inside the device path (one
    client thread: collectives in request order).  After the timed runs a
    sample of (query, shard) phase-1 answers is re-derived by the host
    ``fragment.top`` (which loads those fragments)."""
    import resource
    import threading

    import torch
    import torch.distributed as dist

    from pilosa_amd.models.fragment import TopOptions
    from pilosa_amd.pql import parse_string

    n = 100
    B, nb = args.topn_batch, args.topn_batches
    # request threads of the TopN phase: with 2, the two threads' Python halves
    # convoy on the GIL (cache-only 0.358 ms/request vs 0.216 with 1 and 0.232
    # with 3, profiles/r05_topn/prof_topn_wide_threads.log)
    clients = max(1, args.topn_clients) if world == 1 else 1
    if world > 1:
        gpu.comm = _COMM
    rng = np.random.default_rng(99)
    out = {"path": "Executor.execute(PQL TopN text), lazy holder, device rank caches from .cache files",
           "n": n, "cache_k": args.topn_cache, "batch": B, "clients": clients}

    def timed(texts, first, profile="", nclients=None, warm=1):
        # ``warm`` untimed requests first (the first builds rank caches / slot
        # index / prefix memos), then the rest timed with ``nclients`` request
        # threads; ``profile``: folded stacks of every thread over the first
        # 0.3 s of the timed run
        nclients = clients if nclients is None else nclients
        done = [None] * len(texts)
        lat = [0.0] * len(texts)       # per-request wall time (s)
        err = []
        nxt = [0]
        lock = threading.Lock()

        def client(lo, hi):
            while True:
                with lock:
                    i = nxt[0]
                    if i >= hi or err:
                        return
                    nxt[0] += 1
                try:
                    t_r = time.perf_counter()
                    done[i] = ex.execute("i", texts[i], shards=shards).results
                    lat[i] = time.perf_counter() - t_r
                except BaseException as e:  # noqa: BLE001
                    err.append(e)
                    return
        t0 = time.perf_counter()
        done[0] = ex.execute("i", texts[0], shards=shards).results
        torch.cuda.synchronize(dev)
        first["first_request_s"] = round(time.perf_counter() - t0, 2)
        for i in range(1, warm):
            done[i] = ex.execute("i", texts[i], shards=shards).results
        torch.cuda.synchronize(dev)
        # what the server's Refreezer does after warm-up: the rank caches and
        # slot index the first request built leave the collector's walk
        from pilosa_amd.utils import gctune
        gctune.freeze_long_lived()
        log(f"topn: first request {first['first_request_s']} s")
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        nxt[0] = warm
        prof = None
        gc_t = [0.0, 0, None]   # pause seconds, collections, start of the current one
        if profile:
            import gc

            def gc_cb(phase, info):
                if phase == "start":
                    gc_t[2] = time.perf_counter()
                elif gc_t[2] is not None:
                    gc_t[0] += time.perf_counter() - gc_t[2]
                    gc_t[1] += 1
            gc.callbacks.append(gc_cb)
            from pilosa_amd.utils import pprof
            prof_out = {}
            prof = threading.Thread(target=lambda: prof_out.setdefault("p", pprof.cpu_profile(0.3, 500)), daemon=True)
            prof.start()
        t0 = time.perf_counter()
        cprof = os.environ.get("PILOSA_BENCH_CPROFILE", "") if profile else ""
        if cprof and nclients == 1:
            # deterministic profile of the one request thread (host cost per call)
            import cProfile
            import io
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            client(warm, len(texts))
            pr.disable()
            sio = io.StringIO()
            pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(45)
            with open(cprof, "w") as fh:
                fh.write(sio.getvalue())
        else:
            ts = [threading.Thread(target=client, args=(warm, len(texts))) for _ in range(nclients)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        if err:
            raise err[0]
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if prof is not None:
            gc.callbacks.remove(gc_cb)
            first["gc_pause_s"] = round(gc_t[0], 4)
            first["gc_collections"] = gc_t[1]
            prof.join()
            with open(profile, "w") as fh:
                fh.write(prof_out.get("p", ""))
        elt = torch.tensor([el], dtype=torch.float64, device=dev)
        if world > 1:
            all_reduce(elt, op=dist.ReduceOp.MAX)
        el = float(elt.item())
        last = done[-1]
        lt = np.sort(np.asarray(lat[warm:])) * 1000
        first.update({"qps": round(B * (len(texts) - warm) / el, 2), "ms_per_request": round(el / (len(texts) - warm) * 1000, 2),
                      "timed_requests": len(texts) - warm, "timed_s": round(el, 3),
                      "p50_ms": round(float(lt[len(lt) // 2]), 2) if len(lt) else None,
                      "p99_ms": round(float(lt[min(len(lt) - 1, int(len(lt) * 0.99))]), 2) if len(lt) else None,
                      "request_threads": nclients, "warm_requests": warm,
                      "sample_top3": [(p.id, p.count) for p in last[0][:3]] if last and last[0] else []})
        return done

    l0 = gpu.launches
    log("topn: cache-only requests (distinct calls)")
    # every call of every request distinct: n and threshold vary, so no
    # phase-2 re-count or candidate set is shared between calls by repetition
    nbc = max(nb, args.topn_cache_batches)   # cache-only requests are ~1 ms: a longer window
    W = 8   # untimed: the prefix-bucket memos of the rank caches are built once
    cache_calls = _wide_topn_calls(B * (nbc + W), seed=17)
    cache_q = [" ".join(cache_calls[i * B:(i + 1) * B]) for i in range(nbc + W)]
    out["cache"] = {"calls": f"TopN(f, n=log-uniform 1..1000, threshold one of {len(WIDE_THRESHOLDS)} values "
                             "1..50000), random per call: distinct within and across requests"}
    # cache-only requests are host-bound Python: one request thread (2-3 threads
    # convoy on the GIL, profiles/r05_topn/prof_topn_wide_threads.log)
    res_cache = timed(cache_q, out["cache"], os.environ.get("PILOSA_BENCH_TOPN_PROFILE", ""),
                      nclients=args.topn_cache_clients, warm=W)
    log("topn: cache-only requests (round-4 cycling set: 4 n x 4 thresholds)")
    cyc = _distinct_topn_calls(B * (nbc + W))
    out["cache_cycling"] = {"calls": "TopN(f, n in {10,50,100,500} + offset, threshold in {1,1000,5000,20000})"}
    timed([" ".join(cyc[i * B:(i + 1) * B]) for i in range(nbc + W)], out["cache_cycling"],
          nclients=args.topn_cache_clients, warm=W)
    log("topn: cache-only requests (the same call repeated, round-3 figure)")
    out["cache_repeated"] = {}
    timed([" ".join([f"TopN(f, n={n})"] * B)] * (nbc + W), out["cache_repeated"], nclients=args.topn_cache_clients,
          warm=W)
    # untimed: the first request builds the slot index; the next ones settle
    # the device allocator's segments for this phase's buffers
    WS = 3
    nbs = max(nb, args.topn_src_batches)   # >= 200 requests: ~2-3 s timed
    hot = zipf_rows(rng, B * (nbs + WS), 1000)
    src_calls = [f"TopN(f, Row(f={a}), n={n})" for a in hot]
    src_q = [" ".join(src_calls[i * B:(i + 1) * B]) for i in range(nbs + WS)]
    out["src"] = {}
    log("topn: src requests")
    ib0 = gpu.topn_index_build_s if hasattr(gpu, "topn_index_build_s") else None
    res_src = timed(src_q, out["src"], warm=WS)
    if ib0 is not None:
        out["src"]["slot_index_build_s"] = round(gpu.topn_index_build_s - ib0, 3)
    # the same requests from ONE thread (sequential latency, no overlap)
    tq = src_q[WS:WS + 30]
    torch.cuda.synchronize(dev)
    t_1 = time.perf_counter()
    for q in tq:
        ex.execute("i", q, shards=shards)
    torch.cuda.synchronize(dev)
    out["src"]["single_thread_ms_per_request"] = round((time.perf_counter() - t_1) / max(len(tq), 1) * 1000, 2)
    log(f"topn: src {out['src']}")
    log("topn: verify")
    out["device_launches"] = gpu.launches - l0
    out["batches_declined"] = ex.topn_batch_declined
    out["host_fallbacks"] = ex.gpu_faults
    view = holder.view("i", "f", "standard")
    out["fragments_cold_after_topn"] = sum(f.is_cold() for f in view.all_fragments())
    out["fragments"] = len(view.all_fragments())
    out["peak_host_rss_gb_after_topn"] = round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)
    key = ("i", "f", tuple(shards))
    rc = gpu._rank_cache_map.get(key, (None, None))[1]
    tix = gpu._topn_indexes.get(key, (None, None, None))[1]
    out["rank_cache_k"] = rc.K if rc is not None else 0
    out["rank_cache_cold_shards"] = rc.cold_shards if rc is not None else 0
    out["slot_index_bytes"] = tix.nbytes() if tix is not None else 0
    if world == 1 and shards:
        # a write burst into one shard (an existing row gains 8k bits and
        # climbs that shard's rank cache): the next src request refreshes the
        # slot index in place (only that shard re-indexed) instead of falling
        # back to the pair-count path while a full rebuild is throttled
        fw = holder.index("i").field("f")
        wcols = np.uint64(shards[0]) * np.uint64(SHARD_WIDTH) + np.arange(0, SHARD_WIDTH, 128, dtype=np.uint64)
        r0, d0 = gpu.topn_index_refreshes, ex.topn_batch_declined
        t0 = time.perf_counter()
        fw.import_bits(np.full(len(wcols), NROWS - 1, np.uint64), wcols)
        t1 = time.perf_counter()
        ex.execute("i", src_q[1], shards=shards)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        tt = [time.perf_counter()]
        for q in src_q[2:6]:
            ex.execute("i", q, shards=shards)
        torch.cuda.synchronize(dev)
        tt.append(time.perf_counter())
        out["after_write"] = {"bits": int(len(wcols)), "row": NROWS - 1, "shard": shards[0],
                              "import_s": round(t1 - t0, 3), "first_src_request_s": round(t2 - t1, 3),
                              "next_src_ms_per_request": round((tt[1] - tt[0]) / 4 * 1000, 2),
                              "index_refreshes": gpu.topn_index_refreshes - r0,
                              "batches_declined": ex.topn_batch_declined - d0}
        log(f"topn: after a write burst {out['after_write']}")
    gpu.comm = None
    # correctness: per-shard phase-1 answers (device map step over one shard) vs
    # the host fragment.top on sampled shards (this loads those fragments)
    if args.verify > 0 and shards:
        sel = sorted(set(np.linspace(0, len(shards) - 1, min(4, len(shards))).astype(int).tolist()))
        calls = [parse_string(f"TopN(f, n={n})").calls[0]] + \
            [parse_string(c).calls[0] for c in cache_calls[:3]] + \
            [parse_string(c).calls[0] for c in src_calls[B:B + 3]]
        bad = 0
        for si in sel:
            s = shards[si]
            frag = holder.fragment("i", "f", "standard", s)
            for c in calls:
                dev_pairs = sorted((p.id, p.count) for p in gpu.topn("i", c, [s]))
                src = ex.bitmap_call_shard("i", c.children[0], s) if c.children else None
                _, cn, _, cth, _, _, _ = ex.topn_params("i", c)   # each call's own n and threshold
                host = frag.top(TopOptions(n=cn, src=src, min_threshold=max(1, cth)))
                if dev_pairs != sorted((p.id, p.count) for p in host):
                    bad += 1
        # and the fused batch answers equal the two-phase map/reduce on the device
        agree = [[(p.id, p.count) for p in r] for r in res_src[-1][:2] + res_cache[-1][:4]] == \
            [[(p.id, p.count) for p in ex._topn("i", parse_string(c).calls[0], shards, _exec_opts())]
             for c in src_calls[(len(src_q) - 1) * B:(len(src_q) - 1) * B + 2] + cache_calls[(len(cache_q) - 1) * B:(len(cache_q) - 1) * B + 4]] if world == 1 else None
        out["verify"] = {"shards_checked": len(sel), "queries_per_shard": len(calls), "mismatches": bad,
                         "fused_equals_two_phase": agree, "verified": bad == 0 and agree is not False}
    return out


TOPN_NS = (10, 50, 100, 500)
TOPN_THRESHOLDS = (1, 1000, 5000, 20000)


# >= 64 distinct thresholds, geometric from 1 to 50000
WIDE_THRESHOLDS = tuple(sorted({max(1, int(round(50000 ** (i / 79)))) for i in range(80)}))


def _wide_topn_calls(k: int, seed: int = 17):
    """k cache-only TopN calls with n log-uniform over 1..1000 and the
    threshold drawn from WIDE_THRESHOLDS (>= 64 values), independently per
    call: no candidate set, threshold total or re-count repeats by
    construction across a run."""
    rng = np.random.default_rng(seed)
    ns = np.exp(rng.uniform(0, np.log(1000), size=k)).astype(np.int64) + 1
    th = rng.choice(np.asarray(WIDE_THRESHOLDS), size=k)
    return [f"TopN(f, n={int(n)}, threshold={int(t)})" for n, t in zip(ns, th)]


def _distinct_topn_calls(k: int):
    """k cache-only TopN calls, no two alike within a request: n and
    threshold cycle through TOPN_NS x TOPN_THRESHOLDS, and the n values get
    a per-call offset so every (n, threshold) pair differs."""
    out = []
    for i in range(k):
        n = TOPN_NS[i % len(TOPN_NS)] + (i // 16) % 7
        t = TOPN_THRESHOLDS[(i // len(TOPN_NS)) % len(TOPN_THRESHOLDS)]
        out.append(f"TopN(f, n={n}, threshold={t})")
    return out


def _exec_opts():
    from pilosa_amd.executor import ExecOptions
    return ExecOptions()


def bench_cpu_host(args, ra, rb, nshards, nq=256):
    """CPU stand-in for the reference (no published numbers).

    Runs the same Count(Intersect(Row, Row)) queries through the host C++
    roaring core the way the reference's executor does per shard (row
    extraction from the fragment, then container-pair intersectionCount;
    reference executor.go executeCount -> fragment.row ->
    roaring IntersectionCount) on the first ``args.cpu_baseline_shards``
    shards, single-threaded, and extrapolates to all shards.  The reference
    runs one goroutine per shard, so ``qps_per_core`` times the host core
    count is its ideal-scaling ceiling on that host."""
    from pilosa_amd import _roaring
    k = min(args.cpu_baseline_shards, nshards)
    arena = _roaring.gen_zipf_arena(0, k, args.cols, args.rows, 8.0, 1.6, 50.0, 1, args.threads)
    frags = [_roaring.arena_shard_bitmap(*arena, s) for s in range(k)]
    del arena
    w = SHARD_WIDTH
    n = min(nq, len(ra))
    t0 = time.perf_counter()
    total = 0
    for a, b in zip(ra[:n], rb[:n]):
        a, b = int(a), int(b)
        for f in frags:
            r1 = f.offset_range(0, a * w, (a + 1) * w)
            r2 = f.offset_range(0, b * w, (b + 1) * w)
            total += r1.intersection_count(r2)
    dt = time.perf_counter() - t0
    per_q_all_shards = dt / n * (nshards / k)
    # our host fallback (Executor.count_shard): the rows counted in place
    t0 = time.perf_counter()
    total2 = 0
    for a, b in zip(ra[:n], rb[:n]):
        a, b = int(a), int(b)
        for f in frags:
            total2 += f.range_intersection_count(a * w, f, b * w, w)
    per_q_inplace = (time.perf_counter() - t0) / n * (nshards / k)
    return {"shards_timed": k, "queries": n, "threads": 1, "checksum": total,
            "ms_per_query_all_shards_1core": round(per_q_all_shards * 1000, 3),
            "qps_per_core": round(1.0 / per_q_all_shards, 3),
            "host_fallback_in_place": {"checksum_matches": total2 == total,
                                       "ms_per_query_all_shards_1core": round(per_q_inplace * 1000, 3),
                                       "qps_per_core": round(1.0 / per_q_inplace, 3)}}


def _timed(fn, reps, world, dev):
    """(seconds per call, max over ranks, last result) with a device sync."""
    import torch
    import torch.distributed as dist
    fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    out = None
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize(dev)
    el = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=dev)
    if world > 1:
        all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item()), out


def bench_bsi(args, world, rank, dev):
    """BASELINE config 4: a BSI int field over the same 1B columns (half of
    them hold a value uniform in [-1000, 1e6], bit depth 20): Sum, range
    counts, Min/Max, and Sum for a batch of 32 filters on the per-filter
    VALU kernel vs the bit-plane matrix product on the matrix cores
    (ops/bsi.py).  Every rank evaluates its shard range; sums/counts are
    all-reduced."""
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.bsi import bsi_sum_matrix
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf

    nshards = math.ceil(args.cols / SHARD_WIDTH)
    lo, hi = nshards * rank // world, nshards * (rank + 1) // world
    depth, vmin, vmax = 20, -1000, 1_000_000
    t0 = time.time()
    arena = _roaring.gen_bsi_arena(lo, hi, args.cols, depth, 0.5, vmin, vmax, 7, args.threads)
    bv = DeviceView(*arena, dev, shards=list(range(lo, hi)))
    farena = _roaring.gen_zipf_arena(lo, hi, args.cols, 1000, 1.0, 1.6, 50.0, 11, args.threads)
    fv = DeviceView(*farena, dev, shards=list(range(lo, hi)))
    del arena, farena
    gen_s = time.time() - t0
    eng = GpuEngine(dev)
    rng = np.random.default_rng(5)
    reps = args.config_reps
    res = {"config": "BSI int field v, 1B cols, depth 20, fill 0.5, values [-1000, 1e6]", "gen_s": round(gen_s, 1),
           "hbm_bytes_per_gpu": bv.nbytes(), "queries": {}}

    def red(*ts):
        t = torch.stack([x.reshape(-1)[0].to(torch.int64) for x in ts])
        if world > 1:
            all_reduce(t)
        return [int(x) for x in t.cpu().tolist()]

    def q_sum():
        s, n = eng.bsi_sum_async([None], bv, depth)
        return red(s, n)

    def q_gt():
        return red(eng.bsi_range_count_async(bv, depth, ">", int(rng.integers(0, vmax))))[0]

    def q_between():
        a = int(rng.integers(0, 900_000))
        return red(eng.bsi_range_count_async(bv, depth, "between", a, a + 50_000))[0]

    def q_minmax():
        k = eng.bsi_minmax(None, bv, depth)
        return int(k[..., 4].max())

    FB = 32
    frows = [int(r) for r in rng.integers(0, 200, size=FB)]
    filters = [Leaf(fv, r) for r in frows]

    def q_batch_valu():
        s, n = eng.bsi_sum_async(filters, bv, depth, matrix=False)
        t = torch.cat([s, n])
        if world > 1:
            all_reduce(t)
        return t.cpu().numpy()

    def q_batch_matrix(mode):
        def fn():
            s, n = bsi_sum_matrix(eng, filters, bv, depth, mode=mode)
            t = torch.cat([s, n])
            if world > 1:
                all_reduce(t)
            return t.cpu().numpy()
        return fn

    for name, fn in (("Sum(field=v)", q_sum), ("Count(Row(v > x))", q_gt), ("Count(Row(v >< [a,b]))", q_between),
                     ("Max(field=v)", q_minmax)):
        dt, out = _timed(fn, reps, world, dev)
        res["queries"][name] = {"ms": round(dt * 1000, 3), "qps": round(1 / dt, 1), "sample": out}
    dt_v, out_v = _timed(q_batch_valu, reps, world, dev)
    res["queries"][f"Sum(Row(f=r), field=v) x{FB} per-filter kernel"] = {
        "ms_per_batch": round(dt_v * 1000, 3), "qps": round(FB / dt_v, 1)}
    agree = True
    for mode, label in ((4, "MFMA 32x64 K-sliced tiles"), (3, "MFMA 64x64 tiles"), (2, "MFMA 128x128 tiles"),
                        (0, "VALU popcount tiles")):
        dt_m, out_m = _timed(q_batch_matrix(mode), reps, world, dev)
        res["queries"][f"Sum(Row(f=r), field=v) x{FB} bit-plane matrix, {label}"] = {
            "ms_per_batch": round(dt_m * 1000, 3), "qps": round(FB / dt_m, 1)}
        agree = agree and bool(np.array_equal(out_v, out_m))
    res["batched_sum_paths_agree"] = agree
    s, n = q_sum()
    res["check"] = {"count": n, "mean": s / max(n, 1), "expected_count": args.cols * 0.5,
                    "expected_mean": (vmax + vmin) / 2}
    del bv, fv
    torch.cuda.empty_cache()
    return res


def bench_time_union(args, world, rank, dev):
    """BASELINE config 5: a time field's range query over YMDH views =
    Count(Union) of the covering views (here 2 day views + 5 hour views of a
    1M-row Zipf field over 1B columns, the day views holding 4x the bits),
    batches of 1024 queries on the union count kernel."""
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf, Op

    nshards = math.ceil(args.cols / SHARD_WIDTH)
    lo, hi = nshards * rank // world, nshards * (rank + 1) // world
    t0 = time.time()
    views = []
    for k, bpc in enumerate([1.0, 1.0, 0.25, 0.25, 0.25, 0.25, 0.25]):
        arena = _roaring.gen_zipf_arena(lo, hi, args.cols, args.rows, bpc, 1.6, 50.0, 100 + k, args.threads)
        views.append(DeviceView(*arena, dev, shards=list(range(lo, hi))))
        del arena
    gen_s = time.time() - t0
    eng = GpuEngine(dev)
    rng = np.random.default_rng(9)
    B = 1024

    S = views[0].S

    def progs_for(rows):
        # vectorised QueryProg records (GpuEngine.union_programs), as the native
        # PQL compiler emits them for Count(Intersect): no per-query Python
        return GpuEngine.union_programs(np.stack([v.dense_many(rows) for v in views], axis=1))

    def q_union():
        rows = zipf_rows(rng, B, args.rows)
        t = eng.launch_count(eng.prepare_progs(progs_for(rows), views, S))
        if world > 1:
            all_reduce(t)
        return int(t.sum().item())

    # the vectorised records answer like the expression compiler (one batch)
    chk_rows = zipf_rows(np.random.default_rng(10), 256, args.rows)
    a = eng.launch_count(eng.prepare_progs(progs_for(chk_rows), views, S)).cpu().numpy()
    b = eng.count_async([Op("or", tuple(Leaf(v, int(r)) for v in views)) for r in chk_rows]).cpu().numpy()
    dt, out = _timed(q_union, args.config_reps, world, dev)
    res = {"config": "time field, Count(Row(t=r, from, to)) = Count(Union of 2 D + 5 H views), 1M rows x 1B cols",
           "gen_s": round(gen_s, 1), "hbm_bytes_per_gpu": sum(v.nbytes() for v in views), "batch": B,
           "kernel": "union_count2_kernel" if eng.union_variant == 2 else "union_count_kernel",
           "ms_per_batch": round(dt * 1000, 2), "qps": round(B / dt, 1), "sample_sum": out,
           "programs_match_compiler": bool((a == b).all())}
    del views
    torch.cuda.empty_cache()
    return res


TIME_VIEWS = [("standard_20200101", 1.0), ("standard_20200102", 1.0), ("standard_2020010300", 0.25),
              ("standard_2020010301", 0.25), ("standard_2020010302", 0.25), ("standard_2020010303", 0.25),
              ("standard_2020010304", 0.25)]
TIME_RANGE = "from='2020-01-01T00:00', to='2020-01-03T05:00'"


def bench_configs_disk(args, world, rank, dev, which):
    """BASELINE configs 4 and 5 through the product path.  The fields are
    written as Pilosa fragment files and opened with a lazy ``Holder``; every
    query is PQL text through ``Executor.execute`` (native loader -> HBM):

    * config 4: int field ``v`` (min -1000, max 1e6, bit depth 20; half the
      columns hold a value uniform in [-1000, 1e6]) stored in its ``bsig_v``
      view (exists / sign / magnitude rows, fragment.go:90-93):
      ``Sum(field=v)``, ``Count(Row(v > x))``, ``Count(Row(v >< [a, b]))``,
      ``Min/Max(field=v)`` and one request of 32 ``Sum(Row(g=r), field=v)``
      (the executor batches it onto the bit-plane count matrix, MFMA);
    * config 5: time field ``t`` (quantum YMDH) whose 2 day views + 5 hour
      views cover ``from=2020-01-01T00:00 to=2020-01-03T05:00`` (the
      reference's views_by_time_range, time.go:104-181); requests of 1024
      ``Count(Row(t=r, from=, to=))``.

    A sample of every answer is re-derived on the host executor over a few
    shards (``verified``).  With N GPUs each rank serves its shard range and
    the per-request answers are summed over the ranks (RCCL)."""
    import resource
    import tempfile

    import torch
    import torch.distributed as dist

    from pilosa_amd import _roaring
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.field import FieldOptions
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor

    nshards = math.ceil(args.cols / SHARD_WIDTH)
    lo, hi = nshards * rank // world, nshards * (rank + 1) // world
    shards = list(range(lo, hi))
    own = args.data_dir is None
    base = tempfile.mkdtemp(prefix=f"pilosa_cfg_r{rank}_", dir=os.environ.get("TMPDIR") or "/tmp") if own \
        else os.path.join(args.data_dir, f"cfg_rank{rank}of{world}")
    res = {}
    try:
        tag = f"{args.cols}:{args.rows}:{lo}:{hi}:{which}:v1"
        marker = os.path.join(base, ".bench_data")
        t0 = time.perf_counter()
        if not (os.path.exists(marker) and open(marker).read() == tag):
            shutil.rmtree(base, ignore_errors=True)
            os.makedirs(base, exist_ok=True)
            h = Holder(base).open()
            idx = h.create_index("c", track_existence=False)
            if "4" in which:
                fv = idx.create_field("v", FieldOptions(type="int", min=-1000, max=1_000_000))
                fv.options.bit_depth = 20
                fv.bsi.bit_depth = 20
                fv.save_meta()
                idx.create_field("g", FieldOptions(cache_type="none"))
            if "5" in which:
                idx.create_field("t", FieldOptions(type="time", time_quantum="YMDH"))
            h.close()

            def frag_dir(field, view):
                d = os.path.join(base, "c", field, "views", view, "fragments")
                os.makedirs(d, exist_ok=True)
                return d
            if "4" in which:
                _roaring.write_bsi_fragments(frag_dir("v", "bsig_v"), lo, hi, args.cols, 20, 0.5, -1000, 1_000_000,
                                             7, args.threads)
                _roaring.write_zipf_fragments(frag_dir("g", "standard"), lo, hi, args.cols, 1000, 1.0, 1.6, 50.0, 11,
                                              args.threads, cache_size=0)
            if "5" in which:
                for k, (vname, bpc) in enumerate(TIME_VIEWS):
                    _roaring.write_zipf_fragments(frag_dir("t", vname), lo, hi, args.cols, args.rows, bpc, 1.6, 50.0,
                                                  100 + k, args.threads, cache_size=0)
            with open(marker, "w") as fh:
                fh.write(tag)
        write_s = time.perf_counter() - t0
        log(f"configs {which}: data ready ({write_s:.1f} s)")
        holder = Holder(base, lazy_fragments=True).open()
        gpu = GpuExecutor(holder, dev)
        ex = Executor(holder, gpu=gpu)
        gpu.executor = ex
        ex.strict_gpu = True
        rng = np.random.default_rng(5)

        def reduce_vals(vals):
            if world == 1:   # nothing to combine: no device round trip inside the timed loop
                return [int(v) for v in vals]
            t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=dev)
            all_reduce(t)
            return t.cpu().tolist()

        def flat(r):
            out = []
            for x in r:
                if hasattr(x, "val"):
                    out += [x.val, x.count]
                else:
                    out.append(int(x))
            return out

        def run(texts, reps):
            # first request loads the views (cold load timed separately), then reps timed requests
            t0 = time.perf_counter()
            first = ex.execute("c", texts[0], shards=shards).results
            torch.cuda.synchronize(dev)
            load = time.perf_counter() - t0
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            last = None
            for k in range(reps):
                last = reduce_vals(flat(ex.execute("c", texts[1 + k % (len(texts) - 1)], shards=shards).results))
            torch.cuda.synchronize(dev)
            el = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=dev)
            if world > 1:
                all_reduce(el, op=dist.ReduceOp.MAX)
            return float(el.item()), load, last, first

        def verify(texts):
            # host executor over a few shards (loads those fragments) vs the device on the same shards
            sel = [shards[i] for i in sorted(set(np.linspace(0, len(shards) - 1, min(3, len(shards))).astype(int)))]
            bad = 0
            for q in texts:
                d = flat(ex.execute("c", q, shards=sel).results)
                ex.gpu = None
                try:
                    hst = flat(ex.execute("c", q, shards=sel).results)
                finally:
                    ex.gpu = gpu
                bad += int(d != hst)
            return {"shards": len(sel), "requests": len(texts), "mismatches": bad, "verified": bad == 0}

        reps = args.config_reps
        if "4" in which:
            r4 = {"config": "BSI int field v (bsig_v fragment files, depth 20, fill 0.5, values [-1000, 1e6]), "
                            "1B cols, lazy Holder + Executor.execute", "queries": {}}
            l0 = gpu.launches
            qs = {"Sum(field=v)": ["Sum(field=v)"] * 2,
                  "Count(Row(v > x))": [f"Count(Row(v > {int(x)}))" for x in rng.integers(0, 1_000_000, 8)],
                  "Count(Row(v >< [a,b]))": [f"Count(Row(v >< [{int(a)}, {int(a) + 50000}]))"
                                             for a in rng.integers(0, 900_000, 8)],
                  "Min(field=v)": ["Min(field=v)"] * 2, "Max(field=v)": ["Max(field=v)"] * 2}
            frows = [[int(r) for r in rng.integers(0, 200, 32)] for _ in range(4)]
            qs["Sum(Row(g=r), field=v) x32 per request"] = [" ".join(f"Sum(Row(g={r}), field=v)" for r in rows)
                                                            for rows in frows]
            for name, texts in qs.items():
                log(f"config 4: {name}")
                dt_, load, last, first = run(texts, reps)
                n_calls = texts[0].count("Sum(") if "x32" in name else 1
                r4["queries"][name] = {"ms_per_request": round(dt_ * 1000, 3), "qps": round(n_calls / dt_, 1),
                                       "first_request_s": round(load, 2), "sample": last[:4]}
            r4["device_launches"] = gpu.launches - l0
            r4["fragments_cold"] = sum(f.is_cold() for f in holder.view("c", "v", "bsig_v").all_fragments())
            r4["verify"] = verify(["Sum(field=v)", qs["Count(Row(v > x))"][0], qs["Count(Row(v >< [a,b]))"][0],
                                   "Min(field=v)", "Max(field=v)", qs["Sum(Row(g=r), field=v) x32 per request"][0]])
            res["config4_bsi"] = r4
        if "5" in which:
            B = 1024
            calls5 = [[f"Count(Row(t={int(r)}, {TIME_RANGE}))" for r in zipf_rows(rng, B, args.rows)]
                      for _ in range(4)]
            texts = [" ".join(c) for c in calls5]
            l0 = gpu.launches
            log("config 5: time-range counts")
            dt_, load, last, first = run(texts, reps)
            res["config5_time_union"] = {
                "config": "time field t (quantum YMDH), Count(Row(t=r, from, to)) over 2 day + 5 hour views "
                          "(fragment files), 1M rows x 1B cols, lazy Holder + Executor.execute",
                "covering_views": [v for v, _ in TIME_VIEWS], "batch": B, "ms_per_request": round(dt_ * 1000, 2),
                "qps": round(B / dt_, 1), "first_request_s": round(load, 2), "sample_sum": int(sum(last)),
                "device_launches": gpu.launches - l0,
                "hbm_bytes_per_gpu": sum(dv.nbytes() for _, dv in gpu._arenas.values()),
                "verify": verify([" ".join(calls5[1][:64])])}
        res["data"] = {"write_s": round(write_s, 2), "dir_bytes": _dir_bytes(base),
                       "peak_host_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)}
        holder.close()
        ex.close()
        del gpu
        torch.cuda.empty_cache()
        return res
    finally:
        if own and not args.keep_data:
            shutil.rmtree(base, ignore_errors=True)


def host_pair_counts(bitmaps, pairs):
    """Host roaring oracle: counts[q, k] = |Row(a_q) & Row(b_q)| in shard k."""
    w = SHARD_WIDTH
    out = np.zeros((len(pairs), len(bitmaps)), np.int64)
    for k, bm in enumerate(bitmaps):
        for q, (a, b) in enumerate(pairs):
            r1 = bm.offset_range(0, a * w, (a + 1) * w)
            r2 = bm.offset_range(0, b * w, (b + 1) * w)
            out[q, k] = r1.intersection_count(r2)
    return out


def verify_sample(eng, view, host_bitmap, pairs, answered, world, dev, nshards_check=8):
    """Re-derive a sample of the timed batch's counts on the host: GPU
    per-shard counts of ``pairs`` over the whole local arena vs the host
    roaring core on ``nshards_check`` local shards, and the per-shard sums
    (all-reduced over ranks) vs the answers the timed path returned."""
    import torch
    from pilosa_amd.ops.device import GpuEngine
    S = view.S
    pairs = [(int(a), int(b)) for a, b in pairs]
    progs = GpuEngine.pair_programs(0, view.dense_many(np.array([a for a, _ in pairs], np.uint64)), 0,
                                    view.dense_many(np.array([b for _, b in pairs], np.uint64)))
    per_shard = eng.count_per_shard_progs(progs, [view], S)          # [Q, S]
    sel = sorted(set(np.linspace(0, max(S - 1, 0), min(nshards_check, S)).astype(int).tolist())) if S else []
    host = host_pair_counts([host_bitmap(si) for si in sel], pairs)
    bad_shard = int((per_shard[:, sel] != host).sum()) if sel else 0
    tot = torch.from_numpy(per_shard.sum(axis=1)).to(dev)
    if world > 1:
        all_reduce(tot)
    bad_total = int((tot.cpu().numpy() != np.asarray(answered, np.int64)).sum())
    return {"queries": len(pairs), "shards_checked": len(sel), "mismatch_shard_counts": bad_shard,
            "mismatch_totals": bad_total, "verified": bad_shard == 0 and bad_total == 0}


def kfd_gpu_count(root: str = "/sys/class/kfd/kfd/topology/nodes"):
    """GPUs visible to this process, counted without any HIP call (the
    launcher must not initialise the GPU before it starts the ranks): KFD
    topology nodes with SIMDs are GPUs (CPU nodes report ``simd_count 0``),
    limited by ROCR/HIP/CUDA_VISIBLE_DEVICES.  None when the topology is
    unreadable."""
    try:
        nodes = os.listdir(root)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(root, d, "properties")) as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def _launch_ranks(args) -> int:
    """``bench.py --gpus N`` without a launcher: check that N devices are
    visible (counting them does not initialise the GPU), then run this
    script under torch.distributed.run with one rank per GPU as a child
    process and return its exit code.  PILOSA_BENCH_REHEARSE=1 allows N
    ranks on fewer GPUs (gloo rehearsal, never for reported numbers)."""
    import subprocess

    rehearse = os.environ.get("PILOSA_BENCH_REHEARSE") == "1"
    if not rehearse:
        visible = kfd_gpu_count()
        if visible is None:
            print("bench: cannot count GPUs from the KFD topology (/sys/class/kfd); launch the ranks with "
                  "torch.distributed.run yourself", file=sys.stderr, flush=True)
            return 2
        if visible < args.gpus:
            print(f"bench: --gpus {args.gpus} but {visible} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {args.gpus} ranks: {' '.join(cmd[2:9])} ...")
    return subprocess.call(cmd, env=dict(os.environ))


def setup_dist(mesh: bool = False):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-GPU path on a 1-GPU box: every rank on cuda:0, gloo
    # collectives through host copies (PILOSA_BENCH_REHEARSE=1); never used
    # for reported numbers
    rehearse = os.environ.get("PILOSA_BENCH_REHEARSE") == "1"
    if rehearse:
        local_rank = 0
    dev = torch.device("cuda", local_rank)
    if world > 1 and not rehearse and local_rank >= torch.cuda.device_count():
        raise SystemExit(f"bench: rank {rank} has LOCAL_RANK {local_rank} but {torch.cuda.device_count()} GPU(s)")
    if world > 1 or mesh:
        from pilosa_amd.parallel.collectives import Comm, init
        torch.cuda.set_device(local_rank)
        init("gloo" if rehearse else "nccl", local_rank, timeout_s=600)
        global _COMM
        _COMM = Comm(device=dev, host_copies=rehearse)
    return world, rank, dev


def run_synthetic(args, world, rank, dev, queries, ra, rb):
    """Kernel harness: in-memory arena, batches straight to the engine."""
    import torch
    import torch.distributed as dist

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine
    from pilosa_amd.ops.planner import NativeCountCompiler

    nshards = math.ceil(args.cols / SHARD_WIDTH)
    lo = nshards * rank // world
    hi = nshards * (rank + 1) // world
    t0 = time.time()
    rows, rowptr, sb, meta, payload = _roaring.gen_zipf_arena(lo, hi, args.cols, args.rows, 8.0, 1.6, 50.0, 1,
                                                              args.threads)
    tgen = time.time() - t0
    view = DeviceView(rows, rowptr, sb, meta, payload, dev, shards=list(range(lo, hi)))
    del rows, rowptr, sb, meta, payload
    torch.cuda.synchronize(dev)
    tload = time.time() - t0 - tgen
    eng = GpuEngine(dev)
    compiler = NativeCountCompiler({"f": view})

    def prep(i):
        # host half: PQL text -> device programs (native scanner, general
        # parser for anything else) + batch ordering + program upload
        qs = queries[i * args.batch:(i + 1) * args.batch]
        return eng.prepare_progs(*compiler.compile(qs))

    def launch(h):
        out = eng.launch_count(h)
        if world > 1:
            all_reduce(out)
        return out

    tm = {"prep": 0.0, "launch": 0.0, "wait": 0.0}

    def run(first, n):
        # software pipeline: the host prepares batch i+1 while the GPU runs i
        h = prep(first)
        pending = launch(h)
        res = None
        for i in range(first + 1, first + n):
            t0 = time.perf_counter()
            h = prep(i)
            t1 = time.perf_counter()
            nxt = launch(h)
            t2 = time.perf_counter()
            res = pending.cpu()
            t3 = time.perf_counter()
            tm["prep"] += t1 - t0
            tm["launch"] += t2 - t1
            tm["wait"] += t3 - t2
            pending = nxt
        res = pending.cpu()
        return res

    run(0, args.warmup)
    for k in tm:
        tm[k] = 0.0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    last = run(args.warmup, args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t

    extra = {"path": "kernel harness (in-memory arena, engine direct)", "gen_s": round(tgen, 2),
             "h2d_s": round(tload, 2), "hbm_bytes_per_gpu": view.nbytes(), "containers_per_gpu": view.container_count,
             "shards": nshards, "mean_count": float(last.double().mean()) if last is not None else None,
             "native_compiled": compiler.native_hits, "fallback_compiled": compiler.fallbacks,
             "host_ms_per_step": {k: round(v / max(1, args.steps - 1) * 1000, 3) for k, v in tm.items()}}
    if args.verify > 0:
        b0 = (args.warmup + args.steps - 1) * args.batch
        n = min(args.verify, args.batch)
        pairs = list(zip(ra[b0:b0 + n], rb[b0:b0 + n]))

        def host_bitmap(si):
            return _roaring.arena_shard_bitmap(*_roaring.gen_zipf_arena(lo + si, lo + si + 1, args.cols, args.rows,
                                                                        8.0, 1.6, 50.0, 1, args.threads), 0)
        extra["verify"] = verify_sample(eng, view, host_bitmap, pairs, last.numpy()[:n], world, dev)
    if args.cpu_baseline_shards > 0 and rank == 0:
        extra["cpu_host"] = bench_cpu_host(args, ra, rb, nshards)
    if args.topn_batches > 0:
        extra["topn"] = bench_topn(args, view, eng, np.random.default_rng(99), world, rank, dev)
    return elapsed, extra


def _dir_bytes(path):
    tot = 0
    for root, _, files in os.walk(path):
        for f in files:
            try:
                tot += os.path.getsize(os.path.join(root, f))
            except OSError:
                pass
    return tot


def _evict_page_cache(root: str) -> dict:
    """fsync + POSIX_FADV_DONTNEED every file under ``root`` so the next read
    of the index comes from the device, as after a restart (an unprivileged
    process may drop clean pages of its own files).  Returns what it did."""
    t0 = time.perf_counter()
    files = nbytes = 0
    for dp, _, fns in os.walk(root):
        for fn in fns:
            path = os.path.join(dp, fn)
            try:
                fd = os.open(path, os.O_RDONLY)
            except OSError:
                continue
            try:
                os.fsync(fd)
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
                files += 1
                nbytes += os.fstat(fd).st_size
            except OSError:
                pass
            finally:
                os.close(fd)
    return {"evicted_files": files, "evicted_bytes": nbytes, "s": round(time.perf_counter() - t0, 2),
            "how": "fsync + posix_fadvise(DONTNEED) per file before the load"}


def _write_index(args, base, lo, hi):
    """The headline index's fragment files for shards [lo, hi) under
    ``base`` (reused when the marker matches).  Returns (fragment dir,
    what was done)."""
    from pilosa_amd import _roaring
    from pilosa_amd.models.field import FieldOptions
    from pilosa_amd.models.holder import Holder

    tag = f"{args.cols}:{args.rows}:{lo}:{hi}:zipf1.6/50:8:seed1:cache{args.topn_cache}"
    marker = os.path.join(base, ".bench_data")
    fdir = os.path.join(base, "i", "f", "views", "standard", "fragments")
    t0 = time.perf_counter()
    if os.path.exists(marker) and open(marker).read() == tag:
        return fdir, {"reused": True, "bytes": _dir_bytes(fdir)}
    log("writing fragment files")
    shutil.rmtree(base, ignore_errors=True)
    os.makedirs(base, exist_ok=True)
    need = int(36e9 * (hi - lo) / 954 * (args.rows / NROWS))
    free = shutil.disk_usage(base).free
    if free < need:
        raise SystemExit(f"bench --mode disk: {free / 1e9:.1f} GB free in {base}, need ~{need / 1e9:.1f} GB "
                         "(set --data-dir or use --mode synthetic)")
    h = Holder(base).open()
    h.create_index("i", keys=False, track_existence=True)
    h.index("i").create_field("f", FieldOptions())
    h.close()
    os.makedirs(fdir, exist_ok=True)
    w = _roaring.write_zipf_fragments(fdir, lo, hi, args.cols, args.rows, 8.0, 1.6, 50.0, 1, args.threads,
                                      cache_size=args.topn_cache)
    with open(marker, "w") as fh:
        fh.write(tag)
    return fdir, {"files": int(w["shards"]), "bytes": int(w["bytes"]), "containers": int(w["containers"]),
                  "s": round(time.perf_counter() - t0, 2)}


def run_disk(args, world, rank, dev, queries, ra, rb):
    """Product path: Pilosa-format fragment files on disk -> Holder (lazy) ->
    HBM via the native file loader -> Executor.execute(PQL text)."""
    import resource
    import shutil
    import tempfile
    import threading

    import torch
    import torch.distributed as dist

    from pilosa_amd import _roaring
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.field import FieldOptions
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor

    nshards = math.ceil(args.cols / SHARD_WIDTH)
    lo = nshards * rank // world
    hi = nshards * (rank + 1) // world
    shards = list(range(lo, hi))
    own = args.data_dir is None
    base = tempfile.mkdtemp(prefix=f"pilosa_bench_r{rank}_", dir=os.environ.get("TMPDIR") or "/tmp") if own \
        else os.path.join(args.data_dir, f"rank{rank}of{world}")
    extra = {"path": "Holder(lazy) + file loader -> HBM, Executor.execute(PQL text) per request", "data_dir": base}
    try:
        fdir, extra["write"] = _write_index(args, base, lo, hi)
        if args.cold_load:
            # resume from disk, not from the page cache the write just filled:
            # every fragment file is synced and dropped from the cache first
            extra["page_cache"] = _evict_page_cache(base)
        log("opening holder + loading the view into HBM")
        t1 = time.perf_counter()
        holder = Holder(base, lazy_fragments=True).open()
        t2 = time.perf_counter()
        gpu = GpuExecutor(holder, dev)
        ex = Executor(holder, gpu=gpu)
        ex.strict_gpu = True  # a device fault fails the bench instead of timing the host path
        view = gpu.view_arena("i", "f", "standard", shards)
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        extra.update({"holder_open_s": round(t2 - t1, 2), "load_s": round(t3 - t2, 2), "load": gpu.last_load,
                      "hbm_bytes_per_gpu": view.nbytes(), "containers_per_gpu": int(view.container_count),
                      "cold_loads": gpu.cold_loads, "shards": nshards,
                      "fragments_cold_after_load": sum(f.is_cold() for f in holder.view("i", "f", "standard")
                                                       .all_fragments())})
        assert holder.index("i").available_shards() == shards, "holder must serve exactly this rank's shards"

        texts = [" ".join(queries[i * args.batch:(i + 1) * args.batch]) for i in range(args.warmup + args.steps)]
        results = [None] * len(texts)
        lock = threading.Lock()
        nxt = [0]
        err = []

        from pilosa_amd.executor import ExecOptions
        dopt = ExecOptions()
        dopt.device_counts = world > 1   # N>1: counts stay on the device for the all-reduce

        def client(end):
            while True:
                with lock:
                    i = nxt[0]
                    if i >= end or err:
                        return
                    nxt[0] += 1
                try:
                    r = ex.execute("i", texts[i], shards=shards, opt=dopt).results
                    if world > 1 and isinstance(r, torch.Tensor):
                        ev = torch.cuda.Event()
                        ev.record()      # the batch's kernels, on this thread's stream
                        r = (r, ev)
                    results[i] = r
                except BaseException as e:  # noqa: BLE001
                    err.append(e)
                    return

        comm_stream = torch.cuda.Stream(dev) if world > 1 else None

        def run(first, n):
            nxt[0] = first
            ts = [threading.Thread(target=client, args=(first + n,)) for _ in range(max(1, args.clients))]
            for t in ts:
                t.start()
            # ranks all-reduce each request's counts in request order (one
            # collective per batch, issued from this thread only) on a stream
            # of its own, so it never queues behind the next batch's kernels
            for i in range(first, first + n):
                if world > 1:
                    while results[i] is None and not err:
                        time.sleep(0.0002)
                    if err:
                        break
                    with torch.cuda.stream(comm_stream):
                        r = results[i]
                        if isinstance(r, tuple):   # device counts: reduce them in place
                            tt, ev = r
                            comm_stream.wait_event(ev)
                            tt.record_stream(comm_stream)
                        else:
                            tt = torch.tensor(r, dtype=torch.int64, device=dev)
                        all_reduce(tt)
                        results[i] = gpu.engine.to_host(tt).tolist()
            for t in ts:
                t.join()
            if err:
                raise err[0]

        n0 = gpu.launches
        log("count: warmup")
        run(0, args.warmup)
        # the server's GC policy (utils/gctune.py): start-up objects frozen
        from pilosa_amd.utils import gctune
        gctune.configure()
        gctune.freeze_long_lived()
        assert gpu.launches > n0, "requests did not reach the device"
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        run(args.warmup, args.steps)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t
        last = results[args.warmup + args.steps - 1]
        extra.update({"clients": args.clients, "mean_count": float(np.mean(last)), "launches": gpu.launches - n0,
                      "gpu_faults": ex.gpu_faults, "peak_host_rss_gb":
                      round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)})
        if args.verify > 0:
            b0 = (args.warmup + args.steps - 1) * args.batch
            n = min(args.verify, args.batch)
            pairs = list(zip(ra[b0:b0 + n], rb[b0:b0 + n]))

            def host_bitmap(si):
                with open(os.path.join(fdir, str(shards[si])), "rb") as fh:
                    return _roaring.Bitmap.from_bytes(fh.read())
            extra["verify"] = verify_sample(gpu.engine, view, host_bitmap, pairs, last[:n], world, dev)
        log("count: done")
        if args.topn_batches > 0:
            extra["topn"] = bench_topn_exec(args, holder, ex, gpu, shards, fdir, world, rank, dev)
        holder.close()
        if args.serve_seconds > 0 and world == 1:
            # the server opens the same data dir itself: free this process's arena first
            ex.close()
            del ex, gpu, view
            import gc
            gc.collect()
            torch.cuda.empty_cache()
            extra["serving"] = bench_serving(args, base, dev)
        return elapsed, extra
    finally:
        if own and not args.keep_data:
            shutil.rmtree(base, ignore_errors=True)


def _mesh_root(args, world) -> str:
    """Parent dir of every rank's data dir in a multi-GPU run (deterministic
    per job, so rank 0 can read the other ranks' fragment files to verify)."""
    if args.data_dir is not None:
        return args.data_dir
    return os.path.join(os.environ.get("TMPDIR") or "/tmp", f"pilosa_bench_{os.environ.get('MASTER_PORT', '0')}")


def run_disk_mesh(args, world, rank, dev, queries, ra, rb):
    """N>1 product path, as ``pilosa_amd server`` runs under torchrun: one
    process per GPU, each with its own holder over the fragment files of a
    contiguous shard range (ShardMesh ownership ``(s // block) % world``
    with ``block = ceil(shards / world)``), loaded into its HBM by the file
    loader.  Rank 0 is the front end: every request is
    ``Executor.execute(PQL text)``, which sends it through the mesh
    (parallel/mesh.py) -- Count requests as ``count_text`` (broadcast, each
    rank compiles and counts its share natively, device all-reduce, several
    requests in flight), TopN requests as ``OP_TOPN`` batches (candidate
    union + all-reduced re-count on the devices, pipelined).  Ranks > 0 run
    ``ShardMesh.serve``.  The timed region is bracketed by ``mesh.sync()``
    (every rank drains its in-flight requests, synchronises its device and
    meets the others); the time is the max over ranks.
    Reference: executor.go:2458-2555 (mapReduce over nodes)."""
    import resource
    import threading

    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    from pilosa_amd.parallel.mesh import ShardMesh

    nshards = math.ceil(args.cols / SHARD_WIDTH)
    block = -(-nshards // world)
    own = [s for s in range(nshards) if (s // block) % world == rank]
    lo, hi = (own[0], own[-1] + 1) if own else (0, 0)
    all_shards = list(range(nshards))
    root = _mesh_root(args, world)
    rank_dir = lambda r: os.path.join(root, f"rank{r}of{world}")   # noqa: E731
    base = rank_dir(rank)
    extra = {"path": "ShardMesh product path: rank 0 Executor.execute(PQL text) -> mesh count_text / OP_TOPN; "
                     "every rank: Holder(lazy) + file loader -> HBM",
             "data_dir": base, "block": block}
    holder = ex = None
    try:
        fdir, extra["write"] = _write_index(args, base, lo, hi)
        if args.cold_load:
            extra["page_cache"] = _evict_page_cache(base)
        t1 = time.perf_counter()
        holder = Holder(base, lazy_fragments=True).open()
        gpu = GpuExecutor(holder, dev)
        ex = Executor(holder, gpu=gpu)
        gpu.executor = ex
        ex.strict_gpu = True
        view = gpu.view_arena("i", "f", "standard", own) if own else None
        torch.cuda.synchronize(dev)
        load_s = time.perf_counter() - t1
        mesh = ShardMesh(ex, block=block, device=dev, force=getattr(args, "mesh", False))
        if rank != 0:
            log(f"mesh worker: {len(own)} shards loaded in {load_s:.2f} s, serving")
            mesh.serve()
            return 0.0, {}
        ex.mesh = mesh
        from pilosa_amd.utils import gctune   # the front end's GC policy (Server.open does the same)
        gctune.configure()
        gctune.freeze_long_lived()
        per_rank = {r: len(v.get("i", [])) for r, v in mesh.shard_counts().items()}
        extra.update({"load_s_rank0": round(load_s, 2), "load": gpu.last_load,
                      "hbm_bytes_rank0": view.nbytes() if view is not None else 0,
                      "shards": nshards, "shards_per_rank": per_rank})
        assert sum(per_rank.values()) == nshards, per_rank

        texts = [" ".join(queries[i * args.batch:(i + 1) * args.batch]) for i in range(args.warmup + args.steps)]
        results = [None] * len(texts)
        lock = threading.Lock()
        nxt = [0]
        err = []

        def client(end):
            while True:
                with lock:
                    i = nxt[0]
                    if i >= end or err:
                        return
                    nxt[0] += 1
                try:
                    results[i] = ex.execute("i", texts[i], shards=all_shards).results
                except BaseException as e:  # noqa: BLE001
                    err.append(e)
                    return

        def run(first, n):
            nxt[0] = first
            ts = [threading.Thread(target=client, args=(first + n,)) for _ in range(max(1, args.clients))]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            if err:
                raise err[0]

        seq0 = mesh.seq
        log("mesh count: warmup")
        run(0, args.warmup)
        t_a = mesh.sync()
        run(args.warmup, args.steps)
        t_b = mesh.sync()
        elapsed = max(b - a for a, b in zip(t_a, t_b)) / 1e9
        last = results[args.warmup + args.steps - 1]
        extra.update({"clients": args.clients, "mean_count": float(np.mean(last)),
                      "mesh_count_requests": mesh.seq - seq0, "mesh_max_in_flight": mesh.max_in_flight,
                      "per_rank_elapsed_s": [round((b - a) / 1e9, 4) for a, b in zip(t_a, t_b)],
                      "gpu_faults": ex.gpu_faults,
                      "peak_host_rss_gb_rank0": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)})
        log(f"mesh count: {args.steps} steps in {elapsed:.3f} s")
        if args.verify > 0:
            # per-shard answers through the mesh (the owner rank counts, the
            # others add zero) vs the host roaring core over that shard's file
            # in its owner's data dir
            b0 = (args.warmup + args.steps - 1) * args.batch
            n = min(args.verify, args.batch)
            pairs = [(int(a), int(b)) for a, b in zip(ra[b0:b0 + n], rb[b0:b0 + n])]
            sel = sorted(set(np.linspace(0, nshards - 1, min(8, nshards)).astype(int).tolist()))
            text = " ".join(queries[b0:b0 + n])
            bad = 0
            for s in sel:
                got = ex.execute("i", text, shards=[s]).results
                path = os.path.join(rank_dir((s // block) % world), "i", "f", "views", "standard", "fragments", str(s))
                with open(path, "rb") as fh:
                    bm = _roaring.Bitmap.from_bytes(fh.read())
                want = host_pair_counts([bm], pairs)[:, 0]
                bad += int((np.asarray(got, np.int64) != want).sum())
            extra["verify"] = {"queries": n, "shards_checked": len(sel), "mismatch_shard_counts": bad,
                               "answered_by": "owner rank through the mesh", "verified": bad == 0,
                               "verified_all_ranks": bad == 0}
        if args.mesh_breakdown > 0:
            extra["mesh_breakdown"] = mesh_breakdown(args, ex, mesh, all_shards, queries)
        if args.topn_batches > 0:
            extra["topn"] = bench_topn_mesh(args, ex, mesh, all_shards)
        mesh.stop()
        return elapsed, extra
    finally:
        if ex is not None:
            ex.close()
        if holder is not None:
            holder.close()
        if args.data_dir is None and not args.keep_data:
            shutil.rmtree(base, ignore_errors=True)


def mesh_breakdown(args, ex, mesh, all_shards, queries):
    """Where a mesh request's time goes on the front end:
    ``--mesh-breakdown N`` sequential Count batches and cache-only TopN
    requests under a HIP-event tracer; per span name the mean host ms per
    request and, for GPU spans, the mean device ms between the span's events
    (command publish, native compile/plan, kernel launch, collective issue
    and wait, D2H)."""
    from pilosa_amd.utils import tracing
    n = args.mesh_breakdown
    B = args.batch
    texts = [" ".join(queries[i * B:(i + 1) * B]) for i in range(min(n, len(queries) // B))]
    topn = [" ".join(_wide_topn_calls(args.topn_batch, seed=900 + i)) for i in range(n)]
    for t in topn[:2]:      # their node candidate spaces (n buckets) built untimed
        ex.execute("i", t, shards=all_shards)
    # src TopN requests as the src phase draws them (one untimed first)
    hot = zipf_rows(np.random.default_rng(901), args.topn_batch * (n + 1), 1000)
    src = [" ".join(f"TopN(f, Row(f={a}), n=100)" for a in hot[i * args.topn_batch:(i + 1) * args.topn_batch])
           for i in range(n + 1)]
    ex.execute("i", src[0], shards=all_shards)
    out = {}
    for kind, reqs in (("count", texts), ("topn_cache", topn), ("topn_src", src[1:])):
        if not reqs:
            continue
        tr = tracing.HipEventTracer(limit=200000)
        tracing.set_global_tracer(tr)
        try:
            mesh.sync()
            t0 = time.perf_counter()
            for r in reqs:
                ex.execute("i", r, shards=all_shards)
            mesh.sync()
            wall = time.perf_counter() - t0
        finally:
            tracing.set_global_tracer(tracing.NopTracer())
        agg = {}
        for sp in tr.spans:
            a = agg.setdefault(sp.name, [0, 0.0, 0.0, 0])
            a[0] += 1
            a[1] += sp.duration * 1000
            dm = sp.device_ms(wait=True)
            if dm is not None:
                a[2] += dm
                a[3] += 1
        k = len(reqs)
        out[kind] = {"requests": k, "wall_ms_per_request": round(wall / k * 1000, 3),
                     "spans": {name: {"per_request": round(c / k, 2), "host_ms": round(h / k, 4),
                                      **({"device_ms": round(d / k, 4)} if nd else {})}
                               for name, (c, h, d, nd) in sorted(agg.items(), key=lambda kv: -kv[1][1])}}
    log(f"mesh breakdown: {json.dumps(out)[:2000]}")
    return out


def bench_topn_mesh(args, ex, mesh, all_shards):
    """BASELINE config 3 on N GPUs: TopN requests through rank 0's
    ``Executor.execute`` -> ``ShardMesh.topn_batch`` (OP_TOPN: each rank's
    device runs both phases over its shards, candidates union over the
    ranks, re-counts all-reduced; up to MAX_IN_FLIGHT batches in flight)
    from ``--clients`` request threads.  The fused answers are checked
    against the two-phase map/reduce through the mesh (OP_CALL per phase)."""
    import threading

    from pilosa_amd.executor import ExecOptions
    from pilosa_amd.pql import parse_string

    n = 100
    B, nb = args.topn_batch, args.topn_batches
    rng = np.random.default_rng(99)
    out = {"path": "rank 0 Executor.execute(TopN text) -> ShardMesh OP_TOPN_PLAIN (cache-only) / OP_TOPN (src)",
           "n": n, "batch": B, "clients": {"cache": args.topn_cache_clients, "src": args.topn_clients}}

    def timed(texts, rec, warm=1, profile="", nclients=1):
        done = [None] * len(texts)
        t0 = time.perf_counter()
        done[0] = ex.execute("i", texts[0], shards=all_shards).results
        rec["first_request_s"] = round(time.perf_counter() - t0, 2)
        # untimed warm requests, as the 1-GPU phases take: the node candidate
        # spaces of the requests' n buckets are built once
        for i in range(1, warm):
            done[i] = ex.execute("i", texts[i], shards=all_shards).results
        from pilosa_amd.utils import gctune
        gctune.freeze_long_lived()
        nxt = [warm]
        lock = threading.Lock()
        err = []

        def client():
            while True:
                with lock:
                    i = nxt[0]
                    if i >= len(texts) or err:
                        return
                    nxt[0] += 1
                try:
                    done[i] = ex.execute("i", texts[i], shards=all_shards).results
                except BaseException as e:  # noqa: BLE001
                    err.append(e)
                    return
        mesh.max_in_flight = 0
        b0 = mesh.topn_tensor_batches + mesh.topn_plain_batches
        r0 = mesh.topn_plain_refreshes
        prof = None
        if profile:
            from pilosa_amd.utils import pprof
            prof_out = {}
            prof = threading.Thread(target=lambda: prof_out.setdefault("p", pprof.cpu_profile(0.3, 500)),
                                    daemon=True)
            prof.start()
        t_a = mesh.sync()
        cprof = os.environ.get("PILOSA_BENCH_CPROFILE", "") if profile else ""
        if cprof and max(1, nclients) == 1:
            # deterministic profile of the one request thread (host cost per call)
            import cProfile
            import io
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            client()
            pr.disable()
            sio = io.StringIO()
            pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(45)
            pstats.Stats(pr, stream=sio).sort_stats("cumulative").print_stats(70)
            with open(cprof, "w") as fh:
                fh.write(sio.getvalue())
        else:
            ts = [threading.Thread(target=client) for _ in range(max(1, nclients))]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        t_b = mesh.sync()
        if err:
            raise err[0]
        if prof is not None:
            prof.join()
            with open(profile, "w") as fh:
                fh.write(prof_out.get("p", ""))
        el = max(b - a for a, b in zip(t_a, t_b)) / 1e9
        nt = len(texts) - warm
        rec.update({"qps": round(B * nt / el, 2), "ms_per_request": round(el / nt * 1000, 2), "warm_requests": warm,
                    "device_batches": mesh.topn_tensor_batches + mesh.topn_plain_batches - b0,
                    "space_refreshes": mesh.topn_plain_refreshes - r0, "max_in_flight": mesh.max_in_flight,
                    "sample_top3": [(p.id, p.count) for p in done[-1][0][:3]] if done[-1] and done[-1][0] else []})
        return done

    log("mesh topn: cache-only requests (distinct calls)")
    # the same request counts and warm-up as the 1-GPU phases (bench_topn)
    nbc, W = max(nb, args.topn_cache_batches), 8
    cache_calls = _wide_topn_calls(B * (nbc + W), seed=17)
    out["cache"] = {"calls": f"TopN(f, n=log-uniform 1..1000, threshold one of {len(WIDE_THRESHOLDS)} values "
                             "1..50000), random per call"}
    timed([" ".join(cache_calls[i * B:(i + 1) * B]) for i in range(nbc + W)], out["cache"], warm=W,
          profile=os.environ.get("PILOSA_BENCH_TOPN_PROFILE", ""), nclients=args.topn_cache_clients)
    cyc = _distinct_topn_calls(B * (nbc + W))
    out["cache_cycling"] = {"calls": "TopN(f, n in {10,50,100,500} + offset, threshold in {1,1000,5000,20000})"}
    timed([" ".join(cyc[i * B:(i + 1) * B]) for i in range(nbc + W)], out["cache_cycling"], warm=W,
          nclients=args.topn_cache_clients)
    WS = 3
    nb = max(nb, args.topn_src_batches)
    hot = zipf_rows(rng, B * (nb + WS), 1000)
    src_calls = [f"TopN(f, Row(f={a}), n={n})" for a in hot]
    src_q = [" ".join(src_calls[i * B:(i + 1) * B]) for i in range(nb + WS)]
    out["src"] = {}
    log("mesh topn: src requests")
    res = timed(src_q, out["src"], warm=WS, nclients=args.topn_clients,
                profile=os.environ.get("PILOSA_BENCH_TOPN_SRC_PROFILE", ""))
    if args.verify > 0:
        last = (nb + WS - 1) * B
        calls = [parse_string(c).calls[0] for c in src_calls[last:last + 2]] + [parse_string(f"TopN(f, n={n})").calls[0]]
        fused = [[(p.id, p.count) for p in r] for r in res[-1][:2]] + \
            [[(p.id, p.count) for p in ex.execute("i", f"TopN(f, n={n})", shards=all_shards).results[0]]]
        two_phase = [[(p.id, p.count) for p in ex._topn("i", c, all_shards, ExecOptions())] for c in calls]
        out["verify"] = {"fused_equals_two_phase_mesh": fused == two_phase, "verified": fused == two_phase}
    return out


def bench_serving(args, base, dev):
    """The server product path on the same data dir:
    ``Server`` (lazy holder, GPU executor, native epoll HTTP front end,
    group-commit of concurrent Count requests) under the closed-loop C++ load
    generator: ``--serve-conns`` keep-alive connections, one
    ``Count(Intersect(Row, Row))`` per request for ``--serve-seconds``, then a
    Count + TopN(f, n=100) mix; sampled responses are checked against
    ``Executor.execute``.  Then a bulk import through POST /import (protobuf
    ImportRequest, one per shard, concurrent clients) into the cold fragments
    (mapped copy-on-write containers), and the first query after it, which
    replays the write batches of every shard on the device in shared launches.
    Reference: http/handler.go:293,495 (query, import routes)."""
    import http.client
    import threading

    from pilosa_amd import _httpd
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger
    from pilosa_amd.wire import pb

    out = {"path": "Server(data dir) -> native httpd -> Executor (group commit) -> GPU"}
    t0 = time.perf_counter()
    srv = Server(base, bind="127.0.0.1:0", gpu="on", logger=CaptureLogger()).open()
    try:
        ex = srv.executor
        rng = np.random.default_rng(77)
        a, b = zipf_rows(rng, 20000, args.rows), zipf_rows(rng, 20000, args.rows)
        queries = [f"Count(Intersect(Row(f={x}), Row(f={y})))" for x, y in zip(a, b)]
        ex.execute("i", queries[0])   # loads the view into HBM
        out["open_and_load_s"] = round(time.perf_counter() - t0, 2)
        port = srv.uri.port

        def run(bodies, seconds, samples):
            log(f"serving: {len(bodies)} bodies, {args.serve_conns} conns, {seconds} s")
            res = _httpd.load("127.0.0.1", port, "/index/i/query", [q.encode() for q in bodies], args.serve_conns,
                              4, float(seconds), samples)
            mism = 0
            smp = res.pop("samples", [])
            for k, body in smp:
                want = ex.execute("i", bodies[k]).results
                got = json.loads(body)["results"]
                if [r if isinstance(r, int) else [[p.id, p.count] for p in r] for r in want] != \
                        [r if isinstance(r, int) else [[p["id"], p["count"]] for p in r] for r in got]:
                    mism += 1
            fe = res.pop("first_error", b"")
            return {"req_per_s": round(res["requests"] / seconds, 1), "requests": int(res["requests"]),
                    "errors": int(res["errors"]), "p50_ms": round(res.get("p50_ms", 0.0), 3),
                    "p99_ms": round(res.get("p99_ms", 0.0), 3), "mean_ms": round(res.get("mean_ms", 0.0), 3),
                    "verified": len(smp), "mismatches": mism,
                    "first_error": fe[:200].decode(errors="replace") if fe else ""}
        out["count"] = run(queries, args.serve_seconds, 64)
        tcalls = _distinct_topn_calls(2000)
        mix = [q if k % 10 else tcalls[k] for k, q in enumerate(queries[:2000])]
        prof = None
        if args.serve_profile:
            # every server thread's stacks sampled during the mix (/debug/pprof/profile)
            from pilosa_amd.utils import pprof
            holder_ = {}
            prof = threading.Thread(target=lambda: holder_.setdefault(
                "p", pprof.cpu_profile(seconds=max(2.0, args.serve_seconds / 2), hz=250)), daemon=True)
            prof.start()
        out["count_topn_mix"] = dict(run(mix, max(2.0, args.serve_seconds / 2), 32), topn_fraction=0.1)
        if prof is not None:
            prof.join()
            with open(args.serve_profile, "w") as fh:
                fh.write(holder_.get("p", ""))
        out["conns"] = args.serve_conns
        out["httpd"] = srv.httpd.stats() if hasattr(srv.httpd, "stats") else None

        # ---- bulk import through the HTTP API
        nsh = min(args.import_shards, len(srv.holder.index("i").available_shards()))
        per = args.import_bits_per_shard
        irng = np.random.default_rng(5)
        bodies = []
        for s in range(nsh):
            rows = zipf_rows(irng, per, 1000).astype(np.uint64)
            cols = (np.uint64(s) << np.uint64(20)) + irng.integers(0, 1 << 20, size=per).astype(np.uint64)
            bodies.append((s, rows, cols, pb.ImportRequest(Index="i", Field="f", Shard=s, RowIDs=rows.tolist(),
                                                           ColumnIDs=cols.tolist()).SerializeToString()))
        rss0 = _rss_gb()
        errs = []
        nxt = [0]
        lock = threading.Lock()

        def importer():
            conn = http.client.HTTPConnection("127.0.0.1", port, timeout=300)
            while True:
                with lock:
                    k = nxt[0]
                    nxt[0] += 1
                if k >= len(bodies):
                    return
                conn.request("POST", "/index/i/field/f/import", body=bodies[k][3],
                             headers={"Content-Type": "application/x-protobuf", "Accept": "application/x-protobuf"})
                r = conn.getresponse()
                r.read()
                if r.status != 200:
                    errs.append(r.status)
        log(f"import: {nsh} shards x {per} bits over HTTP")
        t1 = time.perf_counter()
        ts = [threading.Thread(target=importer) for _ in range(args.import_clients)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        t_imp = time.perf_counter() - t1
        gpu = ex.gpu
        w0 = getattr(gpu, "device_writes", 0)
        wl0 = getattr(gpu, "device_write_launches", 0)
        t2 = time.perf_counter()
        ex.execute("i", queries[1])      # first query after the import: device replay of the write batches
        t_replay = time.perf_counter() - t2
        frags = srv.holder.view("i", "f", "standard").all_fragments()
        chk = []
        for s, rows, cols, _ in bodies[:3]:
            r = int(rows[0])
            got = ex.execute("i", f"Count(Row(f={r}))", shards=[s]).results[0]
            chk.append(got == srv.holder.fragment("i", "f", "standard", s).row_count(r))
        out["import"] = {"shards": nsh, "bits": nsh * per, "s": round(t_imp, 3),
                         "bits_per_s": round(nsh * per / t_imp, 1), "http_errors": len(errs),
                         "clients": args.import_clients,
                         "first_query_after_s": round(t_replay, 3),
                         "device_write_batches": int(getattr(gpu, "device_writes", 0) - w0),
                         "device_write_launches": int(getattr(gpu, "device_write_launches", 0) - wl0),
                         "fragments_cold_after_import": sum(f.is_cold() for f in frags), "fragments": len(frags),
                         "rss_growth_gb": round(_rss_gb() - rss0, 2), "device_matches_host": all(chk)}
    finally:
        srv.close()
    return out


def _rss_gb() -> float:
    with open("/proc/self/status") as fh:
        for line in fh:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1e6
    return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="queries per step (concurrent queries per batch)")
    ap.add_argument("--mode", choices=("disk", "synthetic"), default=os.environ.get("PILOSA_BENCH_MODE", "disk"))
    ap.add_argument("--cols", type=int, default=TOTAL_COLS)
    ap.add_argument("--rows", type=int, default=NROWS)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--clients", type=int, default=0,
                    help="disk mode: concurrent request threads; 0 = 2 on one GPU (1 / 2 / 3 / 4 / 6 threads "
                         "measured 221k / 236-237k / 234k / 232k / 225k Count q/s, profiles/r04_r/), 4 on a "
                         "mesh (every batch also waits on its collectives, so more must be in flight)")
    ap.add_argument("--data-dir", default=None, help="disk mode: reuse/keep fragment files under this dir")
    ap.add_argument("--cold-load", type=int, default=1,
                    help="disk mode: drop the fragment files from the page cache before loading (1) or not (0)")
    ap.add_argument("--keep-data", action="store_true")
    ap.add_argument("--verify", type=int, default=64, help="queries re-derived on the host (0 = skip)")
    ap.add_argument("--topn-batches", type=int, default=40,
                    help="also time this many batches of TopN(f, Row(f=a), n=100) (0 = skip)")
    ap.add_argument("--topn-src-batches", type=int, default=240,
                    help="timed src TopN requests (at least --topn-batches)")
    ap.add_argument("--topn-cache-batches", type=int, default=2000,
                    help="timed cache-only TopN requests (at least --topn-batches); ~0.1 ms each, so 2000 "
                         "is a ~0.2 s window (240 was ~25 ms: one stray millisecond moved the figure 5 %%)")
    ap.add_argument("--topn-batch", type=int, default=16, help="TopN queries per batch")
    ap.add_argument("--topn-cache", type=int, default=50000, help="rank-cache size per shard (reference default)")
    ap.add_argument("--topn-clients", type=int, default=3, help="request threads of the src TopN phase")
    ap.add_argument("--topn-cache-clients", type=int, default=1, help="request threads of the cache-only TopN phases")
    ap.add_argument("--topn-pairs-batches", type=int, default=1,
                    help="also time the pair-count src TopN path on this many batches (0 = skip)")
    ap.add_argument("--configs", default=os.environ.get("PILOSA_BENCH_CONFIGS", "4,5"),
                    help="also run BASELINE configs 4 (BSI) and 5 (time union) into extra (empty = skip)")
    ap.add_argument("--config-reps", type=int, default=20)
    ap.add_argument("--serve-seconds", type=float, default=5.0,
                    help="disk mode, 1 GPU: native-HTTP serving run on the same data dir (0 = skip)")
    ap.add_argument("--serve-conns", type=int, default=128)
    ap.add_argument("--serve-profile", default="", help="write folded stacks of the server during the mix here")
    ap.add_argument("--import-shards", type=int, default=64, help="serving phase: shards of the HTTP bulk import")
    ap.add_argument("--import-bits-per-shard", type=int, default=200_000)
    ap.add_argument("--import-clients", type=int, default=8)
    ap.add_argument("--mesh-breakdown", type=int, default=0,
                    help="mesh mode: trace this many Count and cache-only TopN requests (per-span time split)")
    ap.add_argument("--mesh", action="store_true",
                    help="run the multi-GPU product path (ShardMesh over RCCL, one rank per GPU) even at --gpus 1")
    ap.add_argument("--cpu-baseline-shards", type=int, default=0,
                    help="also time the host C++ roaring executor on this many shards (extrapolated)")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus > 1 or args.mesh):
        # launched without a launcher: start one rank per GPU ourselves
        # (nothing here has touched the GPU: no exec from a GPU process)
        raise SystemExit(_launch_ranks(args))
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={env_world} but --gpus {args.gpus}: launch one rank per GPU "
                         "(torch.distributed.run --nproc-per-node N ... --gpus N)")

    import torch
    import torch.distributed as dist

    world, rank, dev = setup_dist(mesh=args.mesh)
    if args.clients <= 0:
        args.clients = 2 if world == 1 else 4
    rng = np.random.default_rng(1234)
    nq = args.batch * (args.steps + args.warmup)
    ra = zipf_rows(rng, nq, args.rows)
    rb = zipf_rows(rng, nq, args.rows)
    queries = [f"Count(Intersect(Row(f={a}), Row(f={b})))" for a, b in zip(ra, rb)]

    fallback = None
    if args.mode == "disk" and args.data_dir is None:
        # every rank writes its shard range under TMPDIR: when any rank lacks
        # the space, all ranks time the synthesised arena instead of failing
        nshards = math.ceil(args.cols / SHARD_WIDTH)
        lo, hi = nshards * rank // world, nshards * (rank + 1) // world
        need = int(36e9 * (hi - lo) / 954 * (args.rows / NROWS))
        free = shutil.disk_usage(os.environ.get("TMPDIR") or "/tmp").free
        short = torch.tensor([1 if free < need else 0], dtype=torch.int64, device=dev)
        if world > 1:
            all_reduce(short, op=dist.ReduceOp.MAX)
        if int(short.item()):
            fallback = (f"--mode disk needs ~{need / 1e9:.1f} GB per rank under TMPDIR, a rank had "
                        f"{free / 1e9:.1f} GB free: timed the synthesised arena instead")
            args.mode = "synthetic"
    mesh_mode = args.mode == "disk" and (world > 1 or args.mesh)
    run = run_disk_mesh if mesh_mode else run_disk if args.mode == "disk" else run_synthetic
    elapsed, extra = run(args, world, rank, dev, queries, ra, rb)
    if world > 1 or args.mesh:
        extra.update({"backend": dist.get_backend(), "world_size": dist.get_world_size()})
    if fallback:
        extra["mode_fallback"] = fallback
    torch.cuda.empty_cache()
    which = [c for c in args.configs.split(",") if c in ("4", "5")]
    if which and args.mode == "disk":
        extra.update(bench_configs_disk(args, world, rank, dev, "".join(which)))
    else:
        if "4" in which:
            extra["config4_bsi"] = bench_bsi(args, world, rank, dev)
        if "5" in which:
            extra["config5_time_union"] = bench_time_union(args, world, rank, dev)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms = elapsed / args.steps * 1000.0
    qps = args.batch * args.steps / elapsed
    if "verify" in extra and not mesh_mode:   # mesh mode: rank 0 verified through the mesh
        ok = torch.tensor([0 if extra["verify"]["verified"] else 1], dtype=torch.int64, device=dev)
        if world > 1:
            all_reduce(ok)
        extra["verify"]["verified_all_ranks"] = int(ok.item()) == 0

    if rank == 0:
        nshards = math.ceil(args.cols / SHARD_WIDTH)
        size = f"{args.rows / 1e6:g}M-row x {args.cols / 1e9:g}B-col"
        rec = {"metric": f"PQL queries/sec (Count(Intersect(Row,Row))) on {size} set field",
               "value": round(qps, 2), "unit": "queries/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "bitmap(u64 words)",
               "data": "synthetic (zipf s=1.6 v=50 rows, 8 bits/column, deterministic per shard)"
                       + ("; written as Pilosa fragment files and loaded from disk" if args.mode == "disk" else ""),
               "config": {"model": f"set field f, {size} ({nshards} shards)", "global_batch": args.batch,
                          "seq_len": args.cols,
                          "parallelism": f"shard-range x{world}" + (
                              f" (ShardMesh over {extra.get('backend')})" if mesh_mode else
                              " + RCCL all-reduce" if world > 1 else "")},
               "verified": extra.get("verify", {}).get("verified_all_ranks"),
               "mode": args.mode, "extra": extra}
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
