#!/usr/bin/env python3
"""Kernel-level timing of the slot-index TopN (ops/topn_index.py) on the
headline arena: phase-1 kernel per src class (hot / warm / cold src rows),
optionally with PILOSA_TOPN_DBG cost isolation (bit 0 skip histogram, bit 1
skip walk; results are then wrong, timings isolate the parts)."""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the A/B module: the shipped variants plus every rejected one and the
# cost-isolation skeletons (python -m pilosa_amd.native.build --kbench)
os.environ.setdefault("PILOSA_HIPKERNELS", "_hipkernels_kbench")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cols", type=int, default=1_000_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import NROWS, SHARD_WIDTH
    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf
    from pilosa_amd.ops.topn import DeviceRankCache
    from pilosa_amd.ops.topn_index import DeviceTopNIndex

    dev = torch.device("cuda", 0)
    S = math.ceil(args.cols / SHARD_WIDTH)
    arena = _roaring.gen_zipf_arena(0, S, args.cols, NROWS, 8.0, 1.6, 50.0, 1, 16)
    view = DeviceView(*arena, dev, shards=list(range(S)))
    del arena
    eng = GpuEngine(dev)
    cache = DeviceRankCache.from_view(view, k=50000)
    t0 = time.perf_counter()
    idx = DeviceTopNIndex(view, cache)
    torch.cuda.synchronize()
    out = {"shards": S, "index_build_s": round(time.perf_counter() - t0, 2), "H32": idx.H32, "H16": idx.H16,
           "lds_bytes": idx.lds, "hot_ranks": idx.R, "slot_entries": idx.entries, "classes": {},
           # set bits of the hot-rank rows: the values one hot-rank launch streams
           # (each counted for all its queries; PMC instructions / this = per value)
           "hot_values_per_launch": int(np.asarray(cache.counts)[:, :idx.R].astype(np.int64).sum())}
    B = args.batch
    from bench import zipf_rows
    mix_rows = [int(r) for r in zipf_rows(np.random.default_rng(7), B, 1000)]
    for name, rows in ((f"hot 0-{B - 1}", range(0, B)), (f"warm 100-{99 + B}", range(100, 100 + B)),
                       ("cold 900-915", range(900, 900 + B)), ("mix", mix_rows)):
        srcs = [Leaf(view, r) for r in list(rows)[:B]]
        src = eng.materialize_batch(srcs, idx.S)
        hot = idx.hot_counts(src, B)
        acc, ns_t, th_t, hist = idx.phase1(src, B, [100] * B, [1] * B, keep_hist=True, hot=hot)
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        for _ in range(args.reps):
            hot = idx.hot_counts(src, B)
        e1.record()
        for _ in range(args.reps):
            idx._launch(1, B, src, ns_t, th_t, acc=acc, hist=hist[0], hot_cnt=hot, tail_built=hist[1])
        e2.record()
        torch.cuda.synchronize()
        ms_hot = e0.elapsed_time(e1) / args.reps
        ms = e1.elapsed_time(e2) / args.reps
        nsrc = int(src[0].sum().item())
        out["classes"][name] = {"hot_ms": round(ms_hot, 3), "phase1_ms": round(ms, 3), "src_bits": nsrc,
                                "dbg": int(os.environ.get("PILOSA_TOPN_DBG", "0"))}
    if not int(os.environ.get("PILOSA_TOPN_DBG", "0")):
        # the bench mix (src rows Zipf over the 1000 hottest): end to end and
        # a synchronised breakdown of one batch
        from pilosa_amd.ops.topn_index import finish_batch_dev
        rng = np.random.default_rng(99)
        batches = [[Leaf(view, int(r)) for r in zipf_rows(rng, B, 1000)] for _ in range(args.reps + 1)]
        idx.topn(eng, batches[0], [100] * B, [1] * B)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in batches[1:]:
            idx.topn(eng, b, [100] * B, [1] * B)
        torch.cuda.synchronize()
        e2e = (time.perf_counter() - t0) / args.reps * 1000
        parts = {}

        def mark(name, t):
            torch.cuda.synchronize()
            now = time.perf_counter()
            parts[name] = round((now - t) * 1000, 3)
            return now
        srcs = batches[1]
        t = time.perf_counter()
        src = idx.materialize(eng, srcs)
        t = mark("materialize", t)
        hot = idx.hot_counts(src, B)
        t = mark("hot", t)
        acc, ns_t, th_t, hist = idx.phase1(src, B, [100] * B, [1] * B, keep_hist=True, hot=hot)
        t = mark("phase1", t)
        pq, pa = idx._candidates(acc, None)
        t = mark("candidates", t)
        cnt = idx.phase2(src, B, ns_t, th_t, pq, pa, hist=hist, hot=hot)
        t = mark("phase2", t)
        finish_batch_dev(idx.space, B, pq, pa, cnt, [100] * B)
        mark("finish", t)
        out["mix"] = {"e2e_ms_per_batch": round(e2e, 3), "qps": round(B / e2e * 1000, 1), "parts_ms": parts,
                      "candidates": int(pa.numel()), "src_bits": int(src[0].sum().item())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
