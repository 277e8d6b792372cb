#!/usr/bin/env python3
"""Secondary BASELINE configs on one GPU (bench.py covers config 2 and TopN):

  config 4  BSI int field, 1B columns (fill 50 %, values in [-1000, 1e6], depth 20):
            Sum(field=v), Count(Row(v > x)), Count(Row(v >< [a, b])), Min/Max(field=v)
  config 5  time-quantum field: Count over a Union of the covering views of a
            time range (2 day views + 5 hour views, Zipf rows, 1B columns)

Every query is timed end to end through the device path used by the executor
(GpuEngine / kernels), one query at a time.  Prints one JSON line per config.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import SHARD_WIDTH, TOTAL_COLS, zipf_rows  # noqa: E402


def timed(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def config4(args, dev):
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf

    S = math.ceil(args.cols / SHARD_WIDTH)
    depth = 20
    t0 = time.time()
    arena = _roaring.gen_bsi_arena(0, S, args.cols, depth, 0.5, -1000, 1_000_000, 7, 16)
    gen_s = time.time() - t0
    bv = DeviceView(*arena, dev, shards=list(range(S)))
    del arena
    eng = GpuEngine(dev)
    res = {"config": "BSI int field, 1B cols, depth 20, fill 0.5", "gen_s": round(gen_s, 1),
           "hbm_bytes": bv.nbytes(), "queries": {}}
    rng = np.random.default_rng(5)

    def q_sum():
        s, n = eng.bsi_sum_async([None], bv, depth)
        return int(s.cpu()[0]), int(n.cpu()[0])

    def q_gt():
        x = int(rng.integers(0, 1_000_000))
        rv = eng.bsi_range_view(bv, depth, ">", x)
        return int(eng.count([Leaf(rv, 0)])[0])

    def q_gt_fused():
        x = int(rng.integers(0, 1_000_000))
        return int(eng.bsi_range_count_async(bv, depth, ">", x).item())

    def q_between():
        a = int(rng.integers(0, 900_000))
        rv = eng.bsi_range_view(bv, depth, "between", a, a + 50_000)
        return int(eng.count([Leaf(rv, 0)])[0])

    def q_min():
        return int(eng.bsi_minmax(None, bv, depth)[..., 0].max())

    # filter rows for batched Sum(Row(f=r), field=v): a Zipf set field, 1 bit/column
    farena = _roaring.gen_zipf_arena(0, S, args.cols, 1000, 1.0, 1.6, 50.0, 11, 16)
    fv = DeviceView(*farena, dev, shards=list(range(S)))
    del farena
    FB = 32

    def q_sum_filtered_batch():
        rows = rng.integers(0, 200, size=FB)
        s, n = eng.bsi_sum_async([Leaf(fv, int(r)) for r in rows], bv, depth)
        return int(s.cpu()[0]), int(n.cpu()[0])

    for name, fn in (("Sum(field=v)", q_sum), ("Count(Row(v > x))", q_gt),
                     ("Count(Row(v > x)) fused predicate+count", q_gt_fused), ("Count(Row(v >< [a,b]))", q_between),
                     ("Min/Max(field=v)", q_min)):
        dt, out = timed(fn, args.reps)
        res["queries"][name] = {"ms": round(dt * 1000, 3), "qps": round(1 / dt, 1), "sample": out}
    dt, out = timed(q_sum_filtered_batch, args.reps)
    res["queries"][f"Sum(Row(f=r), field=v) x{FB} filters per launch"] = {
        "ms_per_batch": round(dt * 1000, 3), "qps": round(FB / dt, 1), "sample": out}
    del fv
    s, n = q_sum()
    res["check"] = {"count": n, "mean": s / max(n, 1),
                    "expected_count": args.cols * 0.5, "expected_mean": (1_000_000 - 1000) / 2}
    del bv
    torch.cuda.empty_cache()
    return res


def config5(args, dev):
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf, Op

    S = math.ceil(args.cols / SHARD_WIDTH)
    nrows = 100_000
    views = []
    t0 = time.time()
    # day views hold ~4x the bits of hour views
    for k, bpc in enumerate([1.0, 1.0, 0.25, 0.25, 0.25, 0.25, 0.25]):
        arena = _roaring.gen_zipf_arena(0, S, args.cols, nrows, bpc, 1.6, 50.0, 100 + k, 16)
        views.append(DeviceView(*arena, dev, shards=list(range(S))))
        del arena
    gen_s = time.time() - t0
    eng = GpuEngine(dev)
    rng = np.random.default_rng(9)
    B = args.batch

    def q_union():
        rows = zipf_rows(rng, B, nrows)
        exprs = [Op("or", tuple(Leaf(v, int(r)) for v in views)) for r in rows]
        return int(eng.count(exprs).sum())

    dt, out = timed(q_union, args.reps)
    res = {"config": "time-quantum field, Union of 7 covering views (2 D + 5 H), 100k rows x 1B cols",
           "gen_s": round(gen_s, 1), "hbm_bytes": sum(v.nbytes() for v in views), "batch": B,
           "queries": {"Count(Row(t=r, from, to))": {"ms_per_batch": round(dt * 1000, 2), "qps": round(B / dt, 1)}}}
    del views
    torch.cuda.empty_cache()
    return res


def config_rowops(args, dev):
    """Row-level calls on the config-2 index (1M rows x 1B cols, 8 bits per
    column): Rows listing (rows_kernel), Rows(column=), Shift (expr_dense +
    shift_dense + spill count), Count(Intersect(Shift(a), b))."""
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf, Op

    S = math.ceil(args.cols / SHARD_WIDTH)
    nrows = 1_000_000
    t0 = time.time()
    arena = _roaring.gen_zipf_arena(0, S, args.cols, nrows, 8.0, 1.6, 50.0, 1, 16)
    gen_s = time.time() - t0
    view = DeviceView(*arena, dev, shards=list(range(S)))
    del arena
    eng = GpuEngine(dev)
    rng = np.random.default_rng(3)
    q = {}

    def rec(name, fn):
        dt, out = timed(fn, args.reps)
        q[name] = {"ms": round(dt * 1000, 3), "result": out}

    rec("Rows(f)", lambda: len(eng.row_ids(view)))
    rec("Rows(f, column=c)", lambda: len(eng.row_ids(view, int(rng.integers(0, args.cols)))))

    def shift_count(a, n, b=None):
        main, spill = eng.shift_views(Leaf(view, a), n)
        if b is None:
            return int(eng.count([Leaf(main, 0), Leaf(spill, 0)]).sum())
        return int(eng.count([Op("and", (Leaf(main, 0), Leaf(view, b)))])[0])

    rec("Count(Shift(Row(f=0), n=1))", lambda: shift_count(0, 1))
    rec("Count(Shift(Row(f=500), n=1000))", lambda: shift_count(500, 1000))
    rec("Count(Intersect(Shift(Row(f=0), n=1), Row(f=1)))", lambda: shift_count(0, 1, 1))
    rec("Count(Row(f=0))", lambda: int(eng.count([Leaf(view, 0)])[0]))
    res = {"config": "row ops on the config-2 index (1M rows x 1B cols)", "gen_s": round(gen_s, 1),
           "hbm_bytes": view.nbytes(), "queries": q}
    del view
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cols", type=int, default=TOTAL_COLS)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--only", default="4,5")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    if "4" in args.only:
        print(json.dumps(config4(args, dev)), flush=True)
    if "5" in args.only:
        print(json.dumps(config5(args, dev)), flush=True)
    if "r" in args.only:
        print(json.dumps(config_rowops(args, dev)), flush=True)


if __name__ == "__main__":
    main()
