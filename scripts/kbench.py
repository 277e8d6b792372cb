#!/usr/bin/env python3
"""Kernel-level A/B harness on the headline dataset: times the device half
(launch_count) of a Count(Intersect) batch for several engine settings with
HIP events.  Usage: python scripts/kbench.py [--batch 1024] [--reps 5] [--shards N]"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the A/B module: the shipped variants plus every rejected one and the
# cost-isolation skeletons (python -m pilosa_amd.native.build --kbench)
os.environ.setdefault("PILOSA_HIPKERNELS", "_hipkernels_kbench")
sys.path.insert(0, ROOT)

from bench import NROWS, SHARD_WIDTH, TOTAL_COLS, zipf_rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shards", type=int, default=0, help="0 = full 954")
    ap.add_argument("--cq", default="0,32,64", help="pair-kernel chunk sizes (queries per wave)")
    ap.add_argument("--no-tile", action="store_true", help="skip the generic tile kernel")
    ap.add_argument("--variants", default="", help="extra kernel variants at --cq's first size, e.g. 4,5 (38@8: at 8 queries per wave)")
    args = ap.parse_args()
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine
    from pilosa_amd.ops.planner import NativeCountCompiler

    dev = torch.device("cuda", 0)
    nshards = args.shards or math.ceil(TOTAL_COLS / SHARD_WIDTH)
    arena = _roaring.gen_zipf_arena(0, nshards, TOTAL_COLS, NROWS, 8.0, 1.6, 50.0, 1, 16)
    view = DeviceView(*arena, dev, shards=list(range(nshards)))
    del arena
    rng = np.random.default_rng(1234)
    ra, rb = zipf_rows(rng, args.batch), zipf_rows(rng, args.batch)
    qs = [f"Count(Intersect(Row(f={a}), Row(f={b})))" for a, b in zip(ra, rb)]
    progs, views, S = NativeCountCompiler({"f": view}).compile(qs)
    results = {}
    ref = None
    configs = [] if args.no_tile else [("tile", {"use_and2": False})]
    configs += [(f"and2_cq{c}", {"and2_cq": int(c), "and2_variant": 1}) for c in args.cq.split(",") if c]
    cq0 = int(args.cq.split(",")[0]) if args.cq else 64
    for v in args.variants.split(","):
        if not v:
            continue
        vv, _, cq = v.partition("@")   # "38@8": variant 38 at 8 queries per wave
        cq = int(cq) if cq else cq0
        configs.append((f"and2var{vv}_cq{cq}", {"and2_cq": cq, "and2_variant": int(vv)}))
    for name, cfg in configs:
        eng = GpuEngine(dev)
        for k, v in cfg.items():
            setattr(eng, k, v)
        h = eng.prepare_progs(progs, views, S)
        out = eng.launch_count(h)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        if ref is None:
            ref = got
        ok = bool(np.array_equal(got, ref)) or name.startswith("dbg")
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.launch_count(h)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        results[name] = {"ms_min": round(min(ts), 3), "ms_med": round(sorted(ts)[len(ts) // 2], 3), "match": ok}
        print(name, results[name], flush=True)
    print(json.dumps({"batch": args.batch, "shards": nshards, "results": results}))


if __name__ == "__main__":
    main()
