#!/usr/bin/env python3
"""Hot-rank TopN kernel in isolation (ops/topn_index.py hot_counts) for
profiling: --shards of the Zipf arena, 16 src rows (--src first row, or "mix"
for the bench's Zipf draw), --reps launches."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--src", default="900")
    args = ap.parse_args()
    import torch

    from bench import NROWS, SHARD_WIDTH
    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf
    from pilosa_amd.ops.topn import DeviceRankCache
    from pilosa_amd.ops.topn_index import DeviceTopNIndex

    dev = torch.device("cuda", 0)
    S = args.shards
    arena = _roaring.gen_zipf_arena(0, S, S * SHARD_WIDTH, NROWS, 8.0, 1.6, 50.0, 1, 16)
    view = DeviceView(*arena, dev, shards=list(range(S)))
    del arena
    eng = GpuEngine(dev)
    cache = DeviceRankCache.from_view(view, k=50000)
    idx = DeviceTopNIndex(view, cache)
    if args.src == "mix":   # the bench's src rows: Zipf over the 1000 hottest
        import numpy as np

        from bench import zipf_rows
        rows = [int(r) for r in zipf_rows(np.random.default_rng(99), 16, 1000)]
    else:
        rows = [int(args.src) + i for i in range(16)]
    src = eng.materialize_batch([Leaf(view, r) for r in rows], S)
    idx.hot_counts(src, 16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        idx.hot_counts(src, 16)
    torch.cuda.synchronize()
    print(json.dumps({"shards": S, "hot_ranks": idx.R, "hot_ms": round((time.perf_counter() - t0) / args.reps * 1e3, 3)}))


if __name__ == "__main__":
    main()
