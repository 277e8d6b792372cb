#!/usr/bin/env python3
"""Host/device breakdown of src-filtered TopN batches (cProfile)."""
import cProfile
import math
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import NROWS, SHARD_WIDTH, TOTAL_COLS, zipf_rows  # noqa: E402


def main():
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf
    from pilosa_amd.ops.topn import DeviceRankCache, topn_batch
    dev = torch.device("cuda", 0)
    S = math.ceil(TOTAL_COLS / SHARD_WIDTH)
    view = DeviceView(*_roaring.gen_zipf_arena(0, S, TOTAL_COLS, NROWS, 8.0, 1.6, 50.0, 1, 16), dev,
                      shards=list(range(S)))
    eng = GpuEngine(dev)
    cache = DeviceRankCache.from_view(view, k=50000)
    rng = np.random.default_rng(3)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    srcs = [Leaf(view, int(a)) for a in zipf_rows(rng, B, 1000)]
    topn_batch(eng, view, cache, srcs[:2], n=100)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.time()
    pr.enable()
    topn_batch(eng, view, cache, srcs, n=100)
    torch.cuda.synchronize()
    pr.disable()
    print("batch", B, "seconds", round(time.time() - t0, 3))
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
