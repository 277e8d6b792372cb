"""bench.py's CPU stand-in (host roaring executor per shard, BASELINE.md
'use our CPU oracle as a stand-in') counts the same as a numpy oracle."""
import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_cpu_host_standin_matches_numpy():
    import bench
    from pilosa_amd import _roaring as R
    args = types.SimpleNamespace(cpu_baseline_shards=2, cols=1_000_000_000, rows=1_000_000, threads=4)
    rng = np.random.default_rng(7)
    ra, rb = bench.zipf_rows(rng, 32), bench.zipf_rows(rng, 32)
    out = bench.bench_cpu_host(args, ra, rb, 954, nq=32)
    arena = R.gen_zipf_arena(0, 2, args.cols, args.rows, 8.0, 1.6, 50.0, 1, 4)
    want = 0
    for s in range(2):
        v = R.arena_shard_bitmap(*arena, s).slice()
        rows, lo = v >> np.uint64(20), v & np.uint64((1 << 20) - 1)
        for a, b in zip(ra, rb):
            want += np.intersect1d(lo[rows == a], lo[rows == b]).size
    assert out["checksum"] == want
    assert out["shards_timed"] == 2 and out["queries"] == 32 and out["qps_per_core"] > 0
