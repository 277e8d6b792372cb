"""Write-path throughput with a GPU-resident view: bulk imports (and point
Set()s) land in the host fragments, then the next read refreshes the HBM
arena -- on the GPU from the recorded write batches (write_kernels.hip,
K11/K12) or, with PILOSA_DEVICE_WRITES=0, by rebuilding the touched
containers on the host and uploading them.

    python scripts/import_bench.py --shards 64 --rows 1000 --batch 1000000
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=64)
    ap.add_argument("--rows", type=int, default=1000)
    ap.add_argument("--fill", type=int, default=2_000_000, help="bits per shard before the timed imports")
    ap.add_argument("--batch", type=int, default=1_000_000, help="bits per import batch (all shards)")
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--points", type=int, default=2000, help="single-bit Set() writes between reads")
    args = ap.parse_args()

    import torch
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    SW = 1 << 20
    rng = np.random.default_rng(0)
    d = tempfile.mkdtemp(prefix="pilosa_import_bench_", dir="/tmp")
    h = Holder(d).open()
    idx = h.create_index("i")
    f = idx.create_field("f")
    S = args.shards
    for s in range(S):
        rows = (rng.zipf(1.5, args.fill) % args.rows).astype(np.uint64)
        cols = (np.uint64(s * SW) + rng.integers(0, SW, args.fill).astype(np.uint64))
        f.import_bits(rows, cols)
    g = GpuExecutor(h, "cuda:0")
    shards = list(range(S))
    g.view_arena("i", "f", "standard", shards)
    torch.cuda.synchronize()
    out = {"mode": "device" if g.device_writes_on else "host", "shards": S, "rows": args.rows,
           "fill_bits_per_shard": args.fill, "batch_bits": args.batch}
    t_imp = t_ref = 0.0
    for b in range(args.batches):
        rows = (rng.zipf(1.5, args.batch) % args.rows).astype(np.uint64)
        cols = rng.integers(0, S * SW, args.batch).astype(np.uint64)
        t0 = time.perf_counter()
        f.import_bits(rows, cols)
        t1 = time.perf_counter()
        g.view_arena("i", "f", "standard", shards)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if b:   # first batch warms the kernels
            t_imp += t1 - t0
            t_ref += t2 - t1
    nb = args.batches - 1
    out["import_s_per_batch"] = round(t_imp / nb, 4)
    out["arena_refresh_s_per_batch"] = round(t_ref / nb, 4)
    out["bits_per_s_end_to_end"] = round(args.batch / ((t_imp + t_ref) / nb))
    # point writes: Set() one bit at a time, then one read
    frags = [f.view("standard").fragment(s) for s in shards]
    t0 = time.perf_counter()
    for k in range(args.points):
        s = int(rng.integers(0, S))
        frags[s].set_bit(int(rng.integers(0, args.rows)), s * SW + int(rng.integers(0, SW)))
    t1 = time.perf_counter()
    g.view_arena("i", "f", "standard", shards)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["points"] = args.points
    out["point_set_s"] = round(t1 - t0, 4)
    out["point_refresh_s"] = round(t2 - t1, 4)
    out["rebuilds"] = g.rebuilds
    out["device_writes"] = g.device_writes
    out["row_updates"] = g.row_updates
    # exactness: the refreshed arena answers like the host
    from pilosa_amd.ops.device import GpuEngine, Leaf
    dv = g.view_arena("i", "f", "standard", shards)
    eng = GpuEngine(torch.device("cuda:0"))
    probe = [int(r) for r in rng.integers(0, args.rows, 16)]
    got = eng.count([Leaf(dv, dv.dense(r)) for r in probe])
    want = [sum(fr.row_count(r) for fr in frags) for r in probe]
    out["verified"] = [int(x) for x in got] == want
    print(json.dumps(out))
    h.close()


if __name__ == "__main__":
    main()
