"""A/B of the Count(Union) kernels on the BASELINE config-5 data (bench.py
bench_time_union: 2 day + 5 hour views of a 1M-row Zipf time field over 1B
columns): union_count_kernel (variant 1) vs union_count2_kernel (variant 2),
the same query batches, results compared."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=0, help="0 = all 954")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, GpuEngine
    dev = torch.device("cuda:0")
    n = args.shards or math.ceil(bench.TOTAL_COLS / bench.SHARD_WIDTH)
    views = []
    for k, bpc in enumerate([1.0, 1.0, 0.25, 0.25, 0.25, 0.25, 0.25]):
        arena = _roaring.gen_zipf_arena(0, n, bench.TOTAL_COLS, bench.NROWS, bpc, 1.6, 50.0, 100 + k, 16)
        views.append(DeviceView(*arena, dev, shards=list(range(n))))
        del arena
    eng = GpuEngine(dev)
    rng = np.random.default_rng(9)
    batches = [bench.zipf_rows(rng, args.batch, bench.NROWS) for _ in range(args.reps)]
    res = {}
    outs = {}
    for variant in (1, 2, 1, 2):
        eng.union_variant = variant
        progs = [GpuEngine.union_programs(np.stack([v.dense_many(rows) for v in views], axis=1))
                 for rows in batches]
        eng.launch_count(eng.prepare_progs(progs[0], views, n))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got = [eng.launch_count(eng.prepare_progs(p, views, n)) for p in progs]
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / len(progs) * 1000
        outs[variant] = torch.cat(got).cpu().numpy()
        res[f"v{variant}"] = {"ms_per_batch": round(ms, 2), "qps": round(args.batch / ms * 1000, 1)}
        print(variant, res[f"v{variant}"], flush=True)
    res["match"] = bool((outs[1] == outs[2]).all())
    print(json.dumps({"shards": n, "batch": args.batch, "results": res}))


if __name__ == "__main__":
    main()
