#!/usr/bin/env python3
"""Row-pair count matrices: i8 MFMA vs VALU popcount (kernels/bitgemm.hip).

Dense rows (~50 % fill, bitmap containers) of one set field over S shards;
times densify and the count-matrix kernel per mode for R x R matrices."""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=64)
    ap.add_argument("--rows", default="32,64,128,256")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    from pilosa_amd import _roaring
    from pilosa_amd.ops.device import DeviceView, kernels
    from pilosa_amd.ops.groupby import WORDS_PER_SHARD, _vd

    dev = torch.device("cuda", 0)
    S = args.shards
    # densify cost on a real arena (Zipf rows, 8 bits/column) ...
    arena = _roaring.gen_zipf_arena(0, S, S << 20, 100_000, 8.0, 1.6, 50.0, 3, 16)
    view = DeviceView(*arena, dev, shards=list(range(S)))
    del arena
    ext = kernels()
    vd = _vd(view)
    out = {"shards": S, "K_bits": S << 20, "results": {}}
    for R in [int(r) for r in args.rows.split(",")]:
        rows = torch.arange(R, dtype=torch.int64, device=dev)
        kw = S * WORDS_PER_SHARD
        A = torch.empty(R * kw, dtype=torch.int64, device=dev)
        ext.densify(vd, rows, 0, S, A)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ext.densify(vd, rows, 0, S, A)
        torch.cuda.synchronize()
        t_dense = time.perf_counter() - t0
        res = {"densify_ms": round(t_dense * 1000, 2)}
        # ... and the count matrix on random 50 %-dense rows (content does not
        # change the kernels' work)
        A = torch.randint(-(1 << 62), 1 << 62, (R * kw,), dtype=torch.int64, device=dev)
        ref = None
        for mode, name in ((0, "valu"), (1, "mfma_lds_table"), (2, "mfma64_mul_unpack")):
            tiles = math.ceil(R / (128 if mode == 2 else 64)) ** 2
            splits = max(1, min(kw // 8, math.ceil(2048 / tiles)))
            C = torch.zeros(R * R, dtype=torch.int32, device=dev)
            ext.bitgemm(A, A, R, R, kw, splits, mode, C)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                C.zero_()
                ext.bitgemm(A, A, R, R, kw, splits, mode, C)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            macs = R * R * (S << 20)
            res[name] = {"ms": round(ms, 3), "Tbitops_per_s": round(macs / ms / 1e9, 1)}
            if ref is None:
                ref = C.clone()
            else:
                res[f"match_{name}"] = bool(torch.equal(ref, C))
        out["results"][R] = res
        del A
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
