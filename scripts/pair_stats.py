#!/usr/bin/env python3
"""Work profile of the pair kernel on the headline batch (host-side, same
arena / batch as scripts/kbench.py): per (unit, 64-query chunk) the v6 walk
-- pairs, stagings of A (a new leaf-0 container), A and B types and sizes,
run lengths -- so kernel restructures can be priced before they are built.
Usage: python scripts/pair_stats.py [--sample 2] [--batch 4096]"""
import argparse
import collections
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import NROWS, TOTAL_COLS, zipf_rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sample", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--cq", type=int, default=64)
    args = ap.parse_args()
    from pilosa_amd import _roaring
    rows, rowptr, sb, meta, payload = _roaring.gen_zipf_arena(0, args.sample, TOTAL_COLS, NROWS, 8.0, 1.6, 50.0, 1, 8)
    rows = np.asarray(rows, np.uint64)
    D = len(rows)
    rp = np.asarray(rowptr).reshape(args.sample, D + 1).astype(np.int64)
    sb = np.asarray(sb, np.int64)
    meta = np.asarray(meta, np.int64)
    typ = (meta >> 4) & 3
    n = (meta >> 6) & 0x1FFFF
    jj = meta & 15
    rng = np.random.default_rng(1234)
    ra, rb = zipf_rows(rng, args.batch), zipf_rows(rng, args.batch)
    keys = np.concatenate([ra, rb])
    u, inv, cnt = np.unique(keys, return_inverse=True, return_counts=True)
    ca, cbb = cnt[inv[:len(ra)]], cnt[inv[len(ra):]]
    sw = (cbb > ca) | ((cbb == ca) & (rb < ra))
    A = np.where(sw, rb, ra)
    B = np.where(sw, ra, rb)
    o = np.lexsort((B, A))
    A, B = A[o], B[o]
    dense = {int(r): i for i, r in enumerate(rows.tolist())}
    st = collections.Counter()
    nb_hist = collections.Counter()
    na_stage_hist = collections.Counter()
    runlen = collections.Counter()
    pairs_per_wave = []

    def bucket(x):
        for b in (16, 64, 256, 512, 1024, 2048, 4096):
            if x <= b:
                return b
        return 99999
    for s in range(args.sample):
        base = sb[s]
        memo = {}

        def conts(r):
            if r in memo:
                return memo[r]
            d = dense.get(int(r))
            out = {}
            if d is not None:
                lo, hi = rp[s, d], rp[s, d + 1]
                out = {int(jj[base + k]): base + k for k in range(lo, hi)}
            memo[r] = out
            return out
        for key in range(16):
            for c0 in range(0, args.batch, args.cq):
                prev = None
                run = 0
                npairs = 0
                for q in range(c0, min(args.batch, c0 + args.cq)):
                    ia, ib = conts(A[q]).get(key), conts(B[q]).get(key)
                    if ia is None or ib is None:
                        continue
                    npairs += 1
                    ta, tb = int(typ[ia]), int(typ[ib])
                    st[f"pair {('-', 'arr', 'bmp', 'run')[ta]}&{('-', 'arr', 'bmp', 'run')[tb]}"] += 1
                    if tb == 1:
                        nb_hist[bucket(int(n[ib]))] += 1
                    if ia != prev:
                        if prev is not None:
                            runlen[min(run, 64)] += 1
                        run = 0
                        st["stagings"] += 1
                        st[f"stage {('-', 'arr', 'bmp', 'run')[ta]}"] += 1
                        if ta == 1:
                            na_stage_hist[bucket(int(n[ia]))] += 1
                        prev = ia
                    run += 1
                if prev is not None:
                    runlen[min(run, 64)] += 1
                pairs_per_wave.append(npairs)
    f = 954 / args.sample
    out = {k: round(v * f) for k, v in sorted(st.items())}
    out["B_array_size_hist"] = {k: round(v * f) for k, v in sorted(nb_hist.items())}
    out["A_array_staged_size_hist"] = {k: round(v * f) for k, v in sorted(na_stage_hist.items())}
    rl = sorted(runlen.items())
    out["run_length_hist"] = {k: round(v * f) for k, v in rl}
    out["one_off_runs"] = round(runlen[1] * f)
    ppw = np.asarray(pairs_per_wave)
    out["pairs_per_wave"] = {"mean": float(ppw.mean()), "p50": float(np.median(ppw)), "max": int(ppw.max())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
