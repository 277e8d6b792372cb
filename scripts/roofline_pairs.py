#!/usr/bin/env python3
"""Roofline inputs of the Count(Intersect) pair kernel on the headline batch,
computed on the host from the same synthetic arena and query batch as
scripts/kbench.py (rng 1234, 4096 Zipf pairs, hot leaf first):

* compulsory bytes  = payload of every distinct container the batch touches
  (each (shard, key) unit reads each of its rows' containers at least once);
* referenced bytes  = what the kernel streams if nothing is reused across
  waves: the staged container once per run of equal leaf-0 rows in a
  64-query chunk, the partner container once per pair;
* pairs per batch by type.

Shards are i.i.d., so SAMPLE shards are generated and scaled to 954.
Usage: python scripts/roofline_pairs.py [--sample 12] [--batch 4096]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import NROWS, TOTAL_COLS, zipf_rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sample", type=int, default=12)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--cq", type=int, default=64)
    args = ap.parse_args()
    from pilosa_amd import _roaring
    S_all = 954
    rows, rowptr, sb, meta, payload = _roaring.gen_zipf_arena(0, args.sample, TOTAL_COLS, NROWS, 8.0, 1.6, 50.0, 1, 8)
    rows = np.asarray(rows, np.uint64)
    D = len(rows)
    rp = np.asarray(rowptr).reshape(args.sample, D + 1).astype(np.int64)
    sb = np.asarray(sb, np.int64)
    meta = np.asarray(meta, np.int64)
    typ = (meta >> 4) & 3
    n = (meta >> 6) & 0x1FFFF
    j = meta & 15
    nbytes = np.where(typ == 2, 8192, np.where(typ == 1, (n + 7) // 8 * 16, 16 + 32 * 64))  # runs: rough
    rng = np.random.default_rng(1234)
    ra, rb = zipf_rows(rng, args.batch), zipf_rows(rng, args.batch)
    # hot leaf first (ops/device.py _hot_leaf_first), then sort by (a, b)
    keys = np.concatenate([ra, rb])
    u, inv, cnt = np.unique(keys, return_inverse=True, return_counts=True)
    ca, cbb = cnt[inv[:len(ra)]], cnt[inv[len(ra):]]
    sw = (cbb > ca) | ((cbb == ca) & (rb < ra))
    A = np.where(sw, rb, ra)
    B = np.where(sw, ra, rb)
    o = np.lexsort((B, A))
    A, B = A[o], B[o]
    dense = {int(r): i for i, r in enumerate(rows.tolist())}
    comp = ref = 0
    ptype = {}
    for s in range(args.sample):
        base = sb[s]

        def conts(r):
            d = dense.get(int(r))
            if d is None:
                return {}
            lo, hi = rp[s, d], rp[s, d + 1]
            return {int(j[base + k]): base + k for k in range(lo, hi)}
        cache = {}

        def get(r):
            if r not in cache:
                cache[r] = conts(r)
            return cache[r]
        touched = set()
        for key in range(16):
            for c0 in range(0, args.batch, args.cq):
                prevA = None
                for q in range(c0, min(args.batch, c0 + args.cq)):
                    ca_, cb_ = get(A[q]).get(key), get(B[q]).get(key)
                    if ca_ is None or cb_ is None:
                        continue
                    t = (int(typ[ca_]), int(typ[cb_]))
                    ptype[t] = ptype.get(t, 0) + 1
                    touched.add(ca_)
                    touched.add(cb_)
                    if A[q] != prevA:
                        ref += int(nbytes[ca_])
                        prevA = A[q]
                    ref += int(nbytes[cb_])
        comp += int(nbytes[list(touched)].sum()) if touched else 0
    f = S_all / args.sample
    names = {1: "array", 2: "bitmap", 3: "run"}
    pairs = {f"{names[a]}&{names[b]}": round(c * f) for (a, b), c in sorted(ptype.items())}
    out = {"sample_shards": args.sample, "batch": args.batch, "pairs_per_batch": pairs,
           "pairs_total": sum(pairs.values()), "compulsory_bytes": round(comp * f),
           "referenced_bytes": round(ref * f),
           "hbm_floor_ms_at_6.3TBps": round(comp * f / 6.3e12 * 1e3, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
