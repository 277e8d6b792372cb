"""Host half of the two-field GroupBy count-matrix path (ops/groupby.py
emit_groups): lexicographic order, previous/limit paging and zero skipping
must equal the reference walk (executor.go:1241-1442), written out below as
a plain lexicographic product."""
import itertools

import numpy as np
import pytest

from pilosa_amd.ops.groupby import emit_groups


def _lex_product(cand, prev):
    k = len(cand)

    def rec(level, prefix):
        for r in cand[level]:
            key = prefix + (r,)
            if prev is not None and key < prev[:len(key)]:
                continue
            if level == k - 1:
                if prev is not None and key <= prev:
                    continue
                yield key
            else:
                yield from rec(level + 1, key)

    yield from rec(0, ())


def _walk(cand_a, cand_b, counts, prev, limit):
    out = []
    pos_a = {r: i for i, r in enumerate(cand_a)}
    pos_b = {r: i for i, r in enumerate(cand_b)}
    for ra, rb in _lex_product([cand_a, cand_b], prev):
        n = int(counts[pos_a[ra], pos_b[rb]])
        if n > 0:
            out.append((ra, rb, n))
            if len(out) >= limit:
                break
    return out


@pytest.mark.parametrize("seed", range(5))
def test_emit_groups_matches_reference_walk(seed):
    rng = np.random.default_rng(seed)
    cand_a = sorted(rng.choice(50, 12, replace=False).tolist())
    cand_b = sorted(rng.choice(40, 9, replace=False).tolist())
    counts = rng.integers(0, 3, size=(len(cand_a), len(cand_b)))
    prevs = [None, (cand_a[3], cand_b[4]), (cand_a[0], -1), (cand_a[-1], cand_b[-1]), (cand_a[5] + 1, 0)]
    for prev, limit in itertools.product(prevs, (1, 7, 1000)):
        assert emit_groups(cand_a, cand_b, counts, prev, limit) == _walk(cand_a, cand_b, counts, prev, limit)
