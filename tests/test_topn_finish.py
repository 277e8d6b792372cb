"""The device-side TopN finish (sort by query, count desc, id asc; trim to n)
agrees with the host one (ops/topn_index.py finish_batch_dev / finish_batch;
reference ordering: executor.go Pairs sort, cache.go:443-470)."""
import numpy as np
import torch

from pilosa_amd.ops.topn_index import finish_batch, finish_batch_dev


def _as_lists(res):
    return [[(p.id, p.count) for p in r] for r in res]


def test_finish_dev_matches_host():
    rng = np.random.default_rng(5)
    space = np.unique(rng.integers(0, 1 << 40, 3000).astype(np.uint64))
    A = len(space)
    Q = 7
    P = 5000
    pq = rng.integers(0, Q, P)
    pa = rng.integers(0, A, P)
    # unique (q, a) pairs like the candidate sets; many ties in count
    key = np.unique(pq * A + pa)
    pq, pa = key // A, key % A
    cnt = rng.integers(0, 6, len(pq)).astype(np.int64)
    ns = [0, 1, 3, 10, 100, 5, 2]
    want = finish_batch(space, Q, pq, pa, cnt, ns)
    got = finish_batch_dev(space, Q, torch.from_numpy(pq), torch.from_numpy(pa).to(torch.int32),
                           torch.from_numpy(cnt), ns)
    assert _as_lists(got) == _as_lists(want)


def test_finish_dev_empty():
    space = np.arange(10, dtype=np.uint64)
    e = torch.zeros(0, dtype=torch.int64)
    assert finish_batch_dev(space, 3, e, e, e, [1, 2, 3]) == [[], [], []]
    z = torch.zeros(4, dtype=torch.int64)
    assert finish_batch_dev(space, 2, z, z, z, [1, 1]) == [[], []]


def test_finish_dev_composite_key_and_fallback_agree(monkeypatch):
    """The one-sort composite-key finish (query | ~count | acc index packed in
    an int64) and the three-stable-sort path it falls back to when the key
    would not fit give the host answer, for random batches with large counts
    and n past the candidate count."""
    rng = np.random.default_rng(11)
    for t in range(60):
        Q = int(rng.integers(1, 40))
        space = np.sort(rng.choice(1 << 50, int(rng.integers(1, 5000)), replace=False)).astype(np.uint64)
        A = len(space)
        key = np.unique(rng.integers(0, Q, 3000) * A + rng.integers(0, A, 3000))
        pq, pa = key // A, key % A
        cnt = rng.integers(0, 1 << 31, len(pq)) if t % 2 else rng.integers(0, 5, len(pq))
        ns = [int(x) for x in rng.integers(0, 120, Q)]
        want = _as_lists(finish_batch(space, Q, pq, pa, cnt, ns))
        got = finish_batch_dev(space, Q, torch.from_numpy(pq).to(torch.int32), torch.from_numpy(pa).to(torch.int32),
                               torch.from_numpy(cnt).to(torch.int64), ns)
        assert _as_lists(got) == want
    # a space too large for the packed key takes the sort-chain path
    big = np.arange(1 << 33, (1 << 33) + 64, dtype=np.uint64)
    pq = torch.tensor([0, 0, 1], dtype=torch.int64)
    pa = torch.tensor([3, 5, 3], dtype=torch.int64)
    cnt = torch.tensor([7, 9, 1], dtype=torch.int64)

    class Huge(np.ndarray):
        def __len__(self):
            return 1 << 40
    huge = big.view(Huge)
    assert _as_lists(finish_batch_dev(huge, 2, pq, pa, cnt, [0, 0])) == \
        _as_lists(finish_batch(big, 2, pq.numpy(), pa.numpy(), cnt.numpy(), [0, 0]))
