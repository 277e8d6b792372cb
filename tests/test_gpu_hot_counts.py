"""Hot-rank TopN counts (kernels/topn_kernels.hip ``topn_hot_kernel``) against
a plain PyTorch fp32 reference on the headline's container mix.

A Zipf arena with the bench's density profile (bits_per_col 8, s 1.6, v 50)
puts bitmap containers at the top ranks, 1k-4k-value arrays after them and
short arrays in the tail, so one launch runs the wave-cooperative path
(bitmaps, big arrays), the quarter-wave path (mid-size arrays) and the
lane-owned path (short arrays) of the kernel, at every lane-owned and
mid-size bound (PILOSA_TOPN_SMALL_N / PILOSA_TOPN_MID_N) and with either
table build (PILOSA_TOPN_TBUILD_MIN: 65537 sends every src to the atomic
build).  The reference builds each
shard's hot rows and src rows as dense 0/1 fp32 matrices per 2^16-column key
and multiplies them (exact: counts < 2^24).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SW = 1 << 20


def _row_cols(arena, s, d):
    """int64 columns (within the shard) of dense row d in shard s, decoded
    straight from the arena's container metadata and payload."""
    rows, rowptr, shard_base, meta, payload = arena[:5]
    D = len(rows)
    rp = rowptr.reshape(-1, D + 1)[s]
    out = []
    for c in range(int(rp[d]), int(rp[d + 1])):
        m = int(meta[int(shard_base[s]) + c])
        j, typ, n, off = m & 15, (m >> 4) & 3, (m >> 6) & 0x1FFFF, (m >> 23) * 8
        if typ == 1:
            v = payload[off:off + n].astype(np.int64)
        elif typ == 2:
            bits = np.unpackbits(payload[off:off + 4096].view(np.uint8), bitorder="little")
            v = np.flatnonzero(bits).astype(np.int64)
        else:
            nr = int(payload[off])
            rr = payload[off + 8:off + 8 + 2 * nr].astype(np.int64).reshape(-1, 2)
            v = np.concatenate([np.arange(a0, a1 + 1) for a0, a1 in rr]) if nr else np.zeros(0, np.int64)
        out.append(v + (j << 16))
    return np.concatenate(out) if out else np.zeros(0, np.int64)


def _reference(arena, cache, R, src_rows):
    """int64[S, Q, R]: |row(cache rank k) & src_q| per shard (rows are their
    own dense index in a generated arena)."""
    import torch

    S = len(arena[2]) - 1
    dev = torch.device("cuda", 0)
    out = np.zeros((S, len(src_rows), R), np.int64)
    for s in range(S):
        hot_rows = cache.rows[s, :R]
        live = cache.counts[s, :R] > 0
        hr, hc = [], []
        for k in range(R):
            if live[k]:
                c = _row_cols(arena, s, int(hot_rows[k]))
                hr.append(np.full(len(c), k, np.int64))
                hc.append(c)
        hr = torch.from_numpy(np.concatenate(hr)).to(dev)
        hc = torch.from_numpy(np.concatenate(hc)).to(dev)
        sr, sc = [], []
        for q, r in enumerate(src_rows):
            c = _row_cols(arena, s, int(r))
            sr.append(np.full(len(c), q, np.int64))
            sc.append(c)
        sr = torch.from_numpy(np.concatenate(sr)).to(dev)
        sc = torch.from_numpy(np.concatenate(sc)).to(dev)
        acc = torch.zeros((R, len(src_rows)), dtype=torch.float32, device=dev)
        for j in range(SW >> 16):
            hm = (hc >> 16) == j
            sm = (sc >> 16) == j
            H = torch.zeros((R, 1 << 16), dtype=torch.float32, device=dev)
            H[hr[hm], hc[hm] & 0xFFFF] = 1.0
            Sd = torch.zeros((len(src_rows), 1 << 16), dtype=torch.float32, device=dev)
            Sd[sr[sm], sc[sm] & 0xFFFF] = 1.0
            acc += H @ Sd.T
        out[s] = acc.T.round().to(torch.int64).cpu().numpy()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("nq", [16, 32])
def test_hot_counts_equal_dense_reference(nq, monkeypatch):
    import torch

    torch.backends.cuda.matmul.allow_tf32 = False
    from pilosa_amd import _roaring
    from pilosa_amd.ops import topn_index
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf
    from pilosa_amd.ops.topn import DeviceRankCache
    from pilosa_amd.ops.topn_index import DeviceTopNIndex

    monkeypatch.setattr(topn_index, "HOT_Q", 32)
    dev = torch.device("cuda", 0)
    S, nrows = 2, 6000
    arena = _roaring.gen_zipf_arena(0, S, S * SW, nrows, 8.0, 1.6, 50.0, 7, 4)
    view = DeviceView(*arena, dev, shards=list(range(S)))
    cache = DeviceRankCache.from_view(view, k=5000)
    idx = DeviceTopNIndex(view, cache)
    assert idx.R >= 1024, idx.R
    # the mix: the containers at the top ranks are bitmaps, then arrays of
    # every size down to a few values
    n = (arena[3] >> 6) & 0x1FFFF
    assert (n > 4096).any()
    assert ((n > 1024) & (n <= 4096)).any() and ((n > 0) & (n <= 64)).any()
    rng = np.random.default_rng(5)
    src_rows = [0, 3, 17, 64, 200, 999, 2500, 5999][:nq] + [int(r) for r in rng.integers(0, nrows, nq)]
    src_rows = src_rows[:nq]
    eng = GpuEngine(dev)
    src = eng.materialize_batch([Leaf(view, r) for r in src_rows], idx.S)
    got = idx.hot_counts(src, nq).view(idx.S, nq, idx.R).cpu().numpy().astype(np.int64)
    want = _reference(arena, cache, idx.R, src_rows)
    bad = np.argwhere(got != want)
    assert bad.size == 0, (len(bad), bad[:5].tolist(), [(got[tuple(b)], want[tuple(b)]) for b in bad[:5]])


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("env", [{"PILOSA_TOPN_SMALL_N": "63"}, {"PILOSA_TOPN_SMALL_N": "1023"},
                                 {"PILOSA_TOPN_SMALL_N": "4096"},
                                 {"PILOSA_TOPN_MID_N": "0"}, {"PILOSA_TOPN_MID_N": "512"},
                                 {"PILOSA_TOPN_MID_N": "2048"}, {"PILOSA_TOPN_TBUILD_MIN": "65537"}],
                         ids=["small63", "small1023", "small4096", "nomid", "mid512", "mid2048", "atomicbuild"])
def test_hot_counts_equal_dense_reference_at_every_bound(env):
    """The same check with other lane-owned and mid-size bounds and the
    atomic table build: each setting is fixed per process."""
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
                        "--timeout", "300", "--timeout-method", "thread",
                        "tests/test_gpu_hot_counts.py::test_hot_counts_equal_dense_reference"],
                       cwd=ROOT, env=dict(os.environ, **env), capture_output=True, text=True, timeout=580)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout.splitlines()[-1], r.stdout[-1000:]
