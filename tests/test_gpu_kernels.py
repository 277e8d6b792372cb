"""Numerics of the gfx950 kernels against the host roaring oracle (C++ CPU)."""
import numpy as np
import pytest

from pilosa_amd import _roaring as R

pytestmark = pytest.mark.gpu


def _random_fragment(rng, nrows=12, shard=0):
    """Rows with every container flavour: sparse arrays, dense bitmaps, runs."""
    vals = []
    base = shard * (1 << 20)
    for r in range(nrows):
        kind = r % 4
        if kind == 0:   # sparse array
            cols = rng.choice(1 << 20, size=rng.integers(1, 3000), replace=False)
        elif kind == 1:  # dense -> bitmap containers
            cols = rng.choice(1 << 20, size=rng.integers(200000, 600000), replace=False)
        elif kind == 2:  # runs
            starts = rng.choice((1 << 20) - 5000, size=20, replace=False)
            cols = np.unique(np.concatenate([np.arange(s, s + rng.integers(1, 5000)) for s in starts]))
        else:           # partial: only a few containers
            cols = rng.choice(70000, size=1000, replace=False) + rng.integers(0, 15) * 65536
        vals.append(np.uint64(r) * np.uint64(1 << 20) + (cols.astype(np.uint64) % np.uint64(1 << 20)))
    b = R.Bitmap(np.concatenate(vals))
    b.optimize()  # creates run containers
    return b


@pytest.fixture(scope="module")
def setup():
    import torch
    from pilosa_amd.ops.device import DeviceView, GpuEngine
    rng = np.random.default_rng(7)
    S = 3
    frags = [_random_fragment(rng, shard=s) for s in range(S)]
    frags.insert(1, None)  # an empty shard
    dev = torch.device("cuda:0")
    view = DeviceView.from_bitmaps(frags, dev, shards=[0, 1, 2, 3])
    return frags, view, GpuEngine(dev)


def _row(frag, r):
    if frag is None:
        return R.Bitmap()
    return frag.offset_range(0, r * (1 << 20), (r + 1) * (1 << 20))


def test_container_mix(setup):
    frags, view, eng = setup
    kinds = set()
    for f in frags:
        if f is not None:
            kinds |= {t for _, t, _ in f.container_info()}
    assert kinds == {"array", "bitmap", "run"}


def test_count_and_intersect_all_pairs(setup):
    from pilosa_amd.ops.device import Leaf, Op
    frags, view, eng = setup
    exprs, want = [], []
    for a in range(12):
        for b in range(12):
            exprs.append(Op("and", (Leaf(view, a), Leaf(view, b))))
            want.append(sum(_row(f, a).intersection_count(_row(f, b)) for f in frags))
        exprs.append(Leaf(view, a))
        want.append(sum(_row(f, a).count() for f in frags))
    got = eng.count(exprs)
    np.testing.assert_array_equal(got, np.array(want))


def test_generic_programs(setup):
    from pilosa_amd.ops.device import Leaf, Op
    frags, view, eng = setup
    L = lambda r: Leaf(view, r)  # noqa: E731
    cases = [
        (Op("or", (L(0), L(1), L(2))), lambda a, b, c, d: a.union(b).union(c)),
        (Op("xor", (L(1), L(2))), lambda a, b, c, d: b.xor(c)),
        (Op("andnot", (L(1), L(2))), lambda a, b, c, d: b.difference(c)),
        (Op("and", (Op("or", (L(0), L(1))), Op("or", (L(2), L(3))))),
         lambda a, b, c, d: a.union(b).intersect(c.union(d))),
        (Op("andnot", (Op("or", (L(1), L(3))), Op("and", (L(0), L(2))))),
         lambda a, b, c, d: b.union(d).difference(a.intersect(c))),
        (Op("and", (L(1), L(99))), lambda a, b, c, d: R.Bitmap()),  # missing row
    ]
    got = eng.count([c[0] for c in cases])
    for (expr, fn), g in zip(cases, got):
        want = 0
        for f in frags:
            rows = [_row(f, r) for r in range(4)]
            want += fn(*rows).count()
        assert g == want, expr


def test_materialize_matches_oracle(setup):
    from pilosa_amd.ops.device import Leaf, Op
    frags, view, eng = setup
    expr = Op("or", (Op("and", (Leaf(view, 1), Leaf(view, 5))), Leaf(view, 2), Leaf(view, 0)))
    bms, shards = eng.materialize(expr)
    for f, s, got in zip(frags, shards, bms):
        if f is None:
            assert got is None
            continue
        want = _row(f, 1).intersect(_row(f, 5)).union(_row(f, 2)).union(_row(f, 0))
        # device returns row-0-relative keys in shard s: compare column sets
        want_cols = want.slice() % (1 << 20)
        got_cols = got.slice() % (1 << 20) if got is not None else np.array([], np.uint64)
        np.testing.assert_array_equal(np.sort(got_cols), np.sort(want_cols))


def test_and2_pair_kernels_match_tile_kernel(setup):
    """Key-major pair kernels (pair_kernels.hip) == per-(query, shard) fast
    kernel on a shuffled batch with repeated/swapped rows, two views, empty
    rows and per-shard output; CQ variants included."""
    import torch
    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf, Op
    frags, view, eng = setup
    rng = np.random.default_rng(11)
    other = [_random_fragment(rng, nrows=6, shard=s) for s in range(4)]
    view2 = DeviceView.from_bitmaps(other, view.device, shards=[0, 1, 2, 3])
    exprs, want = [], []
    for _ in range(700):
        a, b = int(rng.integers(0, 14)), int(rng.integers(0, 14))  # 12,13 -> empty rows
        va, fa = (view2, other) if rng.random() < 0.3 else (view, frags)
        exprs.append(Op("and", (Leaf(va, min(a, 5) if va is view2 else a), Leaf(view, b))))
        ra = min(a, 5) if va is view2 else a
        want.append(sum(_row(x, ra).intersection_count(_row(f, b)) for x, f in zip(fa, frags)))
    # the shipped variants (v6, the serving variant 39); the rejected ones
    # live in the kbench module only (native/build.py --kbench)
    for var in (6, 39):
        for cq in (0, 16, 32, 64):
            e2 = GpuEngine(view.device)
            e2.and2_cq = cq
            e2.and2_variant = var
            np.testing.assert_array_equal(e2.count(exprs), np.array(want), err_msg=f"variant {var} cq {cq}")
    old = GpuEngine(view.device)
    old.use_and2 = False
    np.testing.assert_array_equal(old.count(exprs), np.array(want))
    ps_new = eng.count_per_shard(exprs[:64])
    ps_old = old.count_per_shard(exprs[:64])
    np.testing.assert_array_equal(ps_new, ps_old)
    assert ps_new.shape == (64, 4)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_bitgemm_count_matrix_matches_host(mode):
    """Row-pair count matrix on the matrix cores (mode 1, i8 MFMA) and VALU
    (mode 0) == host roaring intersection counts, all container types, tile
    edges (row counts not multiples of 64)."""
    import numpy as np
    import torch

    from pilosa_amd import _roaring as R
    from pilosa_amd.ops.device import DeviceView
    from pilosa_amd.ops.groupby import pair_count_matrix

    rng = np.random.default_rng(5)
    SW = 1 << 20
    frags = []
    for s in range(3):
        vals = []
        for r in range(70):
            kind = r % 4
            if kind == 0:      # dense -> bitmap containers
                c = rng.choice(SW, 300000, replace=False)
            elif kind == 1:    # sparse -> arrays
                c = rng.choice(SW, 3000, replace=False)
            elif kind == 2:    # runs
                st = int(rng.integers(0, SW - 70000))
                c = np.arange(st, st + 60000 + r)
            else:
                c = rng.choice(SW, 40, replace=False)
            vals.append(np.uint64(r) * np.uint64(SW) + c.astype(np.uint64))
        bm = R.Bitmap(np.concatenate(vals))
        bm.optimize()
        frags.append(bm)
    view = DeviceView.from_bitmaps(frags, torch.device("cuda:0"))
    ra, rb = list(range(0, 70, 2)) + [999], list(range(70))
    got = pair_count_matrix(view, ra, view, rb, mode=mode)
    want = np.zeros((len(ra), len(rb)), np.int64)
    for s, bm in enumerate(frags):
        rows = {r: bm.offset_range(0, r * SW, (r + 1) * SW) for r in range(70)}
        for i, a in enumerate(ra):
            if a not in rows:
                continue
            for k, b in enumerate(rb):
                want[i, k] += rows[a].intersection_count(rows[b])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("variant", [6, 39])
@pytest.mark.parametrize("cq", [4, 8, 16, 32, 64])
def test_pair_kernel_array_size_boundaries(cq, variant):
    """Array containers of 1, 63, 64, 65, 255, 256, 257 (the small-probe
    boundary), 511, 512, 513 and 4096 values against bitmap, array and run
    rows, each paired once (one-off: the gather / LDS-staged-bitmap branches)
    and many times in a row (the staged, reused-row branch), including value 0
    (the pad-correction path) -> host intersection_count, for the shipped
    variants (v6 and the serving variant 39, every queries-per-wave size)."""
    import torch

    from pilosa_amd.ops.device import DeviceView, GpuEngine, Leaf, Op
    rng = np.random.default_rng(cq)
    sizes = [1, 63, 64, 65, 255, 256, 257, 511, 512, 513, 4096]
    rows = []
    for k, n in enumerate(sizes):  # array rows 0..10: key 0 (with value 0 when k is even) and key 3
        c0 = np.sort(rng.choice(65536, n, replace=False))
        if k % 2 == 0:
            c0[0] = 0
        c3 = 3 * 65536 + np.sort(rng.choice(65536, n, replace=False))
        rows.append(np.concatenate([c0, c3]))
    dense = np.concatenate([rng.choice(65536, 30000, replace=False), 3 * 65536 + rng.choice(65536, 9000, replace=False)])
    rows.append(np.concatenate([[0], dense]))                                   # 11: bitmaps, holds value 0
    rows.append(np.concatenate([np.arange(0, 40000), 3 * 65536 + np.arange(100, 30000)]))  # 12: runs
    rows.append(rng.choice(65536, 5000, replace=False) + 65536 * 3)            # 13: one bitmap container
    vals = np.concatenate([np.uint64(r) * np.uint64(1 << 20) + np.unique(c).astype(np.uint64) for r, c in enumerate(rows)])
    frag = R.Bitmap(vals)
    frag.optimize()
    dev = torch.device("cuda:0")
    view = DeviceView.from_bitmaps([frag], dev)
    eng = GpuEngine(dev)
    eng.and2_cq = cq
    eng.and2_variant = variant
    pairs = []
    for a in range(len(rows)):
        for b in range(len(rows)):
            pairs.append((a, b))              # one-off pairs
    for a in (11, 12, 3, 10):
        pairs += [(a, b) for b in range(len(rows))] * 3  # runs of the same staged row
    exprs = [Op("and", (Leaf(view, a), Leaf(view, b))) for a, b in pairs]
    want = [_row(frag, a).intersection_count(_row(frag, b)) for a, b in pairs]
    got = eng.count(exprs)
    np.testing.assert_array_equal(got, np.array(want))
    per = eng.count_per_shard(exprs)
    np.testing.assert_array_equal(per[:, 0], np.array(want))


@pytest.mark.parametrize("variant", [1, 2])
def test_union_count_kernels(setup, variant):
    """Count(Union(...)) of 2..16 leaves on union_count_kernel (1) and
    union_count2_kernel (2): every container mix, repeated leaves, missing
    rows, keys held by one leaf only (the metadata shortcut)."""
    from pilosa_amd.ops.device import Leaf, Op
    frags, view, eng = setup
    old = eng.union_variant
    eng.union_variant = variant
    try:
        rng = np.random.default_rng(11)
        sets = [[0, 1], [2, 3], [0, 2, 3], [1, 1, 2], [3, 7, 11, 99], list(range(12)),
                [5, 9, 2, 6, 10, 3, 7, 11, 0, 4, 8, 1, 2, 3, 99, 98]]
        sets += [list(rng.integers(0, 14, size=rng.integers(2, 17))) for _ in range(24)]
        exprs = [Op("or", tuple(Leaf(view, int(r)) for r in rs)) for rs in sets]
        got = eng.count(exprs)
        for rs, g in zip(sets, got):
            want = 0
            for f in frags:
                u = R.Bitmap()
                for r in rs:
                    u = u.union(_row(f, int(r)))
                want += u.count()
            assert g == want, (variant, rs)
    finally:
        eng.union_variant = old


def _rand_expr(rng, view, depth):
    """Random boolean tree over rows 0..13 (12, 13 are missing rows)."""
    from pilosa_amd.ops.device import Leaf, Op
    if depth == 0 or rng.random() < 0.3:
        r = int(rng.integers(0, 14))
        return Leaf(view, r), ("row", r)
    op = ["and", "or", "xor", "andnot"][int(rng.integers(0, 4))]
    k = int(rng.integers(2, 4))
    kids = [_rand_expr(rng, view, depth - 1) for _ in range(k)]
    return Op(op, tuple(e for e, _ in kids)), (op, [t for _, t in kids])


def _host_eval(tree, frag):
    if tree[0] == "row":
        return _row(frag, tree[1])
    vals = [_host_eval(t, frag) for t in tree[1]]
    out = vals[0]
    for v in vals[1:]:
        out = {"and": out.intersect, "or": out.union, "xor": out.xor, "andnot": out.difference}[tree[0]](v)
    return out


def test_differential_fuzz_count_and_materialize(setup):
    """SURVEY §5.2 differential fuzzing: random expression trees through every
    count route the planner picks (pair kernel, union kernel, flat fold,
    generic interpreter) and through materialize, against the host roaring
    oracle."""
    from pilosa_amd.ops.device import CompileError
    frags, view, eng = setup
    rng = np.random.default_rng(2024)
    exprs, trees = [], []
    while len(exprs) < 160:
        e, t = _rand_expr(rng, view, 3)
        try:
            from pilosa_amd.ops.device import compile_expr
            compile_expr(e, {})
        except CompileError:
            continue
        exprs.append(e)
        trees.append(t)
    got = eng.count(exprs)
    for e, t, g in zip(exprs, trees, got):
        want = sum(_host_eval(t, f).count() for f in frags if f is not None)
        assert g == want, t
    for e, t in list(zip(exprs, trees))[:24]:
        bms, shards = eng.materialize(e)
        for f, b in zip(frags, bms):
            if f is None:
                continue
            want_cols = _host_eval(t, f).slice() % (1 << 20)
            got_cols = b.slice() % (1 << 20) if b is not None else np.array([], np.uint64)
            np.testing.assert_array_equal(np.sort(got_cols), np.sort(want_cols), err_msg=str(t))


@pytest.mark.parametrize("which", ["min", "max"])
@pytest.mark.parametrize("F,sub", [(1, 1), (37, 1), (65, 1), (2500, 1), (9, 4)])
def test_bsi_minmax_fold_kernel_matches_host_fold(which, F, sub):
    """bsi_minmax_fold_kernel == the host fold it replaced (per-shard sign
    rules, sub-shard fold, first fragment holding the extreme) on random
    descent tables with ties, empty keys and all-negative fragments."""
    import torch

    from pilosa_amd.ops.device import kernels
    from pilosa_amd.ops.gpu_executor import _fold_subshards_value, _minmax_per_shard
    rng = np.random.default_rng(F * 7 + sub + (which == "min"))
    S = F * sub
    o = np.zeros((S, 16, 10), np.int64)
    o[:, :, 8] = rng.random((S, 16)) < 0.5          # any positive in the key
    o[:, :, 9] = rng.random((S, 16)) < 0.3          # any negative
    for c in (0, 2, 4, 6):
        o[:, :, c] = rng.integers(0, 6, (S, 16))    # few values: many ties
        o[:, :, c + 1] = rng.integers(1, 50, (S, 16))
    dead = rng.random(S) < 0.2                      # whole shards without values
    o[dead, :, 8:] = 0
    vals, cnts = _minmax_per_shard(o, which)
    vals, cnts = np.asarray(vals, np.int64), np.asarray(cnts, np.int64)
    if sub > 1:
        vals, cnts = _fold_subshards_value(vals, cnts, which == "min", M=sub)
    live = cnts > 0
    if live.any():
        best = vals[live].min() if which == "min" else vals[live].max()
        k = int(np.flatnonzero(live & (vals == best))[0])
        want = [int(vals[k]), int(cnts[k]), 1]
    else:
        want = [0, 0, 0]
    dev = torch.device("cuda", 0)
    out = torch.full((3,), -7, dtype=torch.int64, device=dev)
    kernels().bsi_minmax_fold(torch.from_numpy(o.reshape(-1)).to(dev), F, 16 * sub, int(which == "min"), out)
    assert out.cpu().tolist() == want


@pytest.mark.parametrize("U,n", [(1, 1), (15264, 36), (300, 130), (1000, 4096)])
def test_partial_sum_scatter_matches_torch(U, n):
    """partial_sum_scatter (pair-kernel partial column sums scattered into
    the batch result) == torch sum + index_copy; out-of-range targets are
    dropped."""
    import torch

    from pilosa_amd.ops.device import kernels
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(U + n)
    part = torch.randint(0, 1 << 20, (U, n), generator=g, dtype=torch.int32)
    ti = torch.randperm(n + 3, generator=g)[:n].to(torch.int64)
    want = torch.zeros(n + 3, dtype=torch.int64)
    want.index_copy_(0, ti, part.to(torch.int64).sum(dim=0))
    keep = ti < n + 3
    out = torch.zeros(n + 3, dtype=torch.int64, device=dev)
    kernels().partial_sum_scatter(part.to(dev).view(-1), U, n, ti.to(dev), out)
    assert torch.equal(out.cpu(), want) and bool(keep.all())
    # a target outside out is dropped, not written
    bad = ti.clone()
    bad[0] = n + 100
    out2 = torch.zeros(n + 3, dtype=torch.int64, device=dev)
    kernels().partial_sum_scatter(part.to(dev).view(-1), U, n, bad.to(dev), out2)
    want2 = want.clone()
    want2[ti[0]] = 0
    assert torch.equal(out2.cpu(), want2)


def test_dense_shadows_match_arena_containers():
    """shadow_build_kernel: every shadowed (row, shard, key) is the row's
    container of that key as a bitmap (zeros where the row has none); rows are
    the hottest by bit count; a write leaves the shadow stale (not passed).
    Dense shadows measured slower and ship in the kbench module only
    (PILOSA_HIPKERNELS=_hipkernels_kbench runs this test)."""
    import torch

    from pilosa_amd.ops.device import kernels
    if not hasattr(kernels(), "shadow_build"):
        pytest.skip("dense shadows are built into the kbench module only")

    from pilosa_amd.ops.device import DeviceView
    rng = np.random.default_rng(5)
    frags = []
    for s in range(3):
        rows = rng.zipf(1.5, 60000) % 40
        cols = rng.integers(0, 1 << 20, 60000)
        frags.append(R.Bitmap((rows.astype(np.uint64) << np.uint64(20)) + cols.astype(np.uint64)))
        frags[-1].optimize()
    dev = torch.device("cuda:0")
    view = DeviceView.from_bitmaps(frags, dev)
    assert view.ensure_shadow()
    gen, buf, slot, _, rows = view._shadow
    sh = buf.view(len(rows), view.S, 16, 1024).cpu().numpy()
    counts = [sum(int(f.count_range(int(d_row) << 20, (int(d_row) + 1) << 20)) for f in frags) for d_row in view.rows]
    assert set(rows.tolist()) <= set(range(view.D)) and len(rows) >= 8
    # every shard sampled here (S <= SHADOW_SAMPLE_SHARDS): exactly the hottest rows (up to ties)
    assert sum(counts[d] for d in rows.tolist()) == sum(sorted(counts, reverse=True)[:len(rows)])
    for r, d in enumerate(rows.tolist()):
        rid = int(view.rows[d])
        for s in range(view.S):
            for j in range(16):
                lo = (rid << 20) + (j << 16)
                want = np.zeros(65536, bool)
                got_cols = frags[s].slice_range(lo, lo + 65536) if hasattr(frags[s], "slice_range") else \
                    np.asarray([c for c in frags[s].slice() if lo <= c < lo + 65536], np.uint64)
                want[(np.asarray(got_cols, np.int64) - lo)] = True
                bits = np.unpackbits(sh[r, s, j].view(np.uint8), bitorder="little").astype(bool)
                assert np.array_equal(bits, want), (r, s, j)
    assert slot.cpu().numpy()[rows].tolist() == list(range(len(rows)))
    view.generation += 1                       # a write: the shadow is not passed until rebuilt
    assert not view.shadow_fresh() and int(view.viewdev()["shadow"]) == 0
