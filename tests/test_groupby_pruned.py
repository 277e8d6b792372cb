"""GroupBy with cumulative-intersection pruning (GpuExecutor._pruned_groups,
reference executor.go:3060-3230 groupByIterator) checked on the CPU: the
device count launches are replaced by a host evaluation of the same Leaf/Op
expressions, so the walk order, pruning, paging (previous=) and limit logic
must reproduce the host executor's GroupBy exactly."""
import numpy as np
import pytest

from tests.helpers import SW, Env


class _HostEngine:
    """engine.count() stand-in: evaluates Leaf/Op trees on host fragments."""

    def __init__(self, env, names):
        self.env, self.names = env, names
        self.calls = 0
        self.exprs = 0

    def prepare_progs(self, progs, views, S):
        from pilosa_amd.ops.device import Leaf, Op, OP_AND
        exprs = []
        for p in progs:
            lv = [Leaf(views[int(p["leaf_view"][i])], int(views[int(p["leaf_view"][i])].rows[int(p["leaf_row"][i])])
                       if int(p["leaf_row"][i]) >= 0 else -1) for i in range(int(p["nleaf"]))]
            assert list(p["prog"][:int(p["nprog"])]) == [0] + [v for i in range(1, len(lv)) for v in (i, OP_AND)]
            exprs.append(lv[0] if len(lv) == 1 else Op("and", tuple(lv)))
        return exprs

    def launch_count(self, exprs):
        import torch
        return torch.from_numpy(self.count(exprs))

    def count(self, exprs):
        from pilosa_amd.ops.device import Leaf, Op
        self.calls += 1
        self.exprs += len(exprs)
        idx = self.env.holder.index("i")

        def ev(e):
            if isinstance(e, Leaf):
                if e.row < 0:
                    from pilosa_amd.models.row import Row
                    return Row()
                return idx.field(self.names[id(e.view)]).row(e.row)
            rows = [ev(a) for a in e.args]
            r = rows[0]
            for x in rows[1:]:
                r = r.intersect(x)
            return r
        return np.array([ev(e).count() for e in exprs], np.int64)


@pytest.fixture(scope="module")
def env():
    e = Env()
    e.create_index("i")
    for f in ("a", "b", "c"):
        e.field("i", f)
    rng = np.random.default_rng(9)
    idx = e.holder.index("i")
    for f, nrows, dens in (("a", 7, 0.02), ("b", 5, 0.3), ("c", 9, 0.01)):
        for r in range(nrows):
            k = int(dens * 2 * SW * (0.3 + rng.random()))
            cols = rng.choice(2 * SW, size=k, replace=False).astype(np.uint64)
            idx.field(f).import_bits(np.full(k, r, np.uint64), cols)
    # a row of c that intersects nothing in a (pruned at level 2)
    idx.field("c").import_bits(np.full(3, 40, np.uint64), np.array([2 * SW - 1, 2 * SW - 2, 2 * SW - 3], np.uint64))
    yield e
    e.close()


QUERIES = [
    "GroupBy(Rows(a), Rows(b), Rows(c))",
    "GroupBy(Rows(a), Rows(b), Rows(c), limit=17)",
    "GroupBy(Rows(a), Rows(b), Rows(c), previous=[2, 3, 4], limit=9)",
    "GroupBy(Rows(c), Rows(a))",
    "GroupBy(Rows(a), Rows(c), Rows(b), filter=Row(b=1), limit=30)",
    "GroupBy(Rows(b))",
    "GroupBy(Rows(a), Rows(b), previous=[6, 4])",
    "GroupBy(Rows(a, previous=1), Rows(b), Rows(c), limit=5)",
]


@pytest.mark.parametrize("q", QUERIES)
def test_pruned_groupby_matches_host(env, q):
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    want = env.q1("i", q)
    g = GpuExecutor(env.holder, "cpu", executor=env.executor)
    shards = env.holder.index("i").available_shards()
    names = {id(g.view_arena("i", f, "standard", shards)): f for f in ("a", "b", "c")}
    g.engine = _HostEngine(env, names)
    g._matrix_fits = lambda ra, rb: False  # force the pruned walk for two fields too
    env.executor.gpu = g
    try:
        got = env.q1("i", q)
    finally:
        env.executor.gpu = None
    assert [(tuple(x.row_id for x in gc.group), gc.count) for gc in got] == \
        [(tuple(x.row_id for x in gc.group), gc.count) for gc in want]
    assert g.engine.calls > 0


def test_pruning_skips_empty_prefixes(env):
    """The row of c that meets nothing in a is never extended to b."""
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    g = GpuExecutor(env.holder, "cpu", executor=env.executor)
    shards = env.holder.index("i").available_shards()
    arenas = [g.view_arena("i", f, "standard", shards) for f in ("c", "a", "b")]
    names = {id(v): f for v, f in zip(arenas, ("c", "a", "b"))}
    eng = g.engine = _HostEngine(env, names)
    cand = [[int(r) for r in v.rows] for v in arenas]
    full = len(cand[0]) * len(cand[1]) * len(cand[2])
    out = g._pruned_groups(arenas, cand, None, None, 10 ** 9)
    assert all(k[0] != 40 for k, _ in out)
    assert eng.exprs < len(cand[0]) + len(cand[0]) * len(cand[1]) + full
