"""The collective chain of one OP_TOPN mesh batch (parallel/mesh.py), on gloo.

VERDICT r4 weak 2: a TopN batch used to pay a stale-space vote, a readiness
vote, a size all-gather whose result the host had to read, a data all-gather
and the re-count all-reduce.  The mesh now folds both votes into one
all-reduce and the candidate union is one speculative fixed-capacity
all-gather, so a steady-state batch costs at most 3 data-group collectives
(commands travel on the separate gloo control group).  The device work is
stubbed here (a CPU box has no HIP kernels): the stub makes exactly the
collective calls the device path makes (ops/topn_exec.py ``topn_nosrc`` with
``comm``: ``comm.union`` then ``comm.all_reduce_async`` of the re-counts)."""
import json
import os
import tempfile

import numpy as np
import torch.multiprocessing as mp

from tests.test_mesh import _free_port


class _StubGpu:
    """The GpuExecutor surface OP_TOPN uses.  Rank r's candidates of call q
    are rows {q, 10 + r, 100 + q * r} plus ``extra`` more rows (to overflow
    the union's pad); every rank counts 1 per candidate, so a row's total is
    the world size."""

    def __init__(self, rank, extra=0):
        self.rank = rank
        self.comm = None
        self.extra = extra
        self.stale = True
        self.refreshes = 0
        self.decline = False

    def node_space_stale(self, index, fname, shards):
        return self.stale

    def refresh_node_spaces(self, index, fnames, shards, comm):
        import torch
        for _ in fnames:
            comm.all_gather_var(torch.zeros(1, dtype=torch.int64))
        self.stale = False
        self.refreshes += 1

    def topn_batch_ready(self, index, calls, shards):
        return not self.decline

    def topn_batch(self, index, calls, shards, defer=False):
        import torch

        from pilosa_amd.models.cache import Pair
        from pilosa_amd.parallel.collectives import Pending
        comm = self.comm
        Q = len(calls)
        A = 1 << 20
        keys = []
        for q in range(Q):
            rows = {q, 10 + self.rank, 100 + q * self.rank} | {1000 + k for k in range(self.extra)}
            keys += [q * A + r for r in sorted(rows)]
        # src calls: the slot-index path's union tag (its vote rides in it)
        tag = "topn_src" if all(c.children for c in calls) else "stub"
        u = comm.union(torch.tensor(keys, dtype=torch.int64), tag=tag)
        out = torch.ones(u.numel(), dtype=torch.int64)

        def finish():
            res = [[] for _ in range(Q)]
            for k, c in zip(u.tolist(), out.tolist()):
                res[k // A].append(Pair(k % A, c))
            return res
        return Pending(comm, comm.all_reduce_async(out), finish, keep=out)


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = Holder(tempfile.mkdtemp(prefix=f"chain{rank}_")).open()
    holder.create_index("i").create_field("f")
    ex = Executor(holder)
    stub = _StubGpu(rank)
    mesh = ShardMesh(ex, block=1)
    ex.mesh = mesh
    ex.gpu = stub
    state = [0]

    def toggle():   # OP_RECALC: rank 1 first declines, then finds its space stale
        state[0] += 1
        if rank == 1:
            stub.decline = state[0] == 1
            stub.stale = state[0] == 2
    holder.recalculate_caches = toggle
    try:
        if rank != 0:
            mesh.serve()
            with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
                json.dump({"refreshes": stub.refreshes}, fh)
            return
        q = "TopN(f, n=5) TopN(f, n=3)"
        first = ex.execute("i", q, shards=[0, 1]).results
        per_batch = []
        for _ in range(5):
            c0 = mesh.comm.data_calls
            got = ex.execute("i", q, shards=[0, 1]).results
            per_batch.append(mesh.comm.data_calls - c0)
        # a batch whose candidates overflow the union's pad: re-gathered once
        # at the exact size, and the capacity then fits the next such batch
        stub.extra = 3000
        r0 = mesh.comm.union_retries
        big1 = ex.execute("i", q, shards=[0, 1]).results
        r1 = mesh.comm.union_retries
        big2 = ex.execute("i", q, shards=[0, 1]).results
        r2 = mesh.comm.union_retries
        # src batches: the readiness vote rides in the candidate union, so a
        # steady-state batch is the union + the re-count all-reduce
        qs = "TopN(f, Row(f=1), n=5) TopN(f, Row(f=2), n=3)"
        stub.extra = 0
        ex.execute("i", qs, shards=[0, 1])
        src_batch = []
        for _ in range(3):
            c0 = mesh.comm.data_calls
            src_got = ex.execute("i", qs, shards=[0, 1]).results
            src_batch.append(mesh.comm.data_calls - c0)
        from pilosa_amd.pql import parse_string
        calls = parse_string(qs).calls
        # rank 1 cannot take part (its vote rides in the union): the node
        # abandons the batch after that one collective, the general path answers
        mesh.recalculate_caches()     # (rank 1: decline from now on)
        c0 = mesh.comm.data_calls
        declined = mesh.topn_batch("i", calls, [0, 1])
        declined_calls = mesh.comm.data_calls - c0
        # rank 1's node row space goes stale: its vote makes the node rebuild
        # the spaces (OP_TOPN_SPACES) and re-run the batch once
        mesh.recalculate_caches()     # (rank 1: ready again, space stale)
        ref0 = stub.refreshes
        stale_got = mesh.topn_batch("i", calls, [0, 1])
        stale_refreshes = stub.refreshes - ref0
        mesh.stop()
        canon = lambda rs: [[(p.id, p.count) for p in r] for r in rs]   # noqa: E731
        with open(os.path.join(outdir, "rank0.json"), "w") as fh:
            json.dump({"first": canon(first), "got": canon(got), "per_batch": per_batch,
                       "big_len": [len(r) for r in big1], "big_same": canon(big1) == canon(big2),
                       "retries": [r1 - r0, r2 - r1], "refreshes": stub.refreshes,
                       "src_batch": src_batch, "src_got": canon(src_got), "declined": declined is None,
                       "declined_calls": declined_calls, "stale_got": canon(stale_got or []),
                       "stale_refreshes": stale_refreshes,
                       "batches": mesh.topn_tensor_batches}, fh)
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()


def test_topn_batch_collective_chain(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "rank0.json"))
    r1 = json.load(open(tmp_path / "rank1.json"))
    # union over the ranks, each row counted once per rank
    want = []
    for q in range(2):
        rows = sorted({q, 10, 100} | {q, 11, 100 + q})
        want.append([[r, world] for r in rows])
    assert res["first"] == want and res["got"] == want
    # steady state: the folded vote, one union all-gather, one re-count all-reduce
    assert res["per_batch"] == [3] * 5, res["per_batch"]
    # the spaces were refreshed on both ranks: on the first (stale) batch,
    # and once more after rank 1's stale vote below
    assert res["refreshes"] == 2 and r1["refreshes"] == 2
    assert res["big_len"] == [3000 + len(w) for w in want]
    assert res["big_same"]
    assert res["retries"] == [1, 0], res["retries"]
    assert res["batches"] == 8 + 4 + 1
    # src: union (with the vote) + re-count all-reduce
    assert res["src_batch"] == [2, 2, 2], res["src_batch"]
    assert res["src_got"] == want
    assert res["declined"] and res["declined_calls"] == 1
    assert res["stale_got"] == want and res["stale_refreshes"] == 1
