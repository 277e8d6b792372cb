"""Multi-rank shard mesh (pilosa_amd/parallel/mesh.py) over gloo on the CPU.

Every rank owns a block-cyclic subset of shards in its own holder; rank 0 is
the front end.  Results of a query workload must equal a single-process
executor holding all shards (the reference's multi-node tests assert the same
for HTTP fan-out: executor_test.go TestExecutor_Execute_Remote*)."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

SW = 1 << 20

QUERIES = [
    "Count(Row(f=1))",
    "Count(Intersect(Row(f=1), Row(f=2)))",
    "Count(Union(Row(f=1), Row(g=3)))",
    "Row(f=2)",
    "Difference(Row(f=1), Row(f=2))",
    "Not(Row(f=3))",
    "TopN(f, n=3)",
    "TopN(f, Row(g=3), n=2)",
    "Sum(field=v)",
    "Sum(Row(f=1), field=v)",
    "Min(field=v)",
    "Max(Row(f=2), field=v)",
    "MinRow(field=f)",
    "MaxRow(field=f)",
    "Rows(f)",
    "Rows(f, limit=2)",
    "GroupBy(Rows(f), Rows(g))",
    "GroupBy(Rows(f), limit=3)",
    "Row(v > 10)",
    "Count(Row(v >< [5, 50]))",
    "Count(Row(f=1))Count(Row(f=2))Count(Intersect(Row(f=1), Row(g=3)))",
]


def _free_port():
    from tests.helpers import free_port
    return free_port()


def _data():
    rng = np.random.default_rng(5)
    bits = []
    for _ in range(3000):
        col = int(rng.integers(0, 6 * SW))
        bits.append(("f", int(rng.integers(0, 5)), col))
        if rng.random() < 0.5:
            bits.append(("g", int(rng.integers(0, 4)), col))
    vals = [(int(rng.integers(0, 6 * SW)), int(rng.integers(-20, 100))) for _ in range(500)]
    return bits, vals


def _setup_schema(holder):
    from pilosa_amd.models.field import FieldOptions
    idx = holder.create_index("i")
    idx.create_field("f", FieldOptions(cache_type="ranked", cache_size=1000))
    idx.create_field("g")
    idx.create_field("v", FieldOptions(type="int", min=-100, max=1000))


def _load(ex, bits, vals, mesh=None):
    """Writes: single Set() calls through the executor plus bulk imports
    (routed to owner ranks when a mesh is present)."""
    for fld, row, col in bits[:200]:
        ex.execute("i", f"Set({col}, {fld}={row})")
    rest = bits[200:]
    for fld in ("f", "g"):
        by_shard = {}
        for ff, row, col in rest:
            if ff == fld:
                by_shard.setdefault(col // SW, []).append((row, col))
        for shard, rc in sorted(by_shard.items()):
            rows = [r for r, _ in rc]
            cols = [c for _, c in rc]
            if mesh is not None and mesh.owner(shard) != 0:
                mesh.forward_import("bits", "i", fld, shard, {"rows": rows, "cols": cols})
            else:
                idx = ex.holder.index("i")
                idx.existence_field().import_bits(np.zeros(len(cols), np.uint64), np.asarray(cols, np.uint64))
                idx.field(fld).import_bits(rows, cols)
    for col, v in vals:
        ex.execute("i", f"Set({col}, v={v})")


def _canon(results):
    from pilosa_amd.server.encoding import result_to_json
    return json.dumps([result_to_json(r) for r in results], sort_keys=True, default=str)


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = tempfile.mkdtemp(prefix=f"mesh{rank}_")
    holder = Holder(d).open()
    ex = Executor(holder)
    mesh = ShardMesh(ex, block=1)
    ex.mesh = mesh
    try:
        if rank != 0:
            mesh.serve()
            return
        _setup_schema(holder)
        mesh.apply_schema()
        bits, vals = _data()
        _load(ex, bits, vals, mesh)
        got = [_canon(ex.execute("i", q).results) for q in QUERIES]
        per_rank = mesh.shard_counts()
        with open(os.path.join(outdir, "mesh.json"), "w") as fh:
            json.dump({"got": got, "ops": mesh.ops, "per_rank": {str(k): v for k, v in per_rank.items()}}, fh)
        mesh.stop()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_mesh_matches_single_process(world, tmp_path):
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder

    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "mesh.json"))

    d = tempfile.mkdtemp(prefix="mesh_ref_")
    holder = Holder(d).open()
    ex = Executor(holder)
    _setup_schema(holder)
    bits, vals = _data()
    _load(ex, bits, vals)
    want = [_canon(ex.execute("i", q).results) for q in QUERIES]
    ex.close()
    holder.close()
    for q, g, w in zip(QUERIES, res["got"], want):
        assert g == w, q
    # every rank held a share of the 6 shards; rank 0 stored only its own
    per_rank = res["per_rank"]
    owned = [set(per_rank[str(r)]["i"]) for r in range(world)]
    assert set().union(*owned) == set(range(6))
    for r in range(world):
        assert all(s % world == r for s in owned[r]), (r, owned[r])


def _failover_worker(rank, world, port, outdir):
    """Rank 1 serves the load phase, then dies without a clean shutdown; rank 0
    must notice on its next collective (timeout / peer loss), adopt rank 1's
    fragment files from its data dir and keep answering every query."""
    import datetime as dt

    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=dt.timedelta(seconds=15))
    dirs = {r: os.path.join(outdir, f"rank{r}") for r in range(world)}
    holder = Holder(dirs[rank]).open()
    ex = Executor(holder)
    mesh = ShardMesh(ex, block=1, peer_dirs=dirs)
    ex.mesh = mesh
    if rank != 0:
        mesh.serve()            # until the front end's stop below
        ex.close()
        holder.close()          # releases the fragment flocks, like a dead process
        os._exit(0)             # no destroy_process_group: the peer just vanishes
    _setup_schema(holder)
    mesh.apply_schema()
    bits, vals = _data()
    _load(ex, bits, vals, mesh)
    before = [_canon(ex.execute("i", q).results) for q in QUERIES]
    mesh.stop()
    import time
    time.sleep(1.0)
    after = [_canon(ex.execute("i", q).results) for q in QUERIES]
    with open(os.path.join(outdir, "failover.json"), "w") as fh:
        json.dump({"before": before, "after": after, "failed_over": mesh.failed_over,
                   "error": mesh.failover_error, "mesh_detached": ex.mesh is None}, fh)
    ex.close()
    holder.close()
    os._exit(0)


def test_mesh_failover_adopts_dead_rank_shards(tmp_path):
    mp.start_processes(_failover_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "failover.json"))
    assert res["failed_over"] and res["mesh_detached"], res["error"]
    assert res["after"] == res["before"]


def test_result_codec_round_trip():
    from pilosa_amd.executor import FieldRow, GroupCount, RowIdentifiers, ValCount
    from pilosa_amd.models.cache import Pair
    from pilosa_amd.models.row import Row
    from pilosa_amd.parallel.collectives import RemoteError, decode, encode
    r = Row(np.array([1, 5, 3 << 20], np.uint64))
    r.attrs = {"x": 1}
    objs = [3, None, True, [Pair(1, 2), Pair(3, 4, "k")], ValCount(-5, 6),
            [GroupCount([FieldRow("f", 1), FieldRow("g", 2, "x")], 7)], RowIdentifiers([1, 2], ["a", "b"]),
            {"i": [1, 2]}]
    for o in objs:
        assert decode(encode(o)) == o
    got = decode(encode(r))
    assert [int(c) for c in got.columns()] == [1, 5, 3 << 20] and got.attrs == {"x": 1}
    e = decode(encode(ValueError("boom")))
    assert isinstance(e, RemoteError) and "boom" in str(e)


def _pipeline_worker(rank, world, port, outdir):
    """Concurrent multi-Count requests through the mesh text path: several
    batches in flight (broadcast on the gloo command group, async
    all-reduces), answers equal to one Count per request; a request naming an
    unknown field falls back to the general path and raises its error."""
    import threading

    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = Holder(tempfile.mkdtemp(prefix=f"meshp{rank}_")).open()
    ex = Executor(holder)
    mesh = ShardMesh(ex, block=1)
    ex.mesh = mesh
    try:
        if rank != 0:
            mesh.serve()
            return
        _setup_schema(holder)
        mesh.apply_schema()
        bits, vals = _data()
        _load(ex, bits, vals, mesh)
        rng = np.random.default_rng(3)
        reqs = []
        for _ in range(24):
            qs = [f"Count(Intersect(Row(f={int(a)}), Row(g={int(b)})))" for a, b in
                  zip(rng.integers(0, 5, 6), rng.integers(0, 4, 6))]
            reqs.append(qs)
        got = [None] * len(reqs)

        def run(k):
            got[k] = ex.execute("i", " ".join(reqs[k])).results
        ts = [threading.Thread(target=run, args=(k,)) for k in range(len(reqs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        want = [[ex.execute("i", q).results[0] for q in qs] for qs in reqs]
        err = ""
        try:
            ex.execute("i", "Count(Row(f=1)) Count(Row(zz=1))")
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        with open(os.path.join(outdir, "pipe.json"), "w") as fh:
            json.dump({"got": got, "want": want, "max_in_flight": mesh.max_in_flight, "seq": mesh.seq,
                       "err": err, "rank_errors": mesh.last_count_text_errors}, fh)
        mesh.stop()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()


def test_mesh_count_text_pipelined(tmp_path):
    mp.start_processes(_pipeline_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "pipe.json"))
    assert res["got"] == res["want"]
    assert res["seq"] >= 24
    assert res["max_in_flight"] >= 2, res["max_in_flight"]
    assert "field not found" in res["err"] and res["rank_errors"], res


CALL_QUERIES = ["TopN(f, n=3)", "TopN(f, Row(g=3), n=2)", "Sum(Row(f=1), field=v)", "Rows(f)",
                "GroupBy(Rows(f), Rows(g))", "MaxRow(field=f)", "Min(field=v)", "Row(f=2)"]


def _call_pipeline_worker(rank, world, port, outdir):
    """Concurrent general calls (TopN, Sum, Rows, GroupBy, ...) through the
    mesh: each request's OP_CALL is issued under the front-end lock and
    completed (all-gather wait, decode, reduce) outside it, so requests
    overlap; answers equal the same calls run one at a time."""
    import threading

    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = Holder(tempfile.mkdtemp(prefix=f"meshc{rank}_")).open()
    ex = Executor(holder)
    mesh = ShardMesh(ex, block=1)
    ex.mesh = mesh
    try:
        if rank != 0:
            mesh.serve()
            return
        _setup_schema(holder)
        mesh.apply_schema()
        bits, vals = _data()
        _load(ex, bits, vals, mesh)
        want = {q: _canon(ex.execute("i", q).results) for q in CALL_QUERIES}
        reqs = [CALL_QUERIES[k % len(CALL_QUERIES)] for k in range(48)]
        got = [None] * len(reqs)

        def run(k):
            got[k] = _canon(ex.execute("i", reqs[k]).results)
        ts = [threading.Thread(target=run, args=(k,)) for k in range(len(reqs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        with open(os.path.join(outdir, "calls.json"), "w") as fh:
            json.dump({"ok": [got[k] == want[reqs[k]] for k in range(len(reqs))],
                       "max_in_flight": mesh.max_in_flight}, fh)
        mesh.stop()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()


def test_mesh_general_calls_pipelined(tmp_path):
    mp.start_processes(_call_pipeline_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "calls.json"))
    assert all(res["ok"]), res["ok"]
    assert res["max_in_flight"] >= 2, res["max_in_flight"]


def _call_worker(rank, world, port, outdir):
    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = Holder(tempfile.mkdtemp(prefix=f"call{rank}_")).open()
    ex = Executor(holder)
    mesh = ShardMesh(ex, block=1)
    ex.mesh = mesh
    try:
        if rank != 0:
            mesh.serve()
            return
        _setup_schema(holder)
        mesh.apply_schema()
        bits, vals = _data()
        _load(ex, bits, vals, mesh)
        per_call = {}
        for q in ("Sum(field=v)", "Rows(f)", "Row(f=1)", "Max(Row(f=2), field=v)", "GroupBy(Rows(f), Rows(g))"):
            ex.execute("i", q)                 # learns the call's gather capacity
            c0, b0 = mesh.comm.data_calls, mesh.comm.board_gathers
            got = _canon(ex.execute("i", q).results)
            per_call[q] = [mesh.comm.data_calls - c0, mesh.comm.board_gathers - b0, got]
        # without the results board: ONE fixed-capacity all-gather per call;
        # a capacity far too small: the ranks' partials overflow it, the front
        # end re-issues the call once with a capacity that fits
        mesh.comm.use_board = False
        c0 = mesh.comm.data_calls
        rccl_sum = _canon(ex.execute("i", "Sum(field=v)").results)
        rccl_calls = mesh.comm.data_calls - c0
        mesh._call_cap["Row"] = (4, 0)
        r0 = mesh.call_retries
        big = _canon(ex.execute("i", "Row(f=1)").results)
        retries = mesh.call_retries - r0
        c0 = mesh.comm.data_calls
        again = _canon(ex.execute("i", "Row(f=1)").results)
        with open(os.path.join(outdir, "calls.json"), "w") as fh:
            json.dump({"per_call": per_call, "big": big, "retries": retries, "again": again,
                       "again_calls": mesh.comm.data_calls - c0, "rccl_sum": rccl_sum, "rccl_calls": rccl_calls,
                       "board": mesh.comm.board or mesh.ring}, fh)
        mesh.stop()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()


def test_general_call_is_one_speculative_gather(tmp_path):
    """a general call's small partials go through
    the shared-memory results board (no collective); otherwise they travel in
    ONE fixed-capacity all-gather -- no size all-gather, no host read before
    the data moves; a rank whose partial does not fit says so inside that
    gather and the front end re-issues the call with a capacity that fits."""
    mp.start_processes(_call_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "calls.json"))
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    holder = Holder(tempfile.mkdtemp(prefix="call_ref_")).open()
    ex = Executor(holder)
    _setup_schema(holder)
    bits, vals = _data()
    _load(ex, bits, vals)
    assert res["board"]
    for q, (ncoll, nboard, got) in res["per_call"].items():
        # small partials: the shared-memory results board, no collective
        assert (ncoll, nboard) == (0, 1), (q, ncoll, nboard)
        assert got == _canon(ex.execute("i", q).results), q
    assert res["rccl_calls"] == 1 and res["rccl_sum"] == _canon(ex.execute("i", "Sum(field=v)").results)
    want_row = _canon(ex.execute("i", "Row(f=1)").results)
    ex.close()
    holder.close()
    assert res["retries"] == 1 and res["big"] == want_row
    assert res["again"] == want_row and res["again_calls"] == 1
