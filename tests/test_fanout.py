"""Concurrent node fan-out of the executor's map/reduce (reference
executor.go:2530-2552: one goroutine per node, local included): a query over
three nodes takes about the slowest node's time, not the sum, and a failed
node's shards are retried on their replicas, also concurrently."""
import tempfile
import threading
import time

from pilosa_amd.executor import Executor
from pilosa_amd.models.holder import Holder
from pilosa_amd.shardwidth import SHARD_WIDTH as SW


class _Node:
    def __init__(self, nid):
        self.id = nid
        self.state = "READY"


class _Cluster:
    """Shard s lives on node s % 3 (with ``replicas``, also on the next node)."""

    def __init__(self, nodes, me, replicas):
        self.nodes = nodes
        self.node = me
        self.replicas = replicas
        self.replica_n = 2 if replicas else 1

    def shard_nodes(self, index, s):
        k = len(self.nodes)
        return [self.nodes[s % k], self.nodes[(s + 1) % k]][:2 if self.replicas else 1]


class _SlowClient:
    def __init__(self, delay, fail=()):
        self.delay = delay
        self.fail = set(fail)
        self.calls = []
        self.mu = threading.Lock()
        self.active = 0
        self.max_active = 0

    def query_node(self, node, index, q, shards):
        with self.mu:
            self.calls.append((node.id, tuple(shards)))
            self.active += 1
            self.max_active = max(self.max_active, self.active)
        try:
            time.sleep(self.delay)
            if node.id in self.fail:
                raise ConnectionError(f"{node.id} down")
            return [len(shards) * 10]
        finally:
            with self.mu:
                self.active -= 1


def _executor(client, replicas=False):
    holder = Holder(tempfile.mkdtemp()).open()
    idx = holder.create_index("i")
    f = idx.create_field("f")
    f.set_bit(1, 0)          # shard 0: local node
    f.set_bit(1, 3 * SW)     # shard 3: local node
    nodes = [_Node("n0"), _Node("n1"), _Node("n2")]
    ex = Executor(holder, cluster=_Cluster(nodes, nodes[0], replicas), client=client)
    return ex, holder


def test_fanout_wall_time_is_the_slowest_node():
    client = _SlowClient(0.4)
    ex, holder = _executor(client)
    try:
        t0 = time.perf_counter()
        got = ex.execute("i", "Count(Row(f=1))", shards=list(range(6))).results[0]
        dt = time.perf_counter() - t0
    finally:
        ex.close()
        holder.close()
    # local shards 0, 3 hold 2 bits; nodes n1 (shards 1, 4) and n2 (2, 5) answer 20 each
    assert got == 2 + 20 + 20
    assert client.max_active == 2, client.max_active
    assert dt < 0.75, dt      # two sequential remote calls would take >= 0.8 s


def test_fanout_failover_to_replicas():
    client = _SlowClient(0.05, fail={"n1"})
    ex, holder = _executor(client, replicas=True)
    try:
        got = ex.execute("i", "Count(Row(f=1))", shards=list(range(6))).results[0]
    finally:
        ex.close()
        holder.close()
    # the local node serves shards 0, 3 and (as replica) 2, 5; n1's shards 1, 4
    # fail and move to their replica n2, which answers 20
    assert got == 2 + 20
    assert ("n1", (1, 4)) in client.calls and ("n2", (1, 4)) in client.calls, client.calls


def test_fanout_failover_does_not_starve_the_pool():
    """with every fan-out worker busy on a failing node, the
    replica retries must not wait on futures queued to that same pool.  A
    pool of one thread and one failing node with one replica used to hang."""
    import concurrent.futures as cf

    client = _SlowClient(0.01, fail={"n1"})
    ex, holder = _executor(client, replicas=True)
    ex._fanout = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="fanout-test")
    done = []
    t = threading.Thread(target=lambda: done.append(
        ex.execute("i", "Count(Row(f=1))", shards=list(range(6))).results[0]), daemon=True)
    try:
        t.start()
        t.join(10)
        assert not t.is_alive(), "fan-out pool starved by replica retries"
        assert done == [2 + 20]
    finally:
        ex.close()
        holder.close()
