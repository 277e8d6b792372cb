"""Ported expectations of the reference's api_test.go: keyed imports sent to
the coordinator of a two-node cluster are translated there and forwarded to
the shard's owner, and either node answers with the keys (TestAPI_Import
RowIDColumnKey / SchemaHasNoExists / RowKeyColumnID, TestAPI_ImportValue
ValColumnKey).  Placement uses the test's offset-mod hasher (shard 0 lives on
node1)."""
import time

import pytest

from pilosa_amd.models.field import FieldOptions
from pilosa_amd.server.api import QueryRequest
from pilosa_amd.shardwidth import SHARD_WIDTH
from tests import test_server_ref as ref


class OffsetModHasher:
    def hash(self, key: int, n: int) -> int:
        return (int(key) + 1) % n


@pytest.fixture(scope="module")
def cluster():
    orig = ref.Server

    class _S(orig):
        def __init__(self, *a, **kw):
            kw["hasher"] = OffsetModHasher()
            super().__init__(*a, **kw)
    ref.Server = _S     # the module's cluster harness, with this test's placement
    try:
        c = ref._Cluster(2)
    finally:
        ref.Server = orig
    yield c
    c.close()


def _q(node, index, pql):
    return node.api.query(QueryRequest(index, pql)).results[0]


def _keys(node, index, pql, want):
    """A non-coordinator learns new keys from the coordinator's key log
    (asynchronous replication, as in the reference): poll briefly."""
    deadline = time.time() + 10
    while True:
        got = _q(node, index, pql).keys
        if got == want or time.time() > deadline:
            return got
        time.sleep(0.05)


def test_import_row_id_column_key(cluster):  # RowIDColumnKey, SchemaHasNoExists
    m0, m1 = cluster.nodes
    m0.api.create_index("rick", keys=True, track_existence=True)
    m0.api.create_field("rick", "f", FieldOptions(type="set", cache_type="ranked", cache_size=100))
    keys = [f"col{i}" for i in range(1, 11)]
    m0.api.import_bits("rick", "f", 0, row_ids=[1] * 10, col_keys=keys, timestamps=[0] * 10)
    for m in (m0, m1):
        assert _keys(m, "rick", "Row(f=1)", keys) == keys
    for ii in m1.api.schema():
        assert not any(f["name"].startswith("_") for f in ii["fields"])


def test_import_row_key_column_id(cluster):  # RowKeyColumnID
    m0, m1 = cluster.nodes
    m0.api.create_index("rkci", keys=False)
    m0.api.create_field("rkci", "f", FieldOptions(type="set", cache_type="ranked", cache_size=100, keys=True))
    cols = [1, 2, SHARD_WIDTH + 1]
    m0.api.import_bits("rkci", "f", 0, row_keys=["rowkey"] * 3, col_ids=cols, timestamps=[0] * 3)
    for m in (m0, m1):
        assert list(_q(m, "rkci", "Row(f=rowkey)").columns()) == cols


def test_import_value_column_key(cluster):  # TestAPI_ImportValue ValColumnKey
    m0, m1 = cluster.nodes
    m0.api.create_index("valck", keys=True)
    m0.api.create_field("valck", "f", FieldOptions(type="int", min=-(1 << 63), max=(1 << 63) - 1))
    keys = [f"col{i}" for i in range(1, 11)]
    m0.api.import_values("valck", "f", 0, values=list(range(1, 11)), col_keys=keys)
    for m in (m0, m1):
        assert _keys(m, "valck", "Row(f>0)", keys) == keys
