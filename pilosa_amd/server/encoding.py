"""Query result <-> JSON / protobuf (reference: handler.go QueryResponse
MarshalJSON, encoding/proto/proto.go)."""
from __future__ import annotations

from typing import Any, List, Optional

from pilosa_amd.executor import FieldRow, GroupCount, QueryResponse, RowIdentifiers, ValCount
from pilosa_amd.models.cache import Pair, PairArray
from pilosa_amd.models.row import Row
from pilosa_amd.wire import (ATTR_TYPE_BOOL, ATTR_TYPE_FLOAT, ATTR_TYPE_INT, ATTR_TYPE_STRING,
                             QUERY_RESULT_TYPE_BOOL, QUERY_RESULT_TYPE_GROUPCOUNTS, QUERY_RESULT_TYPE_NIL,
                             QUERY_RESULT_TYPE_PAIR, QUERY_RESULT_TYPE_PAIRS, QUERY_RESULT_TYPE_ROW,
                             QUERY_RESULT_TYPE_ROWIDENTIFIERS, QUERY_RESULT_TYPE_ROWIDS,
                             QUERY_RESULT_TYPE_UINT64, QUERY_RESULT_TYPE_VALCOUNT, pb)


def result_to_json(r: Any):
    if r is None:
        return None
    if isinstance(r, bool):
        return r
    if isinstance(r, int):
        return r
    if isinstance(r, (Row, ValCount, Pair, RowIdentifiers, GroupCount, FieldRow, PairArray)):
        return r.to_json()
    if isinstance(r, list):
        return [result_to_json(x) for x in r]
    return r


def result_json_bytes(r) -> bytes:
    """One result as Go's encoding/json writes it (PairArray natively)."""
    from pilosa_amd.utils import gojson
    if isinstance(r, PairArray):
        return r.json_bytes()
    return gojson.dumps(result_to_json(r)).encode()


def response_json_bytes(resp: QueryResponse) -> bytes:
    """The query response body as Go's json.Encoder writes it (trailing
    newline).  Columnar TopN results (PairArray) are written straight from
    their arrays; everything else through the generic encoder."""
    from pilosa_amd.utils import gojson
    if resp.err is not None or resp.column_attr_sets or \
            not any(isinstance(r, PairArray) for r in resp.results):
        return gojson.encode_line(response_to_json(resp)).encode()
    parts = [result_json_bytes(r) for r in resp.results]
    return b'{"results":[' + b",".join(parts) + b"]}\n"


def response_to_json(resp: QueryResponse) -> dict:
    if resp.err is not None:
        return {"error": str(resp.err)}
    out = {"results": [result_to_json(r) for r in resp.results]}
    if resp.column_attr_sets:
        out["columnAttrs"] = resp.column_attr_sets
    return out


# ------------------------------------------------------------ protobuf
def attrs_to_pb(attrs: Optional[dict]):
    out = []
    for k in sorted(attrs or {}):
        v = attrs[k]
        a = pb.Attr(Key=k)
        if isinstance(v, bool):
            a.Type, a.BoolValue = ATTR_TYPE_BOOL, v
        elif isinstance(v, int):
            a.Type, a.IntValue = ATTR_TYPE_INT, v
        elif isinstance(v, float):
            a.Type, a.FloatValue = ATTR_TYPE_FLOAT, v
        else:
            a.Type, a.StringValue = ATTR_TYPE_STRING, str(v)
        out.append(a)
    return out


def attrs_from_pb(attrs) -> dict:
    d = {}
    for a in attrs:
        if a.Type == ATTR_TYPE_BOOL:
            d[a.Key] = a.BoolValue
        elif a.Type == ATTR_TYPE_INT:
            d[a.Key] = a.IntValue
        elif a.Type == ATTR_TYPE_FLOAT:
            d[a.Key] = a.FloatValue
        else:
            d[a.Key] = a.StringValue
    return d


def result_to_pb(r: Any, call_name: str = ""):
    m = pb.QueryResult()
    if r is None:
        m.Type = QUERY_RESULT_TYPE_NIL
    elif isinstance(r, Row):
        m.Type = QUERY_RESULT_TYPE_ROW
        m.Row.Columns.extend(int(c) for c in r.columns())
        if r.keys:
            m.Row.Keys.extend(r.keys)
        m.Row.Attrs.extend(attrs_to_pb(r.attrs))
    elif isinstance(r, bool):
        m.Type = QUERY_RESULT_TYPE_BOOL
        m.Changed = r
    elif isinstance(r, int):
        m.Type = QUERY_RESULT_TYPE_UINT64
        m.N = r
    elif isinstance(r, ValCount):
        m.Type = QUERY_RESULT_TYPE_VALCOUNT
        m.ValCount.Val, m.ValCount.Count = r.val, r.count
    elif isinstance(r, Pair):
        m.Type = QUERY_RESULT_TYPE_PAIR
        m.Pairs.add(ID=r.id, Key=r.key, Count=r.count)
    elif isinstance(r, RowIdentifiers):
        m.Type = QUERY_RESULT_TYPE_ROWIDENTIFIERS
        m.RowIdentifiers.Rows.extend(r.rows)
        if r.keys:
            m.RowIdentifiers.Keys.extend(r.keys)
    elif isinstance(r, PairArray):
        m.Type = QUERY_RESULT_TYPE_PAIRS
        for i, c in zip(r.ids.tolist(), r.counts.tolist()):
            m.Pairs.add(ID=i, Count=c)
    elif isinstance(r, list) and (not r and call_name == "TopN" or r and isinstance(r[0], Pair)):
        m.Type = QUERY_RESULT_TYPE_PAIRS
        for p in r:
            m.Pairs.add(ID=p.id, Key=p.key, Count=p.count)
    elif isinstance(r, list) and (not r and call_name == "GroupBy" or r and isinstance(r[0], GroupCount)):
        m.Type = QUERY_RESULT_TYPE_GROUPCOUNTS
        for g in r:
            gc = m.GroupCounts.add(Count=g.count)
            for fr in g.group:
                gc.Group.add(Field=fr.field, RowID=fr.row_id, RowKey=fr.row_key)
    elif isinstance(r, list):
        m.Type = QUERY_RESULT_TYPE_ROWIDS
        m.RowIDs.extend(int(x) for x in r)
    else:
        raise TypeError(f"cannot encode result {type(r).__name__}")
    return m


def result_from_pb(m):
    t = m.Type
    if t == QUERY_RESULT_TYPE_NIL:
        return None
    if t == QUERY_RESULT_TYPE_ROW:
        import numpy as np
        r = Row(np.array(list(m.Row.Columns), dtype=np.uint64))
        if m.Row.Keys:
            r.keys = list(m.Row.Keys)
        r.attrs = attrs_from_pb(m.Row.Attrs)
        return r
    if t == QUERY_RESULT_TYPE_BOOL:
        return m.Changed
    if t == QUERY_RESULT_TYPE_UINT64:
        return m.N
    if t == QUERY_RESULT_TYPE_VALCOUNT:
        return ValCount(m.ValCount.Val, m.ValCount.Count)
    if t == QUERY_RESULT_TYPE_PAIR:
        p = m.Pairs[0]
        return Pair(p.ID, p.Count, p.Key)
    if t == QUERY_RESULT_TYPE_PAIRS:
        return [Pair(p.ID, p.Count, p.Key) for p in m.Pairs]
    if t == QUERY_RESULT_TYPE_ROWIDENTIFIERS:
        return RowIdentifiers(list(m.RowIdentifiers.Rows), list(m.RowIdentifiers.Keys) or None)
    if t == QUERY_RESULT_TYPE_ROWIDS:
        return list(m.RowIDs)
    if t == QUERY_RESULT_TYPE_GROUPCOUNTS:
        return [GroupCount([FieldRow(g.Field, g.RowID, g.RowKey) for g in gc.Group], gc.Count)
                for gc in m.GroupCounts]
    raise ValueError(f"unknown result type {t}")


def response_to_pb(resp: QueryResponse, calls: Optional[List] = None) -> bytes:
    m = pb.QueryResponse()
    if resp.err is not None:
        m.Err = str(resp.err)
    else:
        for i, r in enumerate(resp.results):
            name = calls[i].name if calls and i < len(calls) else ""
            m.Results.append(result_to_pb(r, name))
        for cas in resp.column_attr_sets or []:
            s = m.ColumnAttrSets.add(ID=cas.get("id", 0), Key=cas.get("key", ""))
            s.Attrs.extend(attrs_to_pb(cas.get("attrs")))
    return m.SerializeToString()


def response_from_pb(data: bytes) -> QueryResponse:
    m = pb.QueryResponse()
    m.ParseFromString(data)
    if m.Err:
        return QueryResponse(err=m.Err)
    sets = [{"id": s.ID, "key": s.Key, "attrs": attrs_from_pb(s.Attrs)} for s in m.ColumnAttrSets] or None
    return QueryResponse([result_from_pb(r) for r in m.Results], sets)
