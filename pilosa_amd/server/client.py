"""Internal HTTP client for node<->node and CLI<->node traffic
(reference: client.go InternalClient iface, http/client.go).

Query fan-out posts the canonical PQL string with ``Remote=true`` and the
shard list as protobuf (http/client.go:268-316); imports, fragment streaming,
block checksums, translate-log tailing and cluster messages use the same
routes as the reference.  Tracing headers are injected on every request.
"""
from __future__ import annotations

import http.client
import json
import threading
from typing import Dict, List, Optional, Sequence
from urllib.parse import urlencode

from pilosa_amd.errors import PilosaError
from pilosa_amd.server.encoding import response_from_pb
from pilosa_amd.utils import tracing
from pilosa_amd.wire import pb

PROTO = "application/x-protobuf"


class ClientError(PilosaError):
    def __init__(self, status, msg):
        super().__init__(f"server error {status}: {msg}")
        self.status = status
        self.body = msg


class InternalClient:
    def __init__(self, timeout: float = 30.0, skip_verify: bool = False):
        self.timeout = timeout
        self.local_node: Optional[dict] = None   # sender identity for messages that carry one
        self.skip_verify = skip_verify
        self._local = threading.local()

    def _conn(self, uri) -> http.client.HTTPConnection:
        pool = getattr(self._local, "pool", None)
        if pool is None:
            pool = self._local.pool = {}
        key = (uri.host, uri.port)
        c = pool.get(key)
        if c is None:
            if getattr(uri, "scheme", "http") == "https":
                import ssl
                ctx = ssl.create_default_context()
                if self.skip_verify:
                    ctx.check_hostname = False
                    ctx.verify_mode = ssl.CERT_NONE
                c = http.client.HTTPSConnection(uri.host, uri.port, timeout=self.timeout, context=ctx)
            else:
                c = http.client.HTTPConnection(uri.host, uri.port, timeout=self.timeout)
            pool[key] = c
        return c

    def do(self, uri, method: str, path: str, body: bytes = b"", headers: Optional[Dict[str, str]] = None,
           query: Optional[dict] = None, ok=(200,)) -> bytes:
        if query:
            path = path + "?" + urlencode(query)
        hdrs = {"Content-Length": str(len(body))}
        hdrs.update(headers or {})
        tracing.inject_headers(hdrs)
        for attempt in range(2):
            c = self._conn(uri)
            try:
                c.request(method, path, body=body, headers=hdrs)
                resp = c.getresponse()
                data = resp.read()
                break
            except (ConnectionError, http.client.HTTPException, OSError):
                c.close()
                self._local.pool.pop((uri.host, uri.port), None)
                if attempt == 1:
                    raise
        if resp.status not in ok:
            raise ClientError(resp.status, data.decode(errors="replace").strip())
        return data

    # ------------------------------------------------------------ queries
    def query_node(self, node, index: str, query: str, shards: Optional[Sequence[int]]):
        req = pb.QueryRequest(Query=query, Shards=list(shards or []), Remote=True)
        data = self.do(node.uri, "POST", f"/index/{index}/query", req.SerializeToString(),
                       {"Content-Type": PROTO, "Accept": PROTO}, ok=(200, 400))
        resp = response_from_pb(data)
        if resp.err:
            raise PilosaError(resp.err)
        return resp.results

    def query(self, uri, index: str, query: str, **opts) -> dict:
        q = {k: ("true" if v is True else v) for k, v in opts.items() if v not in (None, False)}
        data = self.do(uri, "POST", f"/index/{index}/query", query.encode(), {"Accept": "application/json"},
                       query=q or None, ok=(200, 400, 413))
        return json.loads(data)

    # ------------------------------------------------------------ imports
    def import_bits(self, node, index, field, shard, rows, cols, timestamps=(), clear=False, ignore_key_check=False,
                    row_keys=(), col_keys=()):
        req = pb.ImportRequest(Index=index, Field=field, Shard=shard, RowIDs=list(rows), ColumnIDs=list(cols),
                               Timestamps=list(timestamps or []), RowKeys=list(row_keys), ColumnKeys=list(col_keys))
        q = {}
        if clear:
            q["clear"] = "true"
        if ignore_key_check:
            q["ignoreKeyCheck"] = "true"
        self.do(node.uri, "POST", f"/index/{index}/field/{field}/import", req.SerializeToString(),
                {"Content-Type": PROTO, "Accept": PROTO}, query=q or None)

    def import_values(self, node, index, field, shard, cols, values, clear=False, ignore_key_check=False,
                      col_keys=()):
        req = pb.ImportValueRequest(Index=index, Field=field, Shard=shard, ColumnIDs=list(cols),
                                    Values=list(values), ColumnKeys=list(col_keys))
        q = {}
        if clear:
            q["clear"] = "true"
        if ignore_key_check:
            q["ignoreKeyCheck"] = "true"
        self.do(node.uri, "POST", f"/index/{index}/field/{field}/import", req.SerializeToString(),
                {"Content-Type": PROTO, "Accept": PROTO}, query=q or None)

    def import_roaring(self, node, index, field, shard, views: Dict[str, bytes], clear=False, remote=False):
        req = pb.ImportRoaringRequest(Clear=clear)
        for name, data in views.items():
            req.views.add(Name=name, Data=data)
        q = {"remote": "true"} if remote else None
        self.do(node.uri, "POST", f"/index/{index}/field/{field}/import-roaring/{shard}", req.SerializeToString(),
                {"Content-Type": PROTO, "Accept": PROTO}, query=q)

    # ------------------------------------------------------------ schema
    def create_index(self, uri, index, keys=False, track_existence=True):
        body = json.dumps({"options": {"keys": keys, "trackExistence": track_existence}}).encode()
        self.do(uri, "POST", f"/index/{index}", body, {"Content-Type": "application/json"}, ok=(200, 409))

    def create_field(self, uri, index, field, options: dict):
        body = json.dumps({"options": options}).encode()
        self.do(uri, "POST", f"/index/{index}/field/{field}", body, {"Content-Type": "application/json"},
                ok=(200, 409))

    def schema(self, uri) -> List[dict]:
        return json.loads(self.do(uri, "GET", "/schema"))["indexes"]

    def status(self, uri) -> dict:
        return json.loads(self.do(uri, "GET", "/status"))

    def version(self, uri) -> str:
        return json.loads(self.do(uri, "GET", "/version"))["version"]

    def max_shards(self, uri) -> Dict[str, int]:
        return json.loads(self.do(uri, "GET", "/internal/shards/max"))["standard"]

    def fragment_nodes(self, uri, index, shard) -> List[dict]:
        return json.loads(self.do(uri, "GET", "/internal/fragment/nodes", query={"index": index, "shard": shard}))

    # ------------------------------------------------------------ anti-entropy / resize
    def fragment_blocks(self, uri, index, field, view, shard) -> List[dict]:
        data = self.do(uri, "GET", "/internal/fragment/blocks",
                       query={"index": index, "field": field, "view": view, "shard": shard}, ok=(200, 404))
        try:
            return json.loads(data).get("blocks", [])
        except ValueError:
            return []

    def block_data(self, uri, index, field, view, shard, block):
        req = pb.BlockDataRequest(Index=index, Field=field, View=view, Shard=shard, Block=block)
        data = self.do(uri, "GET", "/internal/fragment/block/data", req.SerializeToString(),
                       {"Content-Type": PROTO}, ok=(200, 404))
        m = pb.BlockDataResponse()
        m.ParseFromString(data)
        return list(m.RowIDs), list(m.ColumnIDs)

    def fragment_data(self, uri, index, field, view, shard) -> bytes:
        return self.do(uri, "GET", "/internal/fragment/data",
                       query={"index": index, "field": field, "view": view, "shard": shard})

    def attr_diff(self, uri, index, field: Optional[str], blocks: List[dict]) -> Dict[int, dict]:
        path = f"/internal/index/{index}/field/{field}/attr/diff" if field else f"/internal/index/{index}/attr/diff"
        data = self.do(uri, "POST", path, json.dumps({"blocks": blocks}).encode(),
                       {"Content-Type": "application/json"})
        return {int(k): v for k, v in json.loads(data).get("attrs", {}).items()}

    def translate_data(self, uri, offset: int) -> bytes:
        return self.do(uri, "GET", "/internal/translate/data", query={"offset": offset})

    def translate_keys(self, uri, index, field, keys) -> List[int]:
        req = pb.TranslateKeysRequest(Index=index, Field=field or "", Keys=list(keys))
        data = self.do(uri, "POST", "/internal/translate/keys", req.SerializeToString(), {"Content-Type": PROTO})
        m = pb.TranslateKeysResponse()
        m.ParseFromString(data)
        return list(m.IDs)

    # ------------------------------------------------------------ messages
    def send_message(self, node, msg: dict):
        """POST one cluster message in the reference's wire format: a type
        byte + protobuf (http/client.go:1017 SendMessage, wire/messages.py)."""
        from pilosa_amd.wire import messages
        self.do(node.uri, "POST", "/internal/cluster/message", messages.encode(msg, self.local_node),
                {"Content-Type": messages.CONTENT_TYPE, "Accept": "application/json"})

    def export_csv(self, uri, index, field, shard) -> str:
        return self.do(uri, "GET", "/export", query={"index": index, "field": field, "shard": shard},
                       headers={"Accept": "text/csv"}).decode()
