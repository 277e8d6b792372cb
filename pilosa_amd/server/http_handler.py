"""HTTP API (reference: http/handler.go routes :276-314).

Stdlib ``ThreadingHTTPServer``; routes, status codes, JSON/protobuf content
negotiation (:977-1052), per-route query-argument validation (:173-227),
tracing header extraction (:229), stats + slow-query logging (:238-272) and
panic recovery (:323) mirror the reference.
"""
from __future__ import annotations

import base64
import json
import re
import socket
import threading
import time
import traceback
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlparse

from pilosa_amd.utils import gojson
from pilosa_amd import _roaring
from pilosa_amd.errors import (APIMethodNotAllowedError, BadRequestError, ConflictError, ErrClusterDoesNotOwnShard,
                               ErrFieldNotFound, ErrFragmentNotFound, ErrIndexNotFound, ErrTooManyWrites,
                               ErrNodeNotCoordinator, ErrResizeNotRunning, NotFoundError, PilosaError, cause)
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.server.api import QueryRequest
from pilosa_amd.server.encoding import response_json_bytes, response_to_json, response_to_pb
from pilosa_amd.utils import tracing
from pilosa_amd.wire import pb

JSON = "application/json"
PROTO = "application/x-protobuf"

# allowed query arguments per route (handler.go populateValidators)
VALIDATORS: Dict[str, Tuple[List[str], List[str]]] = {
    "PostQuery": ([], ["shards", "columnAttrs", "excludeRowAttrs", "excludeColumns", "profile"]),
    "PostImport": ([], ["clear", "ignoreKeyCheck"]),
    "PostImportRoaring": ([], ["remote", "clear"]),
    "GetExport": (["index", "field", "shard"], []),
    "GetFragmentNodes": (["shard", "index"], []),
    "GetFragmentData": (["index", "field", "view", "shard"], []),
    "GetFragmentBlocks": (["index", "field", "view", "shard"], []),
    "GetFragmentBlockData": ([], ["index", "field", "view", "shard", "block"]),
    "PostSchema": ([], ["remote"]),
    "GetTranslateData": ([], ["offset"]),
}


class HTTPError(Exception):
    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status


def _status_for(err: Exception) -> int:
    if isinstance(err, BadRequestError):
        return 400
    if isinstance(err, ConflictError):
        return 409
    if isinstance(err, NotFoundError):
        return 404
    if isinstance(err, APIMethodNotAllowedError):
        return 405
    return 500


class Handler:
    def __init__(self, api, server=None, logger=None, stats=None):
        self.api = api
        self.server = server
        self.logger = logger
        self.stats = stats
        self.allowed_origins: List[str] = []   # CORS (http/handler.go OptHandlerAllowedOrigins)
        self.routes: List[Tuple[str, re.Pattern, Callable, str]] = []
        r = self._route
        r("GET", r"/", self.home, "Home")
        r("POST", r"/cluster/resize/abort", self.post_resize_abort, "PostClusterResizeAbort")
        r("POST", r"/cluster/resize/remove-node", self.post_remove_node, "PostClusterResizeRemoveNode")
        r("POST", r"/cluster/resize/set-coordinator", self.post_set_coordinator, "PostClusterResizeSetCoordinator")
        r("GET", r"/debug/vars", self.debug_vars, "DebugVars")
        r("GET", r"/debug/traces", self.debug_traces, "DebugTraces")
        r("GET", r"/debug/pprof/(?P<rest>.*)", self.debug_pprof, "DebugPprof")
        r("GET", r"/metrics", self.metrics, "Metrics")
        r("GET", r"/export", self.get_export, "GetExport")
        r("GET", r"/index", self.get_schema, "GetIndexes")
        r("GET", r"/index/(?P<index>[^/]+)", self.get_index, "GetIndex")
        r("POST", r"/index/(?P<index>[^/]+)", self.post_index, "PostIndex")
        r("DELETE", r"/index/(?P<index>[^/]+)", self.delete_index, "DeleteIndex")
        r("POST", r"/index/(?P<index>[^/]+)/field/(?P<field>[^/]+)", self.post_field, "PostField")
        r("DELETE", r"/index/(?P<index>[^/]+)/field/(?P<field>[^/]+)", self.delete_field, "DeleteField")
        r("POST", r"/index/(?P<index>[^/]+)/field/(?P<field>[^/]+)/import", self.post_import, "PostImport")
        r("POST", r"/index/(?P<index>[^/]+)/field/(?P<field>[^/]+)/import-roaring/(?P<shard>\d+)",
          self.post_import_roaring, "PostImportRoaring")
        r("POST", r"/index/(?P<index>[^/]+)/query", self.post_query, "PostQuery")
        r("GET", r"/info", self.get_info, "GetInfo")
        r("POST", r"/recalculate-caches", self.post_recalculate, "RecalculateCaches")
        r("GET", r"/schema", self.get_schema, "GetSchema")
        r("POST", r"/schema", self.post_schema, "PostSchema")
        r("GET", r"/status", self.get_status, "GetStatus")
        r("GET", r"/version", self.get_version, "GetVersion")
        r("POST", r"/internal/cluster/message", self.post_cluster_message, "PostClusterMessage")
        r("POST", r"/internal/probe", self.post_probe, "PostProbe")
        r("GET", r"/internal/fragment/block/data", self.get_fragment_block_data, "GetFragmentBlockData")
        r("GET", r"/internal/fragment/blocks", self.get_fragment_blocks, "GetFragmentBlocks")
        r("GET", r"/internal/fragment/data", self.get_fragment_data, "GetFragmentData")
        r("GET", r"/internal/fragment/nodes", self.get_fragment_nodes, "GetFragmentNodes")
        r("POST", r"/internal/index/(?P<index>[^/]+)/attr/diff", self.post_index_attr_diff, "PostIndexAttrDiff")
        r("POST", r"/internal/index/(?P<index>[^/]+)/field/(?P<field>[^/]+)/attr/diff", self.post_field_attr_diff,
          "PostFieldAttrDiff")
        r("DELETE", r"/internal/index/(?P<index>[^/]+)/field/(?P<field>[^/]+)/remote-available-shards/"
          r"(?P<shard>\d+)", self.delete_remote_available_shard, "DeleteRemoteAvailableShard")
        r("GET", r"/internal/nodes", self.get_nodes, "GetNodes")
        r("GET", r"/internal/shards/max", self.get_shards_max, "GetShardsMax")
        r("GET", r"/internal/translate/data", self.get_translate_data, "GetTranslateData")
        r("POST", r"/internal/translate/keys", self.post_translate_keys, "PostTranslateKeys")

    def _route(self, method, pattern, fn, name):
        self.routes.append((method, re.compile("^" + pattern + "$"), fn, name))

    # ------------------------------------------------------------ dispatch
    def dispatch(self, req: "Request"):
        path_ok = False
        for method, pat, fn, name in self.routes:
            m = pat.match(req.path)
            if not m:
                continue
            path_ok = True
            if method != req.method:
                continue
            req.vars = m.groupdict()
            self._validate_args(name, req)
            t0 = time.perf_counter()
            with tracing.remote_parent(req.headers):
                with tracing.span(f"HTTP.{name}"):
                    fn(req)
            dt = time.perf_counter() - t0
            if self.stats is not None:
                self.stats.with_tags(f"path:{req.path}", f"method:{req.method}").timing("http.request", dt)
            lq = getattr(self.server, "long_query_time", 0) if self.server is not None else 0
            if lq and dt > lq and self.logger is not None:
                self.logger.printf("%s %s %.3fs", req.method, req.path, dt)
            return
        if path_ok:
            raise HTTPError(405, "method not allowed")
        raise HTTPError(404, "404 page not found")

    @staticmethod
    def _validate_args(name, req):
        spec = VALIDATORS.get(name)
        if spec is None:
            return
        required, optional = spec
        # the reference answers with a JSON error body through http.Error
        # (http/handler.go queryArgValidator)
        for k in required:
            if k not in req.query:
                raise HTTPError(400, gojson.dumps({"error": f"{k} is required"}))
        allowed = set(required) | set(optional)
        for k in req.query:
            if k not in allowed:
                raise HTTPError(400, gojson.dumps({"error": f"{k} is not a valid argument"}))

    # ------------------------------------------------------------ helpers
    @staticmethod
    def _accept_json(req) -> bool:
        acc = req.headers.get("Accept")
        if acc is None:
            return True
        for v in acc.split(","):
            v = v.strip().split(";")[0]
            if v in ("application/json", "*/*", "*/json", "application/*"):
                return True
        return False

    def _require_json(self, req):
        if not self._accept_json(req):
            raise HTTPError(406, "JSON only acceptable response")

    def _success(self, req, err: Optional[Exception] = None):
        if err is None:
            req.send_json({"success": True})
            return
        req.send(_status_for(err), gojson.encode_line({"success": False, "error": {"message": str(err)}}),
                 "text/plain; charset=utf-8")

    # ------------------------------------------------------------ handlers
    def home(self, req):
        req.send(404, "Welcome. Pilosa is running. Visit https://www.pilosa.com/docs/ for more information.\n",
                 "text/plain; charset=utf-8")

    def get_schema(self, req):
        self._require_json(req)
        req.send_json({"indexes": self.api.schema() or None})   # Go: a nil slice encodes as null

    def post_schema(self, req):
        try:
            body = json.loads(req.body or b"{}")
        except ValueError as e:
            raise HTTPError(400, f"decoding request as JSON Pilosa schema: {e}")
        try:
            self.api.apply_schema(body.get("indexes", []), remote=req.query.get("remote") == "true")
        except PilosaError as e:
            raise HTTPError(400, f"apply schema to Pilosa: {e}")
        req.send(204, "", "text/plain")

    def get_status(self, req):
        self._require_json(req)
        req.send_json(self.api.status())

    def get_info(self, req):
        self._require_json(req)
        req.send_json(self.api.info())

    def get_version(self, req):
        self._require_json(req)
        req.send_json({"version": self.api.version()})

    def get_index(self, req):
        self._require_json(req)
        name = req.vars["index"]
        for ii in self.api.schema():
            if ii["name"] == name:
                req.send_json(ii)
                return
        raise HTTPError(404, f"Index {name} Not Found")

    def post_index(self, req):
        self._require_json(req)
        opts = {"keys": False, "trackExistence": True}
        if req.body:
            try:
                body = json.loads(req.body)
            except ValueError as e:
                self._success(req, BadRequestError(e))
                return
            for k, v in body.items():
                if k == "options" and not isinstance(v, dict):
                    self._success(req, BadRequestError("options is not map[string]interface{}"))
                    return
                if k != "options":
                    self._success(req, BadRequestError(f"unknown key: {k}:{_go_fmt(v)}"))
                    return
                for kk, vv in v.items():
                    if kk not in opts:
                        self._success(req, BadRequestError(f"unknown key: {kk}:{_go_fmt(vv)}"))
                        return
                    opts[kk] = vv
        try:
            self.api.create_index(req.vars["index"], keys=bool(opts["keys"]),
                                  track_existence=bool(opts["trackExistence"]))
            self._success(req)
        except PilosaError as e:
            self._success(req, e)

    def delete_index(self, req):
        self._require_json(req)
        try:
            self.api.delete_index(req.vars["index"])
            self._success(req)
        except PilosaError as e:
            self._success(req, e)

    def post_field(self, req):
        self._require_json(req)
        try:
            body = json.loads(req.body) if req.body else {}
            for k in body:
                if k != "options":
                    raise BadRequestError(f'json: unknown field "{k}"')
            o = FieldOptions.from_json(body.get("options", {}))
            if o.type == "int" and "min" not in body.get("options", {}):
                o.min = -(1 << 63)
            if o.type == "int" and "max" not in body.get("options", {}):
                o.max = (1 << 63) - 1
        except (ValueError, PilosaError) as e:
            self._success(req, e if isinstance(e, BadRequestError) else BadRequestError(e))
            return
        try:
            self.api.create_field(req.vars["index"], req.vars["field"], o)
            self._success(req)
        except PilosaError as e:
            self._success(req, e)

    def delete_field(self, req):
        self._require_json(req)
        try:
            self.api.delete_field(req.vars["index"], req.vars["field"])
            self._success(req)
        except PilosaError as e:
            self._success(req, e)

    def post_query(self, req):
        index = req.vars["index"]
        try:
            if req.headers.get("Content-Type") == PROTO:
                m = pb.QueryRequest()
                m.ParseFromString(req.body)
                qr = QueryRequest(index, m.Query, list(m.Shards), m.ColumnAttrs, m.Remote, m.ExcludeRowAttrs,
                                  m.ExcludeColumns)
            else:
                shards = []
                if req.query.get("shards"):
                    try:
                        shards = [int(x) for x in req.query["shards"].split(",") if x]
                    except ValueError:
                        raise BadRequestError("invalid shard argument")
                qr = QueryRequest(index, (req.body or b"").decode(), shards,
                                  req.query.get("columnAttrs") == "true", False,
                                  req.query.get("excludeRowAttrs") == "true",
                                  req.query.get("excludeColumns") == "true")
        except BadRequestError as e:
            self._write_query_error(req, 400, e)
            return
        try:
            resp = self.api.query(qr)
        except PilosaError as e:
            status = 413 if str(cause(e)) == str(ErrTooManyWrites) else 400
            if isinstance(e, APIMethodNotAllowedError):
                status = 405
            self._write_query_error(req, status, e)
            return
        except Exception as e:  # noqa: BLE001
            self._write_query_error(req, 400, e)
            return
        if self._accept_json(req):
            req.send(200, response_json_bytes(resp), JSON)
        else:
            req.send(200, response_to_pb(resp, getattr(resp, "calls", None)), "application/protobuf")

    def _write_query_error(self, req, status, err):
        if self._accept_json(req):
            req.send(status, gojson.encode_line({"error": str(err)}), JSON)
        else:
            req.send(status, pb.QueryResponse(Err=str(err)).SerializeToString(), "application/protobuf")

    def post_import(self, req):
        if req.headers.get("Content-Type") != PROTO:
            raise HTTPError(415, "Unsupported media type")
        if req.headers.get("Accept") != PROTO:
            raise HTTPError(406, "Not acceptable")
        index, field = req.vars["index"], req.vars["field"]
        clear = req.query.get("clear") == "true"
        ignore = req.query.get("ignoreKeyCheck") == "true"
        try:
            f = self.api.field(index, field)
        except PilosaError as e:
            raise HTTPError(404 if isinstance(e, NotFoundError) else 500, str(e))
        try:
            # packed id / value lists decoded natively straight into numpy
            # (native/wire_decode.cpp), not through protobuf repeated fields
            try:
                m = _roaring.decode_import_request(req.body, f.type == "int")
            except (RuntimeError, ValueError) as e:   # ValueError: invalid UTF-8 in a name or key
                raise HTTPError(400, f"decoding request: {e}")
            if f.type == "int":
                self.api.import_values(index, field, m["Shard"], m["ColumnIDs"], m["Values"], m["ColumnKeys"],
                                       clear=clear, ignore_key_check=ignore)
            else:
                self.api.import_bits(index, field, m["Shard"], m["RowIDs"], m["ColumnIDs"], m["RowKeys"],
                                     m["ColumnKeys"], m["Timestamps"], clear=clear, ignore_key_check=ignore)
        except PilosaError as e:
            if str(e) == str(ErrClusterDoesNotOwnShard):
                raise HTTPError(412, str(e))
            raise HTTPError(500, str(e))
        req.send(200, pb.ImportResponse(Err="").SerializeToString(), PROTO)

    def post_import_roaring(self, req):
        index, field, shard = req.vars["index"], req.vars["field"], int(req.vars["shard"])
        m = pb.ImportRoaringRequest()
        try:
            m.ParseFromString(req.body)
        except Exception as e:  # noqa: BLE001
            raise HTTPError(400, f"unmarshal import request: {e}")
        try:
            self.api.import_roaring(index, field, shard, {v.Name: v.Data for v in m.views},
                                    clear=m.Clear or req.query.get("clear") == "true",
                                    remote=req.query.get("remote") == "true")
        except NotFoundError as e:
            raise HTTPError(404, str(e))
        except BadRequestError as e:
            raise HTTPError(400, str(e))
        except PilosaError as e:
            raise HTTPError(500, str(e))
        req.send(200, pb.ImportResponse(Err="").SerializeToString(), PROTO)

    def get_export(self, req):
        if req.headers.get("Accept") != "text/csv":
            raise HTTPError(406, "Not acceptable")
        try:
            shard = int(req.query["shard"])
        except ValueError:
            raise HTTPError(400, "invalid shard")
        import io
        buf = io.StringIO()
        try:
            self.api.export_csv(req.query["index"], req.query["field"], shard, buf)
        except PilosaError as e:
            if str(e) == str(ErrFragmentNotFound):
                req.send(200, "", "text/csv")
                return
            if str(e) == str(ErrClusterDoesNotOwnShard):
                raise HTTPError(412, str(e))
            raise HTTPError(404 if isinstance(e, NotFoundError) else 500, str(e))
        req.send(200, buf.getvalue(), "text/csv")

    def get_fragment_nodes(self, req):
        self._require_json(req)
        try:
            shard = int(req.query["shard"])
        except ValueError:
            raise HTTPError(400, "shard should be an unsigned integer")
        req.send_json([n.to_json() for n in self.api.shard_nodes(req.query["index"], shard)])

    def get_nodes(self, req):
        self._require_json(req)
        req.send_json([n.to_json() for n in self.api.hosts()])

    def get_fragment_block_data(self, req):
        m = pb.BlockDataRequest()
        try:
            if req.body:
                m.ParseFromString(req.body)
            else:
                q = req.query
                m.Index, m.Field, m.View = q.get("index", ""), q.get("field", ""), q.get("view", "")
                m.Shard, m.Block = int(q.get("shard", 0)), int(q.get("block", 0))
        except Exception as e:  # noqa: BLE001
            raise HTTPError(400, str(e))
        try:
            rows, cols = self.api.fragment_block_data(m.Index, m.Field, m.View or "standard", m.Shard, m.Block)
        except PilosaError as e:
            raise HTTPError(404 if str(e) == str(ErrFragmentNotFound) else 500, str(e))
        out = pb.BlockDataResponse(RowIDs=[int(x) for x in rows], ColumnIDs=[int(x) for x in cols])
        req.send(200, out.SerializeToString(), "application/protobuf")

    def get_fragment_blocks(self, req):
        self._require_json(req)
        q = req.query
        try:
            shard = int(q["shard"])
        except ValueError:
            raise HTTPError(400, "shard required")
        try:
            blocks = self.api.fragment_blocks(q["index"], q["field"], q["view"], shard)
        except PilosaError as e:
            raise HTTPError(404 if str(e) == str(ErrFragmentNotFound) else 500, str(e))
        req.send_json({"blocks": blocks})

    def get_fragment_data(self, req):
        q = req.query
        try:
            shard = int(q["shard"])
        except ValueError:
            raise HTTPError(400, "shard required")
        try:
            data = self.api.fragment_data(q["index"], q["field"], q["view"], shard)
        except PilosaError as e:
            raise HTTPError(404, str(e))
        req.send(200, data, "application/octet-stream")

    def get_shards_max(self, req):
        self._require_json(req)
        req.send_json({"standard": self.api.max_shards()})

    def post_recalculate(self, req):
        self.api.recalculate_caches()
        req.send(204, "", "text/plain")

    def post_probe(self, req):
        """Indirect liveness probe for a peer's failure detector
        (parallel/swim.py): probe ``uri`` within ``timeout`` seconds and say
        whether it answered (memberlist's indirect ping)."""
        try:
            body = json.loads(req.body or b"{}")
            uri, timeout = str(body["uri"]), float(body.get("timeout", 0.5))
        except (ValueError, KeyError, TypeError) as e:
            raise HTTPError(400, f"probe request: {e}")
        srv = self.server
        ok = srv.probe_for_peer(uri, timeout) if srv is not None else False
        if ok is None:
            raise HTTPError(400, "probe request: uri is not a member of this cluster")
        req.send_json({"ok": bool(ok)})

    def post_cluster_message(self, req):
        """Type byte + protobuf body (http/handler.go:1474); a JSON body is
        also taken, for tooling.  Failures are 400s, as in the reference."""
        from pilosa_amd.wire import messages
        ctype = (req.headers.get("Content-Type") or "").split(";")[0].strip()
        try:
            if ctype == messages.CONTENT_TYPE:
                msg = messages.decode(req.body)
            elif ctype == "application/json":
                msg = json.loads(req.body)
            else:
                raise HTTPError(415, "Unsupported media type")
        except ValueError as e:
            raise HTTPError(400, str(e))
        try:
            self.api.cluster_message(msg)
        except (PilosaError, KeyError, ValueError) as e:
            raise HTTPError(400, str(e))
        req.send_json({})

    def get_translate_data(self, req):
        try:
            off = int(req.query.get("offset", "0"))
        except ValueError:
            raise HTTPError(400, "invalid offset")
        req.send(200, self.api.translate_data(off), "application/octet-stream")

    def post_translate_keys(self, req):
        m = pb.TranslateKeysRequest()
        m.ParseFromString(req.body)
        ids = self.api.translate_keys(m.Index, m.Field, list(m.Keys))
        req.send(200, pb.TranslateKeysResponse(IDs=ids).SerializeToString(), PROTO)

    def _attr_diff(self, req, store):
        try:
            body = json.loads(req.body)
        except ValueError as e:
            raise HTTPError(400, str(e))
        # attrBlocks checksums are Go []byte: base64 in JSON (attr.go:80-83)
        try:
            theirs = {int(b["id"]): base64.b64decode(b.get("checksum") or "") for b in body.get("blocks", [])}
        except (ValueError, TypeError, KeyError) as e:
            raise HTTPError(400, str(e))
        out = {}
        for bid, chk in store.blocks():
            if theirs.get(bid) != chk:
                for i, a in store.block_data(bid).items():
                    out[str(i)] = dict(sorted(a.items()))   # a Go map encodes with sorted keys
        req.send_json({"attrs": out})

    def post_index_attr_diff(self, req):
        idx = self.api.holder.index(req.vars["index"])
        if idx is None:
            raise HTTPError(404, str(ErrIndexNotFound))
        self._attr_diff(req, idx.column_attr_store)

    def post_field_attr_diff(self, req):
        f = self.api.holder.field(req.vars["index"], req.vars["field"])
        if f is None:
            raise HTTPError(404, str(ErrFieldNotFound))
        self._attr_diff(req, f.row_attr_store)

    def delete_remote_available_shard(self, req):
        try:
            self.api.delete_available_shard(req.vars["index"], req.vars["field"], int(req.vars["shard"]), remote=True)
            self._success(req)
        except PilosaError as e:
            self._success(req, e)

    def post_resize_abort(self, req):
        # http/handler.go handlePostClusterResizeAbort: not the coordinator ->
        # 400, no job running -> 200 with the message, anything else (the
        # method is not allowed in this cluster state) -> 500
        self._require_json(req)
        try:
            self.api.resize_abort()
            req.send_json({"info": ""})
        except PilosaError as e:
            if e is ErrNodeNotCoordinator:
                raise HTTPError(400, str(e))
            if e is ErrResizeNotRunning:
                req.send_json({"info": str(e)})
                return
            raise HTTPError(500, str(e))

    def post_remove_node(self, req):
        try:
            body = json.loads(req.body)
            node_id = body["id"]
        except (KeyError, ValueError, TypeError) as e:
            req.send(400, str(e) + "\n", "text/plain; charset=utf-8")
            return
        try:
            n = self.api.remove_node(node_id)
        except NotFoundError as e:
            req.send(404, f"removing node: {e}\n", "text/plain; charset=utf-8")
            return
        except PilosaError as e:
            req.send(500, f"removing node: {e}\n", "text/plain; charset=utf-8")
            return
        req.send_json({"remove": n.to_json()})

    def post_set_coordinator(self, req):
        try:
            body = json.loads(req.body)
            old, new = self.api.set_coordinator(body["id"])
            req.send_json({"old": old.to_json() if old else None, "new": new.to_json()})
        except (PilosaError, KeyError, ValueError) as e:
            req.send(400, gojson.encode_line({"error": str(e)}), JSON)

    def debug_vars(self, req):
        st = self.stats
        req.send_json(st.expvar() if hasattr(st, "expvar") else {})

    def metrics(self, req):
        st = self.stats
        req.send(200, st.prometheus() if hasattr(st, "prometheus") else "", "text/plain; version=0.0.4")

    def debug_traces(self, req):
        t = tracing.global_tracer()
        tid = req.query.get("trace")
        if tid and hasattr(t, "tree"):
            req.send_json(t.tree(tid, wait=False))   # one trace as a span tree
            return
        spans = getattr(t, "spans", [])
        req.send_json([s.to_dict(wait=False) for s in spans[-1000:]])

    def debug_pprof(self, req):
        from pilosa_amd.utils import pprof
        try:
            body = pprof.render(req.vars.get("rest", ""), {k: v for k, v in req.query.items()})
        except KeyError:
            req.send(404, "Unknown profile\n", "text/plain; charset=utf-8")
            return
        except ValueError as e:
            req.send(400, f"{e}\n", "text/plain; charset=utf-8")
            return
        req.send(200, body, "text/plain; charset=utf-8")


class Request:
    __slots__ = ("method", "path", "query", "headers", "body", "vars", "_h", "sent", "cors")

    def __init__(self, h: BaseHTTPRequestHandler, method: str):
        u = urlparse(h.path)
        self.method = method
        self.path = u.path.rstrip("/") or "/"
        self.query = {k: v[-1] for k, v in parse_qs(u.query, keep_blank_values=True).items()}
        self.headers = h.headers
        n = int(h.headers.get("Content-Length") or 0)
        self.body = h.rfile.read(n) if n else b""
        self.vars = {}
        self._h = h
        self.sent = False
        self.cors = ""     # the allowed Origin echoed back (CORS), else ""

    def send(self, status: int, body, ctype: str, extra: Tuple = ()):
        if isinstance(body, str):
            body = body.encode()
        h = self._h
        h.send_response(status)
        if ctype:
            h.send_header("Content-Type", ctype)
        h.send_header("Content-Length", str(len(body)))
        if self.cors:
            h.send_header("Access-Control-Allow-Origin", self.cors)
            h.send_header("Vary", "Origin")
        for k, v in extra:
            h.send_header(k, v)
        h.end_headers()
        if body:
            h.wfile.write(body)
        self.sent = True

    def send_json(self, obj, status: int = 200):
        self.send(status, gojson.encode_line(obj), JSON)


def make_http_server(handler: Handler, bind: str) -> ThreadingHTTPServer:
    host, _, port = bind.rpartition(":")
    host = host or "0.0.0.0"

    class _H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"
        # headers and body go out as separate writes; without TCP_NODELAY the
        # body waits for the peer's delayed ACK of the headers (~40 ms per
        # keep-alive request)
        disable_nagle_algorithm = True

        def log_message(self, fmt, *args):  # quiet
            pass

        def _do(self, method):
            req = None
            try:
                req = Request(self, method)
                origin = self.headers.get("Origin")
                if origin and origin in handler.allowed_origins:
                    req.cors = origin
                    want = self.headers.get("Access-Control-Request-Method")
                    if method == "OPTIONS" and want:   # CORS preflight
                        req.send(200, b"", "", (("Access-Control-Allow-Methods", want),
                                                ("Access-Control-Allow-Headers", "Content-Type")))
                        return
                handler.dispatch(req)
            except HTTPError as e:
                if req is not None and not req.sent:
                    req.send(e.status, str(e) + "\n", "text/plain; charset=utf-8")
            except Exception as e:  # noqa: BLE001 - panic recovery (handler.go:323)
                msg = f"PANIC: {e}\n{traceback.format_exc()}"
                if handler.logger is not None:
                    handler.logger.printf("%s", msg)
                if req is not None and not req.sent:
                    req.send(500, msg, "text/plain; charset=utf-8")

        def do_GET(self):
            self._do("GET")

        def do_POST(self):
            self._do("POST")

        def do_DELETE(self):
            self._do("DELETE")

        def do_PATCH(self):
            self._do("PATCH")

        def do_OPTIONS(self):
            self._do("OPTIONS")   # preflight for an allowed origin, else 405 / 404 from the routes

    class _Srv(ThreadingHTTPServer):
        # listen backlog (socketserver's default of 5 drops SYNs under
        # 100+ concurrent clients)
        request_queue_size = 1024

        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            self._conns = set()
            self._conns_mu = threading.Lock()

        def process_request(self, request, client_address):
            with self._conns_mu:
                self._conns.add(request)
            super().process_request(request, client_address)

        def shutdown_request(self, request):
            with self._conns_mu:
                self._conns.discard(request)
            super().shutdown_request(request)

        def server_close(self):
            # a closed node must not keep answering on keep-alive connections
            super().server_close()
            with self._conns_mu:
                conns, self._conns = list(self._conns), set()
            for c in conns:
                try:
                    c.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass

    srv = _Srv((host, int(port)), _H)
    srv.daemon_threads = True
    return srv


def _go_fmt(v) -> str:
    """Go's %v of a decoded JSON value (the reference's error texts embed it)."""
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_fmt(x)}" for k, x in sorted(v.items())) + "]"
    if isinstance(v, list):
        return "[" + " ".join(_go_fmt(x) for x in v) + "]"
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return "<nil>"
    return str(v)
