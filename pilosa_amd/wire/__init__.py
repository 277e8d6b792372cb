"""Protobuf wire format without protoc.

``pilosa.proto`` (same field numbers as the reference's internal/*.proto) is
parsed by a small proto3-subset reader into a ``FileDescriptorProto``; message
classes are then created with ``google.protobuf.message_factory``.  Usage::

    from pilosa_amd.wire import pb
    m = pb.QueryRequest(Query="Count(Row(f=1))", Shards=[0, 1])
    data = m.SerializeToString()
"""
from __future__ import annotations

import os
import re
import types

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_HERE = os.path.dirname(os.path.abspath(__file__))
_SCALARS = {
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "uint32": descriptor_pb2.FieldDescriptorProto.TYPE_UINT32,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
}
_FDP = descriptor_pb2.FieldDescriptorProto


def _parse(text: str, package: str) -> descriptor_pb2.FileDescriptorProto:
    text = re.sub(r"//[^\n]*", "", text)
    fd = descriptor_pb2.FileDescriptorProto(name="pilosa_amd_wire.proto", package=package, syntax="proto3")
    for m in re.finditer(r"message\s+(\w+)\s*\{([^}]*)\}", text):
        name, body = m.group(1), m.group(2)
        msg = fd.message_type.add(name=name)
        for fm in re.finditer(r"(repeated\s+)?(map<\s*(\w+)\s*,\s*(\w+)\s*>|\w+)\s+(\w+)\s*=\s*(\d+)\s*;", body):
            repeated, typ, mk, mv, fname, num = fm.groups()
            f = msg.field.add(name=fname, number=int(num), json_name=fname)
            if typ.startswith("map<"):
                entry = msg.nested_type.add(name=fname[0].upper() + fname[1:] + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=_SCALARS[mk], label=_FDP.LABEL_OPTIONAL)
                vf = entry.field.add(name="value", number=2, label=_FDP.LABEL_OPTIONAL)
                if mv in _SCALARS:
                    vf.type = _SCALARS[mv]
                else:
                    vf.type = _FDP.TYPE_MESSAGE
                    vf.type_name = f".{package}.{mv}"
                f.label = _FDP.LABEL_REPEATED
                f.type = _FDP.TYPE_MESSAGE
                f.type_name = f".{package}.{name}.{entry.name}"
                continue
            f.label = _FDP.LABEL_REPEATED if repeated else _FDP.LABEL_OPTIONAL
            if typ in _SCALARS:
                f.type = _SCALARS[typ]
            else:
                f.type = _FDP.TYPE_MESSAGE
                f.type_name = f".{package}.{typ}"
    return fd


def _load():
    with open(os.path.join(_HERE, "pilosa.proto")) as fh:
        fd = _parse(fh.read(), "internal")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    ns = types.SimpleNamespace()
    for m in fd.message_type:
        desc = pool.FindMessageTypeByName(f"internal.{m.name}")
        setattr(ns, m.name, message_factory.GetMessageClass(desc))
    return ns


pb = _load()

# QueryResult.Type codes (reference encoding/proto/proto.go)
QUERY_RESULT_TYPE_NIL = 0
QUERY_RESULT_TYPE_ROW = 1
QUERY_RESULT_TYPE_PAIRS = 2
QUERY_RESULT_TYPE_VALCOUNT = 3
QUERY_RESULT_TYPE_UINT64 = 4
QUERY_RESULT_TYPE_BOOL = 5
QUERY_RESULT_TYPE_ROWIDS = 6
QUERY_RESULT_TYPE_GROUPCOUNTS = 7
QUERY_RESULT_TYPE_ROWIDENTIFIERS = 8
QUERY_RESULT_TYPE_PAIR = 9

# Attr.Type codes
ATTR_TYPE_STRING = 1
ATTR_TYPE_INT = 2
ATTR_TYPE_BOOL = 3
ATTR_TYPE_FLOAT = 4
