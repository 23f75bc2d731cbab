"""Helpers for protobuf descriptors built at runtime (no protoc in the image): the
recommender's gRPC API (recommender/proto.py) and the kubelet device-plugin API
(agent/deviceplugin.py) are both declared field by field with these."""
from __future__ import annotations

from typing import Any

from google.protobuf import descriptor_pb2

F = descriptor_pb2.FieldDescriptorProto


def field(msg: Any, name: str, num: int, typ: int, label: int = F.LABEL_OPTIONAL, type_name: str = "") -> None:
    """Add field `name` = `num` of type `typ` to message descriptor `msg`."""
    f = msg.field.add()
    f.name, f.number, f.type, f.label = name, num, typ, label
    if type_name:
        f.type_name = type_name


def map_entry(msg: Any, name: str, num: int, package: str) -> None:
    """map<string, string> field `name` = a repeated nested *Entry message (the proto3 map
    encoding), in proto package `package`."""
    entry = msg.nested_type.add(name="".join(p.capitalize() for p in name.split("_")) + "Entry")
    entry.options.map_entry = True
    field(entry, "key", 1, F.TYPE_STRING)
    field(entry, "value", 2, F.TYPE_STRING)
    field(msg, name, num, F.TYPE_MESSAGE, F.LABEL_REPEATED, f".{package}.{msg.name}.{entry.name}")
