"""`recommender.recommender` gRPC API, built at runtime from descriptors.

Wire-identical to the reference's proto (reference pkg/recommender/protos/recom.proto:1-17):

    package recommender;
    service recommender {
      rpc ImputeConfigurations (Request) returns (Reply);
      rpc ImputeInterference (Request) returns (Reply);
    }
    message Request { string index = 1; }
    message Reply   { repeated float result = 1; repeated string columns = 2; }

`grpc_tools`/protoc are not installed, so instead of generated `recom_pb2*.py` stubs the
FileDescriptorProto is assembled here and message classes come from the descriptor pool.
A second service, `gpusched.recommender.Extended`, adds what the MI355X build needs
(bulk table export for the in-process prediction cache, resource-resize advice, model
version, co-run observations for online interference learning, co-run groups for the online
co-run model) without touching the
reference API.
"""
from __future__ import annotations

from typing import Any, Callable, Dict

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from ..utils.protodesc import F as _F, field as _field


def _build_pool() -> descriptor_pool.DescriptorPool:
    pool = descriptor_pool.DescriptorPool()
    # ---- reference-compatible file --------------------------------------------------
    fd = descriptor_pb2.FileDescriptorProto(name="recom.proto", package="recommender", syntax="proto3")
    req = fd.message_type.add(name="Request")
    _field(req, "index", 1, _F.TYPE_STRING)
    rep = fd.message_type.add(name="Reply")
    _field(rep, "result", 1, _F.TYPE_FLOAT, _F.LABEL_REPEATED)
    _field(rep, "columns", 2, _F.TYPE_STRING, _F.LABEL_REPEATED)
    svc = fd.service.add(name="recommender")
    for m in ("ImputeConfigurations", "ImputeInterference"):
        svc.method.add(name=m, input_type=".recommender.Request", output_type=".recommender.Reply")
    pool.Add(fd)
    # ---- extension file ---------------------------------------------------------------
    fx = descriptor_pb2.FileDescriptorProto(name="gpusched_recommender.proto",
                                            package="gpusched.recommender", syntax="proto3")
    fx.dependency.append("recom.proto")
    tbl = fx.message_type.add(name="TableRequest")
    _field(tbl, "table", 1, _F.TYPE_STRING)            # "configurations" | "interference"
    row = fx.message_type.add(name="Row")
    _field(row, "index", 1, _F.TYPE_STRING)
    _field(row, "values", 2, _F.TYPE_FLOAT, _F.LABEL_REPEATED)
    tab = fx.message_type.add(name="Table")
    _field(tab, "columns", 1, _F.TYPE_STRING, _F.LABEL_REPEATED)
    _field(tab, "rows", 2, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, ".gpusched.recommender.Row")
    _field(tab, "version", 3, _F.TYPE_STRING)
    rz = fx.message_type.add(name="ResizeRequest")
    _field(rz, "pod", 1, _F.TYPE_STRING)
    _field(rz, "requested_cu", 2, _F.TYPE_INT32)
    _field(rz, "requested_hbm_gib", 3, _F.TYPE_FLOAT)
    _field(rz, "slo", 4, _F.TYPE_FLOAT)
    rzr = fx.message_type.add(name="ResizeReply")
    _field(rzr, "recommended_cu", 1, _F.TYPE_INT32)
    _field(rzr, "recommended_hbm_gib", 2, _F.TYPE_FLOAT)
    _field(rzr, "samples", 3, _F.TYPE_INT32)
    _field(rzr, "reason", 4, _F.TYPE_STRING)
    ver = fx.message_type.add(name="VersionReply")
    _field(ver, "configurations", 1, _F.TYPE_STRING)
    _field(ver, "interference", 2, _F.TYPE_STRING)
    _field(ver, "model", 3, _F.TYPE_STRING)
    _field(ver, "corun", 4, _F.TYPE_STRING)              # co-run model version served
    emp = fx.message_type.add(name="Empty")
    del emp
    cr = fx.message_type.add(name="CoRun")                # one pod's co-run observation
    _field(cr, "pod", 1, _F.TYPE_STRING)                 # pod (or workload) name
    _field(cr, "co_runners", 2, _F.TYPE_STRING, _F.LABEL_REPEATED)
    _field(cr, "loss", 3, _F.TYPE_FLOAT)                 # predicted-alone minus achieved throughput
    orq = fx.message_type.add(name="ObserveRequest")
    _field(orq, "observations", 1, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, ".gpusched.recommender.CoRun")
    orp = fx.message_type.add(name="ObserveReply")
    _field(orp, "accepted", 1, _F.TYPE_INT32)
    _field(orp, "interference", 2, _F.TYPE_STRING)       # interference table version now served
    _field(orp, "observations", 3, _F.TYPE_INT32)        # total learned so far
    cg = fx.message_type.add(name="CorunGroup")          # one GPU's co-running pods (models.corun)
    _field(cg, "workloads", 1, _F.TYPE_STRING, _F.LABEL_REPEATED)     # pod or workload names
    _field(cg, "iters", 2, _F.TYPE_FLOAT, _F.LABEL_REPEATED)
    _field(cg, "start_ms", 3, _F.TYPE_FLOAT, _F.LABEL_REPEATED)       # start offsets in the group
    _field(cg, "ms", 4, _F.TYPE_FLOAT, _F.LABEL_REPEATED)             # measured wall ms
    _field(cg, "target", 5, _F.TYPE_BOOL, _F.LABEL_REPEATED)          # observation (else co-runner only)
    _field(cg, "mfma_share", 6, _F.TYPE_FLOAT, _F.LABEL_REPEATED)     # MFMA share of kernel time (-1 unknown)
    _field(cg, "cu_fill", 7, _F.TYPE_FLOAT, _F.LABEL_REPEATED)        # CU fill of its kernels (-1 unknown)
    ocq = fx.message_type.add(name="ObserveCorunRequest")
    _field(ocq, "groups", 1, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, ".gpusched.recommender.CorunGroup")
    ocp = fx.message_type.add(name="ObserveCorunReply")
    _field(ocp, "accepted", 1, _F.TYPE_INT32)
    _field(ocp, "corun", 2, _F.TYPE_STRING)              # co-run model version now served
    _field(ocp, "observations", 3, _F.TYPE_INT32)
    s2 = fx.service.add(name="Extended")
    s2.method.add(name="ExportTable", input_type=".gpusched.recommender.TableRequest",
                  output_type=".gpusched.recommender.Table")
    s2.method.add(name="RecommendResources", input_type=".gpusched.recommender.ResizeRequest",
                  output_type=".gpusched.recommender.ResizeReply")
    s2.method.add(name="Version", input_type=".gpusched.recommender.Empty",
                  output_type=".gpusched.recommender.VersionReply")
    s2.method.add(name="ObserveInterference", input_type=".gpusched.recommender.ObserveRequest",
                  output_type=".gpusched.recommender.ObserveReply")
    s2.method.add(name="ObserveCorun", input_type=".gpusched.recommender.ObserveCorunRequest",
                  output_type=".gpusched.recommender.ObserveCorunReply")
    pool.Add(fx)
    return pool


POOL = _build_pool()


def _cls(full_name: str) -> Any:
    return message_factory.GetMessageClass(POOL.FindMessageTypeByName(full_name))


Request = _cls("recommender.Request")
Reply = _cls("recommender.Reply")
TableRequest = _cls("gpusched.recommender.TableRequest")
Row = _cls("gpusched.recommender.Row")
Table = _cls("gpusched.recommender.Table")
ResizeRequest = _cls("gpusched.recommender.ResizeRequest")
ResizeReply = _cls("gpusched.recommender.ResizeReply")
VersionReply = _cls("gpusched.recommender.VersionReply")
Empty = _cls("gpusched.recommender.Empty")
CoRun = _cls("gpusched.recommender.CoRun")
ObserveRequest = _cls("gpusched.recommender.ObserveRequest")
ObserveReply = _cls("gpusched.recommender.ObserveReply")
CorunGroup = _cls("gpusched.recommender.CorunGroup")
ObserveCorunRequest = _cls("gpusched.recommender.ObserveCorunRequest")
ObserveCorunReply = _cls("gpusched.recommender.ObserveCorunReply")

SERVICE = "recommender.recommender"
EXT_SERVICE = "gpusched.recommender.Extended"
METHODS: Dict[str, Any] = {
    f"/{SERVICE}/ImputeConfigurations": (Request, Reply),
    f"/{SERVICE}/ImputeInterference": (Request, Reply),
    f"/{EXT_SERVICE}/ExportTable": (TableRequest, Table),
    f"/{EXT_SERVICE}/RecommendResources": (ResizeRequest, ResizeReply),
    f"/{EXT_SERVICE}/Version": (Empty, VersionReply),
    f"/{EXT_SERVICE}/ObserveInterference": (ObserveRequest, ObserveReply),
    f"/{EXT_SERVICE}/ObserveCorun": (ObserveCorunRequest, ObserveCorunReply),
}


def set_protobuf_reply(data: Any, columns: Any, reply: Any) -> Any:
    """Same contract as reference pkg/recommender/utils.py:37-42."""
    for v in data:
        reply.result.append(float(v))
    for c in columns:
        reply.columns.append(str(c))
    return reply


def generic_handler(service: str, impls: Dict[str, Callable[[Any, Any], Any]]) -> grpc.GenericRpcHandler:
    handlers = {}
    for meth, fn in impls.items():
        req_cls, rep_cls = METHODS[f"/{service}/{meth}"]
        handlers[meth] = grpc.unary_unary_rpc_method_handler(
            fn, request_deserializer=req_cls.FromString, response_serializer=rep_cls.SerializeToString)
    return grpc.method_handlers_generic_handler(service, handlers)


def stub_method(channel: grpc.Channel, full_method: str) -> Callable[..., Any]:
    req_cls, rep_cls = METHODS[full_method]
    return channel.unary_unary(full_method, request_serializer=req_cls.SerializeToString,
                               response_deserializer=rep_cls.FromString)
