"""``home_native.v1`` protobuf messages and the ``Inference`` gRPC service.

Wire-identical to the reference contract (src/lumen/proto/ml_service.proto:1-88;
5 byte-identical copies across the reference packages): same package, message
names, field numbers and types, the same service and method paths
(``/home_native.v1.Inference/{Infer,GetCapabilities,StreamCapabilities,Health}``).

There is no ``protoc`` / grpc_tools in this image, so the file descriptor is
assembled in code with ``descriptor_pb2`` and registered in the default pool;
message classes come from the protobuf message factory, and the gRPC glue
(servicer base, ``add_InferenceServicer_to_server``, ``InferenceStub``) is
written against grpcio's generic-handler API.
"""
from __future__ import annotations

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, empty_pb2, message_factory

PACKAGE = "home_native.v1"
FILE_NAME = "ml_service.proto"
SERVICE = f"{PACKAGE}.Inference"

_F = descriptor_pb2.FieldDescriptorProto


def _field(msg, name, number, ftype, label=_F.LABEL_OPTIONAL, type_name=None):
    f = msg.field.add()
    f.name, f.number, f.type, f.label = name, number, ftype, label
    f.json_name = "".join(w.capitalize() if i else w for i, w in enumerate(name.split("_")))
    if type_name:
        f.type_name = type_name
    return f


def _map(msg, name, number):
    """map<string, string> field -> nested XxxEntry message with map_entry option."""
    entry_name = "".join(w.capitalize() for w in name.split("_")) + "Entry"
    e = msg.nested_type.add()
    e.name = entry_name
    e.options.map_entry = True
    _field(e, "key", 1, _F.TYPE_STRING)
    _field(e, "value", 2, _F.TYPE_STRING)
    _field(msg, name, number, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, f".{PACKAGE}.{msg.name}.{entry_name}")


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = FILE_NAME
    fd.package = PACKAGE
    fd.syntax = "proto3"
    fd.dependency.append("google/protobuf/empty.proto")
    fd.options.go_package = "server/proto"

    en = fd.enum_type.add()
    en.name = "ErrorCode"
    for i, n in enumerate(["ERROR_CODE_UNSPECIFIED", "ERROR_CODE_INVALID_ARGUMENT", "ERROR_CODE_UNAVAILABLE",
                           "ERROR_CODE_DEADLINE_EXCEEDED", "ERROR_CODE_INTERNAL"]):
        v = en.value.add()
        v.name, v.number = n, i

    err = fd.message_type.add()
    err.name = "Error"
    _field(err, "code", 1, _F.TYPE_ENUM, type_name=f".{PACKAGE}.ErrorCode")
    _field(err, "message", 2, _F.TYPE_STRING)
    _field(err, "detail", 3, _F.TYPE_STRING)

    io = fd.message_type.add()
    io.name = "IOTask"
    _field(io, "name", 1, _F.TYPE_STRING)
    _field(io, "input_mimes", 2, _F.TYPE_STRING, _F.LABEL_REPEATED)
    _field(io, "output_mimes", 3, _F.TYPE_STRING, _F.LABEL_REPEATED)
    _map(io, "limits", 4)

    cap = fd.message_type.add()
    cap.name = "Capability"
    _field(cap, "service_name", 1, _F.TYPE_STRING)
    _field(cap, "model_ids", 2, _F.TYPE_STRING, _F.LABEL_REPEATED)
    _field(cap, "runtime", 3, _F.TYPE_STRING)
    _field(cap, "max_concurrency", 4, _F.TYPE_UINT32)
    _field(cap, "precisions", 5, _F.TYPE_STRING, _F.LABEL_REPEATED)
    _map(cap, "extra", 6)
    _field(cap, "tasks", 7, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, f".{PACKAGE}.IOTask")
    _field(cap, "protocol_version", 8, _F.TYPE_STRING)

    req = fd.message_type.add()
    req.name = "InferRequest"
    _field(req, "correlation_id", 1, _F.TYPE_STRING)
    _field(req, "task", 2, _F.TYPE_STRING)
    _field(req, "payload", 3, _F.TYPE_BYTES)
    _map(req, "meta", 4)
    _field(req, "payload_mime", 5, _F.TYPE_STRING)
    _field(req, "seq", 6, _F.TYPE_UINT64)
    _field(req, "total", 7, _F.TYPE_UINT64)
    _field(req, "offset", 8, _F.TYPE_UINT64)

    rsp = fd.message_type.add()
    rsp.name = "InferResponse"
    _field(rsp, "correlation_id", 1, _F.TYPE_STRING)
    _field(rsp, "is_final", 2, _F.TYPE_BOOL)
    _field(rsp, "result", 3, _F.TYPE_BYTES)
    _map(rsp, "meta", 4)
    _field(rsp, "error", 5, _F.TYPE_MESSAGE, type_name=f".{PACKAGE}.Error")
    _field(rsp, "seq", 6, _F.TYPE_UINT64)
    _field(rsp, "total", 7, _F.TYPE_UINT64)
    _field(rsp, "offset", 8, _F.TYPE_UINT64)
    _field(rsp, "result_mime", 9, _F.TYPE_STRING)
    _field(rsp, "result_schema", 10, _F.TYPE_STRING)

    svc = fd.service.add()
    svc.name = "Inference"
    for name, it, ot, cs, ss in [("Infer", "InferRequest", "InferResponse", True, True),
                                 ("GetCapabilities", ".google.protobuf.Empty", "Capability", False, False),
                                 ("StreamCapabilities", ".google.protobuf.Empty", "Capability", False, True),
                                 ("Health", ".google.protobuf.Empty", ".google.protobuf.Empty", False, False)]:
        m = svc.method.add()
        m.name = name
        m.input_type = it if it.startswith(".") else f".{PACKAGE}.{it}"
        m.output_type = ot if ot.startswith(".") else f".{PACKAGE}.{ot}"
        m.client_streaming, m.server_streaming = cs, ss
    return fd


def _register():
    pool = descriptor_pool.Default()
    try:
        return pool.FindFileByName(FILE_NAME)
    except KeyError:
        pass
    _ = empty_pb2.DESCRIPTOR  # make sure google/protobuf/empty.proto is in the pool
    return pool.AddSerializedFile(_build_file().SerializeToString())


DESCRIPTOR = _register()


def _cls(name):
    return message_factory.GetMessageClass(DESCRIPTOR.message_types_by_name[name])


Error = _cls("Error")
IOTask = _cls("IOTask")
Capability = _cls("Capability")
InferRequest = _cls("InferRequest")
InferResponse = _cls("InferResponse")
Empty = empty_pb2.Empty

_ec = DESCRIPTOR.enum_types_by_name["ErrorCode"]
ERROR_CODE_UNSPECIFIED = _ec.values_by_name["ERROR_CODE_UNSPECIFIED"].number
ERROR_CODE_INVALID_ARGUMENT = _ec.values_by_name["ERROR_CODE_INVALID_ARGUMENT"].number
ERROR_CODE_UNAVAILABLE = _ec.values_by_name["ERROR_CODE_UNAVAILABLE"].number
ERROR_CODE_DEADLINE_EXCEEDED = _ec.values_by_name["ERROR_CODE_DEADLINE_EXCEEDED"].number
ERROR_CODE_INTERNAL = _ec.values_by_name["ERROR_CODE_INTERNAL"].number


class ErrorCode:
    UNSPECIFIED = ERROR_CODE_UNSPECIFIED
    INVALID_ARGUMENT = ERROR_CODE_INVALID_ARGUMENT
    UNAVAILABLE = ERROR_CODE_UNAVAILABLE
    DEADLINE_EXCEEDED = ERROR_CODE_DEADLINE_EXCEEDED
    INTERNAL = ERROR_CODE_INTERNAL

    @staticmethod
    def Name(v: int) -> str:
        return _ec.values_by_number[v].name


# --------------------------------------------------------------------------- gRPC glue
def _path(method: str) -> str:
    return f"/{SERVICE}/{method}"


class InferenceServicer:
    """Base servicer: every method is UNIMPLEMENTED until overridden."""

    def Infer(self, request_iterator, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")

    def GetCapabilities(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")

    def StreamCapabilities(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")

    def Health(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")


def add_InferenceServicer_to_server(servicer, server) -> None:
    handlers = {
        "Infer": grpc.stream_stream_rpc_method_handler(
            servicer.Infer, request_deserializer=InferRequest.FromString,
            response_serializer=InferResponse.SerializeToString),
        "GetCapabilities": grpc.unary_unary_rpc_method_handler(
            servicer.GetCapabilities, request_deserializer=Empty.FromString,
            response_serializer=Capability.SerializeToString),
        "StreamCapabilities": grpc.unary_stream_rpc_method_handler(
            servicer.StreamCapabilities, request_deserializer=Empty.FromString,
            response_serializer=Capability.SerializeToString),
        "Health": grpc.unary_unary_rpc_method_handler(
            servicer.Health, request_deserializer=Empty.FromString, response_serializer=Empty.SerializeToString),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))


class InferenceStub:
    """Client stub for ``home_native.v1.Inference``."""

    def __init__(self, channel):
        self.Infer = channel.stream_stream(_path("Infer"), request_serializer=InferRequest.SerializeToString,
                                           response_deserializer=InferResponse.FromString)
        self.GetCapabilities = channel.unary_unary(_path("GetCapabilities"), request_serializer=Empty.SerializeToString,
                                                   response_deserializer=Capability.FromString)
        self.StreamCapabilities = channel.unary_stream(_path("StreamCapabilities"),
                                                       request_serializer=Empty.SerializeToString,
                                                       response_deserializer=Capability.FromString)
        self.Health = channel.unary_unary(_path("Health"), request_serializer=Empty.SerializeToString,
                                          response_deserializer=Empty.FromString)


def proto_source() -> str:
    """The equivalent .proto text (for clients that want to regenerate stubs)."""
    from pathlib import Path

    return (Path(__file__).with_name("ml_service.proto")).read_text()
