"""gRPC bindings for the ``metisfl`` services without generated ``_pb2_grpc``
modules (there is no protoc in this environment).

Stubs, servicer base classes and ``add_*_to_server`` functions are derived
from the runtime service descriptors (proto/__init__.py), so the method
paths (``/metisfl.ControllerService/JoinFederation`` ...) are exactly the
ones the reference's generated code uses (controller_pb2_grpc.py,
learner_pb2_grpc.py) and the two sides interoperate on the wire.

Besides the typed stub, ``raw_unary`` gives a bytes-in / bytes-out callable:
the controller forwards RunTask / EvaluateModel requests that the native
engine already serialized, so models are never parsed in Python on the hot
control path.
"""
from __future__ import annotations

import types

import grpc
from google.protobuf import message_factory

from metisfl_amd.proto import controller_pb2, learner_pb2


def _cls(desc):
    return message_factory.GetMessageClass(desc)


def _path(service, method) -> str:
    return f"/{service.full_name}/{method.name}"


def make_stub_class(service):
    """Typed client stub: one attribute per RPC, like the generated *Stub."""

    def __init__(self, channel: grpc.Channel):
        for m in service.methods:
            setattr(self, m.name, channel.unary_unary(
                _path(service, m),
                request_serializer=_cls(m.input_type).SerializeToString,
                response_deserializer=_cls(m.output_type).FromString))

    return type(f"{service.name}Stub", (object,), {"__init__": __init__,
                                                    "__doc__": f"Client stub for {service.full_name}."})


def make_servicer_class(service):
    """Servicer base: every RPC answers UNIMPLEMENTED until overridden."""

    def _unimplemented(name):
        def handler(self, request, context):
            context.set_code(grpc.StatusCode.UNIMPLEMENTED)
            context.set_details(f"Method {name} not implemented!")
            raise NotImplementedError(f"Method {name} not implemented!")
        handler.__name__ = name
        return handler

    body = {m.name: _unimplemented(m.name) for m in service.methods}
    body["__doc__"] = f"Servicer base class for {service.full_name}."
    return type(f"{service.name}Servicer", (object,), body)


def make_add_to_server(service):
    def add(servicer, server: grpc.Server, raw_requests=(), raw_responses=()) -> None:
        """``raw_requests``: RPC names whose handler receives the request as
        bytes (large-model RPCs forwarded to the native engine unparsed);
        ``raw_responses``: RPC names whose handler returns serialized bytes."""
        handlers = {}
        for m in service.methods:
            handlers[m.name] = grpc.unary_unary_rpc_method_handler(
                getattr(servicer, m.name),
                request_deserializer=None if m.name in raw_requests else _cls(m.input_type).FromString,
                response_serializer=None if m.name in raw_responses else _cls(m.output_type).SerializeToString)
        server.add_generic_rpc_handlers(
            (grpc.method_handlers_generic_handler(service.full_name, handlers),))
    add.__name__ = f"add_{service.name}Servicer_to_server"
    return add


def raw_unary(channel: grpc.Channel, service, method_name: str):
    """Bytes-in / typed-out callable for ``method_name`` (request already
    serialized by the native engine)."""
    m = service.methods_by_name[method_name]
    return channel.unary_unary(_path(service, m), request_serializer=lambda b: b,
                               response_deserializer=_cls(m.output_type).FromString)


def _varint(buf: bytes, i: int):
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def split_fields(buf: bytes) -> dict:
    """Top-level fields of a serialized message WITHOUT parsing nested
    messages: {field_number: [value, ...]} (length-delimited fields as
    memoryview slices, varints as ints).  Used to peel learner_id /
    auth_token off a MarkTaskCompleted request and hand the embedded task
    (the whole model) to the engine as bytes."""
    out: dict = {}
    mv = memoryview(buf)
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = mv[i:i + ln]
            i += ln
        elif wt == 1:
            v = mv[i:i + 8]
            i += 8
        elif wt == 5:
            v = mv[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.setdefault(field, []).append(v)
    return out


def _namespace(name: str, service) -> types.SimpleNamespace:
    ns = types.SimpleNamespace()
    setattr(ns, f"{service.name}Stub", make_stub_class(service))
    setattr(ns, f"{service.name}Servicer", make_servicer_class(service))
    setattr(ns, f"add_{service.name}Servicer_to_server", make_add_to_server(service))
    ns.SERVICE = service
    ns.__name__ = name
    return ns


CONTROLLER_SERVICE = controller_pb2._CONTROLLERSERVICE
LEARNER_SERVICE = learner_pb2._LEARNERSERVICE

# drop-in namespaces mirroring the generated modules
controller_pb2_grpc = _namespace("controller_pb2_grpc", CONTROLLER_SERVICE)
learner_pb2_grpc = _namespace("learner_pb2_grpc", LEARNER_SERVICE)
