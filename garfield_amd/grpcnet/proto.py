"""Protobuf message classes of ``garfield.proto``, built at import time.

No ``grpc_tools``/``protoc`` exists in this image, so the file descriptor is
assembled with ``descriptor_pb2`` and the classes come from the message factory;
the wire format is identical to protoc-generated code (reference
``tensorflow_impl/libs/garfield_pb2.py``)."""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto

_MESSAGES = {
    "Request": [("iter", 1, _F.TYPE_INT32), ("job", 2, _F.TYPE_STRING), ("req_id", 3, _F.TYPE_INT32)],
    "Response": [("iter", 1, _F.TYPE_INT32), ("job", 2, _F.TYPE_STRING), ("req_id", 3, _F.TYPE_INT32)],
    "Model": [("model", 1, _F.TYPE_BYTES), ("init", 2, _F.TYPE_BOOL), ("iter", 3, _F.TYPE_INT32)],
    "Gradients": [("gradients", 1, _F.TYPE_BYTES), ("iter", 2, _F.TYPE_FLOAT)],
}

# (method, request, response)
METHODS = [("GetModel", "Request", "Model"), ("SendModel", "Model", "Response"),
           ("GetGradient", "Request", "Gradients"), ("SendGradient", "Gradients", "Response")]
SERVICE = "MessageExchange"


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="garfield_amd_garfield.proto", syntax="proto3")
    for name, fields in _MESSAGES.items():
        m = fd.message_type.add(name=name)
        for fname, num, ftype in fields:
            m.field.add(name=fname, number=num, type=ftype, label=_F.LABEL_OPTIONAL)
    svc = fd.service.add(name=SERVICE)
    for meth, req, resp in METHODS:
        svc.method.add(name=meth, input_type=f".{req}", output_type=f".{resp}")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {name: message_factory.GetMessageClass(pool.FindMessageTypeByName(name)) for name in _MESSAGES}


_CLASSES = _build()
Request = _CLASSES["Request"]
Response = _CLASSES["Response"]
Model = _CLASSES["Model"]
Gradients = _CLASSES["Gradients"]
CLASSES = _CLASSES
