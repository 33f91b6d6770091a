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


def _build_schema(fname: str, messages: dict, service: str, methods: list):
    """Messages: name -> [(field, number, type, repeated?, message type name?)]."""
    fd = descriptor_pb2.FileDescriptorProto(name=fname, syntax="proto3")
    for name, fields in messages.items():
        m = fd.message_type.add(name=name)
        for f in fields:
            fname_, num, ftype = f[:3]
            rep = len(f) > 3 and f[3]
            fld = m.field.add(name=fname_, number=num, type=ftype,
                              label=_F.LABEL_REPEATED if rep else _F.LABEL_OPTIONAL)
            if len(f) > 4:
                fld.type_name = f".{f[4]}"
    svc = fd.service.add(name=service)
    for meth, req, resp in methods:
        svc.method.add(name=meth, input_type=f".{req}", output_type=f".{resp}")
    pool = descriptor_pool.DescriptorPool()   # one pool per schema: both define Request / Model
    pool.Add(fd)
    return {name: message_factory.GetMessageClass(pool.FindMessageTypeByName(name)) for name in messages}


def _build():
    return _build_schema("garfield_amd_garfield.proto", _MESSAGES, SERVICE, METHODS)


_CLASSES = _build()
Request = _CLASSES["Request"]
Response = _CLASSES["Response"]
Model = _CLASSES["Model"]
Gradients = _CLASSES["Gradients"]
CLASSES = _CLASSES

# --------------------------------------------------------------------------------------
# Legacy schema (reference tensorflow_impl/applications/Garfield_legacy/all.proto:5-65):
# service TrainMessageExchange, served next to MessageExchange by every node (legacy.proto)

_LEGACY_MESSAGES = {
    "Empty": [],
    "Request": [("iter", 1, _F.TYPE_INT32), ("req_id", 2, _F.TYPE_INT32)],
    "PublicKey": [("index", 1, _F.TYPE_INT32), ("pubKey", 2, _F.TYPE_BYTES)],
    "Model": [("model", 1, _F.TYPE_BYTES), ("init", 2, _F.TYPE_BOOL), ("iter", 3, _F.TYPE_INT32)],
    "Signature": [("init", 1, _F.TYPE_BOOL), ("signature", 2, _F.TYPE_BYTES), ("index", 3, _F.TYPE_INT32)],
    "CompleteModel": [("inputs", 1, _F.TYPE_BYTES), ("labels", 2, _F.TYPE_BYTES),
                      ("model", 3, _F.TYPE_MESSAGE, False, "Model"), ("iter", 4, _F.TYPE_INT32),
                      ("correctProc", 5, _F.TYPE_INT32, True), ("signatures", 6, _F.TYPE_BYTES, True),
                      ("msgHash", 7, _F.TYPE_BYTES)],
    "GradHashes": [("gradHash", 1, _F.TYPE_STRING, True), ("iter", 2, _F.TYPE_INT32)],
    "GradHash": [("index", 1, _F.TYPE_INT32), ("g_hash", 2, _F.TYPE_BYTES), ("iter", 3, _F.TYPE_INT32)],
    "Gradients": [("gradients", 1, _F.TYPE_BYTES), ("iter", 2, _F.TYPE_FLOAT), ("lipschitz", 3, _F.TYPE_FLOAT)],
}
LEGACY_METHODS = [("GetPublicKey", "Empty", "PublicKey"), ("GetUnifiedModel", "Empty", "Model"),
                  ("GetCompleteModel", "Request", "CompleteModel"), ("GetOnlyHash", "Request", "CompleteModel"),
                  ("GetGradHashes", "Request", "GradHashes"), ("GetGradHash", "Request", "GradHash"),
                  ("GetGradients", "Request", "Gradients"), ("GetModel", "Request", "Model")]
LEGACY_SERVICE = "TrainMessageExchange"
LEGACY = _build_schema("garfield_amd_all.proto", _LEGACY_MESSAGES, LEGACY_SERVICE, LEGACY_METHODS)
