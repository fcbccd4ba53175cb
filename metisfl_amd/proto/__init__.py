"""``metisfl`` wire-format message classes, built at import time from the
``.proto`` files in ``schema/`` (see loader.py).

Exposes ``model_pb2``, ``metis_pb2``, ``controller_pb2``, ``learner_pb2`` and
``service_common_pb2`` namespaces with the same class names the reference's
generated modules have, e.g. ``model_pb2.Model``, ``metis_pb2.ControllerParams``.
"""
from __future__ import annotations

import sys
import types

from google.protobuf import message_factory

from metisfl_amd.proto import loader

_pool = loader.load()

_FILES = {
    "model_pb2": "metisfl/proto/model.proto",
    "service_common_pb2": "metisfl/proto/service_common.proto",
    "metis_pb2": "metisfl/proto/metis.proto",
    "controller_pb2": "metisfl/proto/controller.proto",
    "learner_pb2": "metisfl/proto/learner.proto",
}


def _make_module(modname: str, filename: str) -> types.ModuleType:
    fd = _pool.FindFileByName(filename)
    mod = types.ModuleType(f"{__name__}.{modname}")
    mod.DESCRIPTOR = fd
    for name, desc in fd.message_types_by_name.items():
        setattr(mod, name, message_factory.GetMessageClass(desc))
    for name, svc in fd.services_by_name.items():
        setattr(mod, f"_{name.upper()}", svc)
    return mod


for _m, _f in _FILES.items():
    _mod = _make_module(_m, _f)
    globals()[_m] = _mod
    sys.modules[_mod.__name__] = _mod

model_pb2 = globals()["model_pb2"]
metis_pb2 = globals()["metis_pb2"]
controller_pb2 = globals()["controller_pb2"]
learner_pb2 = globals()["learner_pb2"]
service_common_pb2 = globals()["service_common_pb2"]


def message_class(full_name: str):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(full_name))
