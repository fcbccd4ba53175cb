"""numpy / device buffers <-> ``TensorSpec`` / ``Model`` protos.

Wire layout (reference: proto_messages_factory.py:399-505,
proto_tensor_serde.h:14-32): ``value`` holds the flattened tensor bytes in
the byte order recorded in ``DType.byte_order``; ``length`` is the element
count; ``dimensions`` the shape.  bf16 has no DType code in the schema, so
bf16 tensors are widened to FLOAT32 at the API boundary.
"""
from __future__ import annotations

import sys

import numpy as np

from metisfl_amd.proto import model_pb2

_NP_TO_DT = {
    np.dtype("int8"): model_pb2.DType.INT8,
    np.dtype("int16"): model_pb2.DType.INT16,
    np.dtype("int32"): model_pb2.DType.INT32,
    np.dtype("int64"): model_pb2.DType.INT64,
    np.dtype("uint8"): model_pb2.DType.UINT8,
    np.dtype("uint16"): model_pb2.DType.UINT16,
    np.dtype("uint32"): model_pb2.DType.UINT32,
    np.dtype("uint64"): model_pb2.DType.UINT64,
    np.dtype("float32"): model_pb2.DType.FLOAT32,
    np.dtype("float64"): model_pb2.DType.FLOAT64,
}
_DT_TO_NP = {v: k for k, v in _NP_TO_DT.items()}


def _byte_order_code(dt: np.dtype) -> int:
    if dt.itemsize == 1:
        return model_pb2.DType.NA
    bo = dt.byteorder
    if bo == "=":
        bo = "<" if sys.byteorder == "little" else ">"
    return model_pb2.DType.LITTLE_ENDIAN_ORDER if bo == "<" else model_pb2.DType.BIG_ENDIAN_ORDER


def numpy_to_tensor_spec(arr: np.ndarray, spec: model_pb2.TensorSpec | None = None) -> model_pb2.TensorSpec:
    arr = np.asarray(arr)
    if arr.dtype.name == "bfloat16" or str(arr.dtype) == "bfloat16":
        arr = arr.astype(np.float32)
    base = arr.dtype.newbyteorder("=")
    if base not in _NP_TO_DT:
        raise TypeError(f"unsupported dtype {arr.dtype}")
    spec = spec if spec is not None else model_pb2.TensorSpec()
    spec.length = int(arr.size)
    del spec.dimensions[:]
    spec.dimensions.extend(int(d) for d in arr.shape)
    spec.type.type = _NP_TO_DT[base]
    spec.type.byte_order = _byte_order_code(arr.dtype)
    spec.type.fortran_order = bool(arr.flags["F_CONTIGUOUS"] and not arr.flags["C_CONTIGUOUS"])
    spec.value = np.ascontiguousarray(arr).tobytes()
    return spec


def tensor_spec_to_numpy(spec: model_pb2.TensorSpec) -> np.ndarray:
    dt = _DT_TO_NP[spec.type.type]
    if spec.type.byte_order == model_pb2.DType.BIG_ENDIAN_ORDER:
        dt = dt.newbyteorder(">")
    elif spec.type.byte_order == model_pb2.DType.LITTLE_ENDIAN_ORDER:
        dt = dt.newbyteorder("<")
    arr = np.frombuffer(spec.value, dtype=dt, count=spec.length)
    shape = tuple(spec.dimensions) if len(spec.dimensions) else (spec.length,)
    # ``value`` always holds the elements in logical (C) order -- the encoder
    # above and the reference (proto_messages_factory.py:462 ``arr.flatten()``,
    # :492 plain reshape) both write it so; ``fortran_order`` only records the
    # source array's memory layout and must not re-order the decode.
    return arr.reshape(shape)


def model_from_arrays(names, arrays, trainables=None, he_scheme=None) -> model_pb2.Model:
    """Build a ``Model``; with ``he_scheme`` every variable is CKKS-encrypted
    into a ``ciphertext_tensor`` (length / dims keep the plaintext shape)."""
    m = model_pb2.Model()
    trainables = trainables if trainables is not None else [True] * len(names)
    for name, arr, tr in zip(names, arrays, trainables):
        v = m.variables.add()
        v.name = name
        v.trainable = bool(tr)
        a = np.asarray(arr)
        if he_scheme is not None:
            spec = v.ciphertext_tensor.tensor_spec
            numpy_to_tensor_spec(a.astype(np.float64), spec)
            spec.value = he_scheme.encrypt(a.reshape(-1).astype(np.float64))
        else:
            numpy_to_tensor_spec(a, v.plaintext_tensor.tensor_spec)
    return m


def model_to_arrays(model: model_pb2.Model, he_scheme=None):
    """-> (names, arrays, trainables); decrypts ciphertext variables."""
    names, arrays, tr = [], [], []
    for v in model.variables:
        names.append(v.name)
        tr.append(v.trainable)
        if v.HasField("ciphertext_tensor"):
            if he_scheme is None:
                raise ValueError(f"variable {v.name} is encrypted and no HE scheme was given")
            spec = v.ciphertext_tensor.tensor_spec
            vals = np.asarray(he_scheme.decrypt(spec.value, spec.length))
            shape = tuple(spec.dimensions) if len(spec.dimensions) else (spec.length,)
            arrays.append(vals.reshape(shape).astype(_DT_TO_NP.get(spec.type.type, np.float64)))
        else:
            arrays.append(tensor_spec_to_numpy(v.plaintext_tensor.tensor_spec))
    return names, arrays, tr
