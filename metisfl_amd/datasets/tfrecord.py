"""TFRecord datasets without TensorFlow (reference: the TFDatasetUtils /
MRIScanGen pipeline of examples/keras/neuroimaging.py:32-230).

The container framing (length + masked CRC32C + data + masked CRC32C) is
read and written by the native engine (``_engine.tfrecord_read`` /
``tfrecord_write``: one mmap pass, SSE4.2 CRC32C); each record is a
``tf.train.Example`` whose features are single ``bytes_list`` values holding
the row's raw array bytes -- exactly what the reference writes
(``_bytes_feature(chunk.flatten().tostring())``) and decodes
(``tf.io.decode_raw(feature, schema[attr])``).

The reference keeps the per-feature dtypes in a cloudpickle ``.schema`` file;
unpickling is not something this framework does with files it did not write,
so the schema travels as JSON (``{feature: numpy dtype string}``) in
``<file>.schema.json``, and can always be passed explicitly.
"""
from __future__ import annotations

import collections
import json
import os

import numpy as np

from metisfl_amd.proto import message_class

_TF_DTYPES = {  # tf.as_dtype(...).name -> numpy (the names the reference's schema holds)
    "float16": "<f2", "float32": "<f4", "float64": "<f8", "int8": "i1", "int16": "<i2", "int32": "<i4",
    "int64": "<i8", "uint8": "u1", "uint16": "<u2", "uint32": "<u4", "uint64": "<u8", "bool": "?",
}


def _example_cls():
    return message_class("tensorflow.Example")


def _engine():
    from metisfl_amd import _engine as E
    return E


def schema_path(path: str) -> str:
    return path + ".schema.json"


def write_examples(path: str, mappings: "collections.OrderedDict[str, np.ndarray]") -> dict:
    """Serialize row i of every array as one Example {name: bytes_list[raw]}.
    Returns (and writes next to ``path``) the ordered {name: dtype} schema."""
    arrays = collections.OrderedDict((k, np.asarray(v)) for k, v in mappings.items())
    n = {len(v) for v in arrays.values()}
    if len(n) != 1:
        raise ValueError("all arrays need the same number of rows")
    Example = _example_cls()
    records = []
    for i in range(n.pop()):
        ex = Example()
        for k, v in arrays.items():
            row = np.ascontiguousarray(v[i])
            ex.features.feature[k].bytes_list.value.append(row.astype(row.dtype.newbyteorder("<")).tobytes())
        records.append(ex.SerializeToString())
    _engine().tfrecord_write(path, records)
    schema = collections.OrderedDict((k, np.dtype(v.dtype).newbyteorder("<").str) for k, v in arrays.items())
    with open(schema_path(path), "w") as f:
        json.dump({"features": list(schema.items()),
                   "shapes": {k: list(v.shape[1:]) for k, v in arrays.items()}}, f)
    return dict(schema)


def read_schema(path: str):
    with open(schema_path(path)) as f:
        d = json.load(f)
    return collections.OrderedDict(d["features"]), {k: tuple(v) for k, v in d.get("shapes", {}).items()}


def read_examples(path: str, schema: dict | None = None, shapes: dict | None = None,
                  verify: bool = True) -> "collections.OrderedDict[str, np.ndarray]":
    """Decode every Example of ``path`` into stacked arrays, one per feature.
    ``schema`` maps feature -> numpy dtype (or TF dtype name); without it the
    JSON sidecar written by :func:`write_examples` is used.  Like the
    reference's deserializer, an unordered schema is decoded in sorted key
    order."""
    if schema is None:
        schema, side_shapes = read_schema(path)
        shapes = shapes or side_shapes
    if not isinstance(schema, collections.OrderedDict):
        schema = collections.OrderedDict((k, schema[k]) for k in sorted(schema))
    dtypes = {k: np.dtype(_TF_DTYPES.get(str(v), v)) for k, v in schema.items()}
    Example = _example_cls()
    cols: dict[str, list] = {k: [] for k in schema}
    for rec in _engine().tfrecord_read(path, verify):
        ex = Example()
        ex.ParseFromString(rec)
        for k in schema:
            f = ex.features.feature[k]
            if f.WhichOneof("kind") != "bytes_list" or len(f.bytes_list.value) != 1:
                raise ValueError(f"feature {k!r} is not a single raw bytes value")
            cols[k].append(np.frombuffer(f.bytes_list.value[0], dtype=dtypes[k]))
    out = collections.OrderedDict()
    for k, rows in cols.items():
        a = np.stack(rows) if rows else np.zeros((0,), dtypes[k])
        if shapes and k in shapes and rows:
            a = a.reshape((len(rows),) + tuple(shapes[k]))
        elif a.ndim == 2 and a.shape[1] == 1:
            a = a[:, 0]  # scalar features (labels)
        out[k] = a.astype(dtypes[k].newbyteorder("="), copy=False)
    return out


def exists(path: str) -> bool:
    return os.path.exists(path) and os.path.exists(schema_path(path))
