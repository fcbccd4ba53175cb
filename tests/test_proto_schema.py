"""Wire-format compatibility of the runtime-built ``metisfl`` schema.

The reference's generated ``*_pb2.py`` files embed their FileDescriptorProto
as a bytes literal.  We read that literal with ``ast.literal_eval`` (no code
from the reference is executed or imported) and compare every message,
field number, label, type and enum value with our schema.  If the reference
tree is not mounted the comparison is skipped; the golden-bytes tests below
always run.
"""
import ast
import os

import pytest
from google.protobuf import descriptor_pb2

from metisfl_amd.proto import controller_pb2, learner_pb2, metis_pb2, model_pb2, service_common_pb2
from metisfl_amd.proto import loader

REF = "/root/reference/metisfl/proto"


def _ref_fdp(fn):
    path = os.path.join(REF, fn.replace(".proto", "_pb2.py"))
    if not os.path.exists(path):
        pytest.skip("reference tree not mounted")
    tree = ast.parse(open(path).read())
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "AddSerializedFile":
            raw = ast.literal_eval(node.args[0])
            fdp = descriptor_pb2.FileDescriptorProto()
            fdp.ParseFromString(raw)
            return fdp
        if isinstance(node, ast.keyword) and node.arg == "serialized_pb":
            raw = ast.literal_eval(node.value)
            fdp = descriptor_pb2.FileDescriptorProto()
            fdp.ParseFromString(raw)
            return fdp
    pytest.skip("no serialized descriptor in reference stub")


def _messages(fdp):
    out = {}

    def walk(m, prefix):
        full = f"{prefix}.{m.name}"
        fields = {f.name: (f.number, f.label, f.type, f.type_name, f.proto3_optional,
                           f.HasField("oneof_index")) for f in m.field}
        out[full] = fields
        for e in m.enum_type:
            out[f"{full}.{e.name}"] = {v.name: v.number for v in e.value}
        for n in m.nested_type:
            walk(n, full)

    for m in fdp.message_type:
        walk(m, fdp.package)
    for e in fdp.enum_type:
        out[f"{fdp.package}.{e.name}"] = {v.name: v.number for v in e.value}
    return out


@pytest.mark.parametrize("fn", loader.SCHEMA_FILES)
def test_schema_matches_reference_descriptor(fn):
    ref = _ref_fdp(fn)
    ours = [f for f in loader.build_file_protos() if f.name.endswith(fn)][0]
    assert ref.package == ours.package == "metisfl"
    rm, om = _messages(ref), _messages(ours)
    assert set(rm) == set(om)
    for k in rm:
        assert rm[k] == om[k], k
    rs = {s.name: [(m.name, m.input_type, m.output_type) for m in s.method] for s in ref.service}
    os_ = {s.name: [(m.name, m.input_type, m.output_type) for m in s.method] for s in ours.service}
    assert rs == os_


def test_golden_bytes_tensor_spec():
    m = model_pb2.Model()
    v = m.variables.add()
    v.name = "w"
    v.trainable = True
    t = v.plaintext_tensor.tensor_spec
    t.length = 2
    t.dimensions.extend([2])
    t.type.type = model_pb2.DType.FLOAT32
    t.type.byte_order = model_pb2.DType.LITTLE_ENDIAN_ORDER
    t.value = b"\x00\x00\x80\x3f\x00\x00\x00\x40"  # [1.0, 2.0] little endian
    # hand-encoded: Model{1: Variable{1:"w", 2:1, 3: Plaintext{1: Spec{1:2, 2:[2], 3:{1:8,2:2}, 4:bytes}}}}
    spec = bytes([0x08, 0x02, 0x12, 0x01, 0x02, 0x1A, 0x04, 0x08, 0x08, 0x10, 0x02, 0x22, 0x08]) + t.value
    plain = bytes([0x0A, len(spec)]) + spec
    var = bytes([0x0A, 0x01]) + b"w" + bytes([0x10, 0x01, 0x1A, len(plain)]) + plain
    golden = bytes([0x0A, len(var)]) + var
    assert m.SerializeToString() == golden


def test_all_services_present():
    assert len(controller_pb2._CONTROLLERSERVICE.methods) == 12
    assert [m.name for m in learner_pb2._LEARNERSERVICE.methods] == [
        "EvaluateModel", "GetServicesHealthStatus", "RunTask", "ShutDown"]
    assert service_common_pb2.Ack().DESCRIPTOR.fields_by_name["timestamp"].number == 2
    assert metis_pb2.FederatedTaskRuntimeMetadata.DESCRIPTOR.fields_by_name[
        "model_tensor_quantifiers"].number == 18


def test_fortran_ordered_array_round_trips():
    """A transposed (F-contiguous) weight keeps its values: the bytes are in
    logical C order and the fortran_order flag only records the layout, as
    in the reference (proto_messages_factory.py:462,492)."""
    import numpy as np
    from metisfl_amd.utils.tensor_codec import numpy_to_tensor_spec, tensor_spec_to_numpy
    a = np.asfortranarray(np.arange(6, dtype=np.float32).reshape(2, 3))
    spec = numpy_to_tensor_spec(a)
    assert spec.type.fortran_order
    assert spec.value == np.arange(6, dtype=np.float32).tobytes()
    np.testing.assert_array_equal(tensor_spec_to_numpy(spec), a)
    t = np.arange(12, dtype=np.float64).reshape(3, 4).T  # a view, F-contiguous
    np.testing.assert_array_equal(tensor_spec_to_numpy(numpy_to_tensor_spec(t)), t)
