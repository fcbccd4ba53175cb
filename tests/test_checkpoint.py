"""Background checkpoints (parallel/checkpoint.py): a snapshot is taken at
submit time (later writes to the tensors do not leak into it), the write
runs on a background thread, LATEST only moves to complete checkpoints,
older ones are pruned, errors surface on the next wait, and legacy flat
checkpoints still resolve."""
import json
import os
import time

import pytest
import torch

from metisfl_amd.parallel import checkpoint as ck


def test_snapshot_is_taken_at_submit_time(tmp_path):
    snap = ck.AsyncSnapshot(torch.device("cpu"))
    t = torch.arange(10, dtype=torch.float32)
    out = {}

    def write(h):
        time.sleep(0.1)  # the caller mutates the tensor meanwhile
        out.update({k: v.clone() for k, v in h.items()})

    ms = snap.submit({"t": t}, write)
    t.add_(100.0)
    snap.wait()
    assert ms >= 0 and torch.equal(out["t"], torch.arange(10, dtype=torch.float32))


def test_writer_errors_surface_on_wait():
    snap = ck.AsyncSnapshot(torch.device("cpu"))

    def write(h):
        raise OSError("disk full")

    snap.submit({"t": torch.zeros(1)}, write)
    with pytest.raises(RuntimeError) as ei:
        snap.wait()
    assert isinstance(ei.value.__cause__, OSError)
    snap.wait()  # reported once


def test_try_submit_skips_while_busy():
    snap = ck.AsyncSnapshot(torch.device("cpu"))
    snap.submit({"t": torch.zeros(1)}, lambda h: time.sleep(0.3))
    assert snap.try_submit({"t": torch.zeros(1)}, lambda h: None) is None
    snap.wait()
    assert snap.try_submit({"t": torch.zeros(1)}, lambda h: None) is not None
    snap.wait()


def test_latest_points_at_complete_checkpoints_and_prunes(tmp_path):
    root = str(tmp_path)
    assert ck.resolve(root) is None
    for gi in (1, 2, 3):
        d = tmp_path / f"round_{gi}"
        d.mkdir()
        (d / "federation.json").write_text(json.dumps({"global_iteration": gi}))
        ck.publish(root, f"round_{gi}", keep=2)
    assert ck.resolve(root).endswith("round_3")
    assert sorted(os.listdir(root)) == ["LATEST", "round_2", "round_3"]
    # a round directory without federation.json (a crash mid-write) is never resolved
    (tmp_path / "round_4").mkdir()
    assert ck.resolve(root).endswith("round_3")


def test_legacy_flat_checkpoint_resolves(tmp_path):
    (tmp_path / "federation.json").write_text("{}")
    assert ck.resolve(str(tmp_path)) == str(tmp_path)


def test_native_tensor_writer_roundtrips(tmp_path):
    ts = {"step": torch.tensor(7, dtype=torch.int64), "perm": torch.randperm(33, dtype=torch.int32),
          "m": torch.randn(5, 3), "h": torch.randn(4).to(torch.bfloat16), "flag": torch.tensor([True, False]),
          "empty": torch.zeros(0)}
    p = str(tmp_path / "x.safetensors")
    ck.save_tensors(ts, p)
    got = ck.load_tensors(p)
    assert sorted(got) == sorted(ts)
    for k, v in ts.items():
        assert got[k].dtype == v.dtype and got[k].shape == v.shape and torch.equal(got[k], v), k
    assert not os.path.exists(p + ".tmp")


def test_native_federated_model_writer_matches_python_proto(tmp_path):
    from types import SimpleNamespace
    import numpy as np
    from metisfl_amd.proto import model_pb2
    from metisfl_amd.utils.tensor_codec import model_from_arrays, model_to_arrays
    shapes = [(3, 4), (4,), (2, 2, 2)]
    specs, off = [], 0
    for i, sh in enumerate(shapes):
        n = int(np.prod(sh))
        specs.append(SimpleNamespace(name=f"v{i}", shape=sh, offset=off, numel=n, trainable=i != 1))
        off += n
    flat = np.random.default_rng(0).standard_normal(off).astype(np.float32)
    p = str(tmp_path / "community_model.pb")
    ck.write_federated_model(p, flat, specs, 3, 11)
    fm = model_pb2.FederatedModel()
    fm.ParseFromString(open(p, "rb").read())
    assert fm.num_contributors == 3 and fm.global_iteration == 11
    names, arrays, trainable = model_to_arrays(fm.model)
    assert names == ["v0", "v1", "v2"] and list(trainable) == [True, False, True]
    for s, a in zip(specs, arrays):
        assert a.shape == s.shape and np.array_equal(a, flat[s.offset: s.offset + s.numel].reshape(s.shape))
    ref = model_pb2.FederatedModel(num_contributors=3, global_iteration=11)
    ref.model.CopyFrom(model_from_arrays(names, [flat[s.offset: s.offset + s.numel].reshape(s.shape) for s in specs],
                                         [s.trainable for s in specs]))
    got = model_pb2.FederatedModel()
    got.ParseFromString(open(p, "rb").read())
    assert got == ref
