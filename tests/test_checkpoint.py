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
