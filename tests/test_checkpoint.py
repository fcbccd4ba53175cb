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
from metisfl_amd.utils.launch import exits_hard


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


@exits_hard  # a finished rank skips interpreter finalisation (utils/launch.py)
def _publish_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.watchdog import RankWatchdog
    comm = Comm(backend="gloo")
    lost = []
    wd = RankWatchdog(comm, interval_s=0.2, timeout_s=1.5, on_failure=lambda r, p: lost.append(p)).start()
    store = dist.distributed_c10d._get_default_store()
    res = {}
    if rank == 0:
        # rank 1 never reports its files: rank 0 waits (in short polls) for
        # 4 s, well past the peers' 1.5 s heartbeat timeout
        os.makedirs(os.path.join(out_dir, "ck", "round_1"), exist_ok=True)
        t0 = time.time()
        try:
            ck.publish(os.path.join(out_dir, "ck"), "round_1", store, world, "test_publish/1", timeout_s=4.0)
            res["published"] = True
        except TimeoutError:
            res["published"] = False
        res["waited_s"] = time.time() - t0
    else:
        time.sleep(5.0)  # alive and beating, but never sets its key
    res["lost"] = lost
    comm.barrier()
    wd.stop()
    with open(os.path.join(out_dir, f"pub_{rank}.json"), "w") as f:
        json.dump(res, f)
    comm.close()


def test_publish_wait_keeps_rank0_heartbeat(tmp_path):
    """rank 0's publish waits for the other ranks' checkpoint keys
    through the store client its heartbeats also use.  With one peer that
    never reports, rank 0 gives up after its timeout and, meanwhile, keeps
    beating: no rank reports rank 0 (or anyone) lost."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_publish_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0 = json.load(open(tmp_path / "pub_0.json"))
    r1 = json.load(open(tmp_path / "pub_1.json"))
    assert r0["published"] is False and r0["waited_s"] >= 3.9
    assert r0["lost"] == [] and r1["lost"] == []
    assert not (tmp_path / "ck" / "LATEST").exists()
