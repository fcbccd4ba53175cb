"""The collective (torch.distributed) federation engine across real processes:
world size 2 on the gloo backend (the RCCL path on GPUs runs the identical
code).  Checks FedAvg numerics against the host reference, identical
community models on every rank, the semi-synchronous step budgets, the
native controller's bookkeeping on rank 0, and checkpoint / resume."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from metisfl_amd.utils.launch import exits_hard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@exits_hard  # a finished rank skips interpreter finalisation (utils/launch.py)
def _worker(rank, world, port, out_dir, mode):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.engine_bridge import CollectiveController
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig
    comm = Comm(backend="gloo")
    net = ResNet18(batch_size=4, device="cpu", seed=rank + 1, width_mult=0.125,
                   optimizer=OptimizerSpec("momentum_sgd", learning_rate=0.01, momentum=0.9))
    rng = np.random.default_rng(rank)
    n = 8 + 4 * rank  # unequal shards -> unequal FedAvg weights
    ds = net.make_dataset(rng.standard_normal((n, 32, 32, 3)).astype(np.float32), rng.integers(0, 10, n),
                          seed=rank)
    cfg = FederationConfig(protocol="semi_synchronous" if mode == "semi" else "synchronous", batch_size=4,
                           local_epochs=1, semi_sync_lambda=2.0, evaluate_test=False,
                           secure_aggregation=mode == "secure",
                           aggregation="fed_stride" if mode == "stride" else "fed_avg",
                           stride_length=1 if mode == "stride" else 0)
    sizes = [8 + 4 * r for r in range(world)]
    engine = CollectiveController(cfg, sizes) if rank == 0 else None
    fed = CollectiveFederation(comm, net, ds, cfg, engine=engine)
    res = {"rank": rank, "rounds": []}
    if mode == "resume":
        fed.resume(os.path.join(out_dir, "ckpt"))
    for r in range(2 if mode != "resume" else 1):
        # local model before aggregation, for the host FedAvg reference
        orig = fed.aggregate

        def spy(meta, _orig=orig, _r=r):
            np.save(os.path.join(out_dir, f"local_r{_r}_rank{rank}.npy"), net.state.model32.numpy())
            return _orig(meta)
        fed.aggregate = spy
        rec = fed.run_round()
        fed.aggregate = orig
        np.save(os.path.join(out_dir, f"community_r{rec.global_iteration}_rank{rank}.npy"),
                net.state.model32.numpy())
        res["rounds"].append({"gi": rec.global_iteration, "weights": rec.weights,
                              "updates": list(rec.num_local_updates), "next": list(fed.num_local_updates)})
        if mode == "ckpt" and r == 0:
            fed.save_checkpoint(os.path.join(out_dir, "ckpt"))
    if rank == 0:
        md = engine.runtime_metadata(0).metadata
        tl = engine.local_task_lineage(0)
        res["engine"] = {"rounds": len(md), "quantifiers": len(md[-1].model_tensor_quantifiers),
                         "lineage": {k: len(v.task_metadata) for k, v in tl.learner_task.items()},
                         "learners": len(engine.participating_learners().learner)}
    with open(os.path.join(out_dir, f"res_{mode}_{rank}.json"), "w") as f:
        json.dump(res, f)
    comm.close()


def _run(tmp_path, mode, world=2):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world,
                       join=True, start_method="spawn")
    return [json.load(open(tmp_path / f"res_{mode}_{r}.json")) for r in range(world)]


def test_sync_fedavg_two_ranks_matches_host_reference(tmp_path):
    res = _run(tmp_path, "sync")
    w = res[0]["rounds"][0]["weights"]
    assert np.allclose(w, [8 / 20, 12 / 20])
    for r in (0, 1):
        gi = r + 1
        a = np.load(tmp_path / f"community_r{gi}_rank0.npy")
        b = np.load(tmp_path / f"community_r{gi}_rank1.npy")
        assert np.array_equal(a, b)  # every learner holds the same community model
        l0 = np.load(tmp_path / f"local_r{r}_rank0.npy").astype(np.float64)
        l1 = np.load(tmp_path / f"local_r{r}_rank1.npy").astype(np.float64)
        ref = w[0] * l0 + w[1] * l1
        assert np.allclose(a, ref, rtol=1e-5, atol=1e-6)
    eng = res[0]["engine"]
    assert eng["rounds"] == 2 and eng["learners"] == 2 and eng["quantifiers"] > 0
    assert sorted(eng["lineage"].values()) == [2, 2]


def test_fed_stride_three_ranks_matches_engine_fedstride(tmp_path):
    """FedStride (stride 1: the most memory-bounded rolling fold) on the
    collective path equals the native engine's host FedStride over the same
    local models and weights (up to fp32 summation order)."""
    from metisfl_amd import _engine as E
    from metisfl_amd.proto import model_pb2
    from metisfl_amd.utils.tensor_codec import model_from_arrays, model_to_arrays
    res = _run(tmp_path, "stride", world=3)
    w = res[0]["rounds"][0]["weights"]
    assert np.allclose(w, np.array([8, 12, 16]) / 36)
    for r in (0, 1):
        gi = r + 1
        comm = [np.load(tmp_path / f"community_r{gi}_rank{k}.npy") for k in range(3)]
        assert all(np.array_equal(comm[0], c) for c in comm[1:])
        locs = [np.load(tmp_path / f"local_r{r}_rank{k}.npy") for k in range(3)]
        models = [model_from_arrays(["flat"], [l]).SerializeToString() for l in locs]
        fm = model_pb2.FederatedModel()
        fm.ParseFromString(E.aggregate_models("fed_stride", models, [float(x) for x in w], 1))
        ref = model_to_arrays(fm.model)[1][0]
        assert np.allclose(comm[0], ref, rtol=1e-5, atol=1e-6)


def test_secure_ckks_aggregation_two_ranks(tmp_path):
    """CKKS secure aggregation (reference PWA path): ciphertexts cross the
    process boundary, every rank decrypts the same weighted average."""
    res = _run(tmp_path, "secure")
    w = res[0]["rounds"][0]["weights"]
    for r in (0, 1):
        gi = r + 1
        a = np.load(tmp_path / f"community_r{gi}_rank0.npy")
        b = np.load(tmp_path / f"community_r{gi}_rank1.npy")
        assert np.array_equal(a, b)
        l0 = np.load(tmp_path / f"local_r{r}_rank0.npy").astype(np.float64)
        l1 = np.load(tmp_path / f"local_r{r}_rank1.npy").astype(np.float64)
        assert np.abs(a - (w[0] * l0 + w[1] * l1)).max() < 1e-5


def test_semi_sync_step_budgets(tmp_path):
    res = _run(tmp_path, "semi")
    r0 = res[0]["rounds"]
    # round 1 uses epochs * ceil(n / batch); the end of round 1 recomputes
    # the budgets from lambda * slowest epoch time, so round 2 already runs
    # with them (controller.cc:520-569, as the native engine does)
    assert r0[0]["updates"] == [2, 3]
    assert r0[1]["updates"] == r0[0]["next"]  # round 2 ran the recomputed budgets
    assert all(u >= 1 for u in r0[1]["updates"])
    assert res[0]["rounds"][1]["updates"] == res[1]["rounds"][1]["updates"]


def test_checkpoint_resume_reproduces_the_next_round(tmp_path):
    _run(tmp_path, "ckpt")
    straight = np.load(tmp_path / "community_r2_rank0.npy")
    os.remove(tmp_path / "community_r2_rank0.npy")
    _run(tmp_path, "resume")
    resumed = np.load(tmp_path / "community_r2_rank0.npy")
    assert np.allclose(straight, resumed, rtol=1e-6, atol=1e-7)


@exits_hard  # a finished rank skips interpreter finalisation (utils/launch.py)
def _wd_worker(rank, world, port, out_dir):
    import time as _t
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.watchdog import RankWatchdog
    comm = Comm(backend="gloo")
    seen = []
    wd = RankWatchdog(comm, interval_s=0.1, timeout_s=0.6, on_failure=lambda r, p: seen.append(p)).start()
    comm.barrier()
    if rank == 1:
        wd.pause()  # fault injection: rank 1 hangs (heartbeats stop)
    _t.sleep(2.0)
    with open(os.path.join(out_dir, f"wd_{rank}.json"), "w") as f:
        json.dump(seen, f)
    wd.stop()
    comm.barrier()
    comm.close()


def test_watchdog_detects_a_hung_rank(tmp_path):
    mp.start_processes(_wd_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    assert json.load(open(tmp_path / "wd_0.json")) == [1]   # rank 0 saw rank 1 go silent
    assert json.load(open(tmp_path / "wd_1.json")) == []    # rank 0 kept beating
