"""Asynchronous FedRec federation over point-to-point collectives (gloo,
world size 3; the RCCL path on GPUs is the same code): every submission is
applied, the incremental community equals the host recomputation over each
learner's latest model, and finishers receive a community model."""
import json
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from metisfl_amd.utils.launch import exits_hard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@exits_hard  # a finished rank skips interpreter finalisation (utils/launch.py)
def _worker(rank, world, port, out_dir, staleness="none", threaded=True):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig
    comm = Comm(backend="gloo")
    net = HousingMLP(batch_size=4, device="cpu", seed=rank + 1,
                     optimizer=OptimizerSpec("vanilla_sgd", learning_rate=0.01))
    rng = np.random.default_rng(rank)
    n = 8 + 4 * rank
    ds = net.make_dataset(rng.standard_normal((n, 13)).astype(np.float32),
                          rng.standard_normal(n).astype(np.float32), seed=rank)
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, staleness=staleness)
    fed = AsyncCollectiveFederation(comm, net, ds, cfg, tasks_per_learner=3, poll_every=1,
                                    serve_in_thread=threaded)
    ups = fed.run()
    res = {"rank": rank, "final": net.state.model32.numpy().tolist()}
    if rank == 0:
        ref = fed.community_reference()
        got = fed._community().double().numpy()
        res["updates"] = [(u.learner, u.task, u.weight) for u in ups]
        res["stale"] = [(u.staleness, u.base_weight, u.weight) for u in ups]
        res["max_err"] = float(np.abs(got - ref).max() / (np.abs(ref).max() + 1e-12))
    with open(os.path.join(out_dir, f"async_{staleness}_{rank}.json"), "w") as f:
        json.dump(res, f)
    comm.barrier()
    comm.close()


import pytest  # noqa: E402


@pytest.mark.parametrize("threaded", [True, False], ids=["service-thread", "chunked"])
def test_async_fedrec_three_learners(tmp_path, threaded):
    world = 3
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), "none", threaded), nprocs=world,
                       join=True, start_method="spawn")
    res = [json.load(open(tmp_path / f"async_none_{r}.json")) for r in range(world)]
    ups = res[0]["updates"]
    assert len(ups) == world * 3
    for r in range(world):
        tasks = [t for (l, t, _) in ups if l == r]
        assert tasks == [0, 1, 2]  # every task of every learner applied, in order
        assert all(w == 8 + 4 * r for (l, _, w) in ups if l == r)  # NUM_TRAINING_EXAMPLES weights
    assert res[0]["max_err"] < 1e-5
    for r in res:
        assert np.all(np.isfinite(r["final"]))


def test_staleness_functions():
    from metisfl_amd.parallel.async_federation import staleness_discount as sd
    assert sd("none", 7) == 1.0
    assert sd("polynomial", 0) == 1.0 and abs(sd("polynomial", 3, a=0.5) - 0.5) < 1e-12
    assert sd("hinge", 4, a=0.5, b=4) == 1.0 and abs(sd("hinge", 6, a=0.5, b=4) - 0.5) < 1e-12


def test_async_staleness_aware_weights(tmp_path):
    """Polynomial staleness discount: every applied weight is the
    NUM_TRAINING_EXAMPLES weight times (1 + staleness)^-0.5, staleness counts
    the community versions published since the learner's base model, and the
    incremental community still equals the host recomputation."""
    world = 3
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), "polynomial"), nprocs=world,
                       join=True, start_method="spawn")
    r0 = json.load(open(tmp_path / "async_polynomial_0.json"))
    assert len(r0["stale"]) == world * 3
    for i, (st, w0, w) in enumerate(r0["stale"]):
        assert 0 <= st <= i
        assert abs(w - w0 * (1.0 + st) ** -0.5) < 1e-9
    assert r0["stale"][0][0] == 0          # the very first update is fresh
    assert any(st > 0 for st, _, _ in r0["stale"])
    assert r0["max_err"] < 1e-5


@exits_hard  # a finished rank skips interpreter finalisation (utils/launch.py)
def _coloc_worker(rank, world, port, out_dir, per_rank, tasks):
    """Rank r hosts ``per_rank`` co-located learners (global ids r*per_rank + j)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig
    comm = Comm(backend="gloo")
    nets, dss = [], []
    gids = [rank * per_rank + j for j in range(per_rank)]
    for g in gids:
        net = HousingMLP(batch_size=4, device="cpu", seed=g + 1, optimizer=OptimizerSpec("vanilla_sgd", 0.01))
        rng = np.random.default_rng(g)
        n = 8 + 4 * g
        nets.append(net)
        dss.append(net.make_dataset(rng.standard_normal((n, 13)).astype(np.float32),
                                    rng.standard_normal(n).astype(np.float32), seed=g))
    owners = [g // per_rank for g in range(world * per_rank)]
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, staleness="polynomial")
    fed = AsyncCollectiveFederation(comm, nets, dss, cfg, tasks_per_learner=tasks, gids=gids, owners=owners,
                                    learner_ids=[f"L{g}" for g in range(len(owners))])
    ups = fed.run()
    res = {"rank": rank, "finals": [n.state.model32.numpy().tolist() for n in nets]}
    if rank == 0:
        res["updates"] = [(u.learner, u.task, u.base_weight, u.staleness) for u in ups]
        ref = fed.community_reference()
        got = fed._community().double().numpy()
        res["max_err"] = float(np.abs(got - ref).max() / (np.abs(ref).max() + 1e-12))
        res["community"] = got.tolist()
    with open(os.path.join(out_dir, f"coloc_{rank}.json"), "w") as f:
        json.dump(res, f)
    comm.barrier()
    comm.close()


def test_async_fedrec_colocated_learners_on_two_ranks(tmp_path):
    """The reference schedules asynchronously per LEARNER whatever the
    placement (asynchronous_scheduler.h:12-18): 2 ranks x 2 co-located
    learners = 4 FedRec participants; every task of every learner is applied
    in order with its own NUM_TRAINING_EXAMPLES weight, and the incremental
    community equals the host recomputation over each learner's latest model."""
    world, per, tasks = 2, 2, 3
    mp.start_processes(_coloc_worker, args=(world, _free_port(), str(tmp_path), per, tasks), nprocs=world,
                       join=True, start_method="spawn")
    r0 = json.load(open(tmp_path / "coloc_0.json"))
    ups = r0["updates"]
    assert len(ups) == world * per * tasks
    for g in range(world * per):
        assert [t for (l, t, _, _) in ups if l == g] == list(range(tasks))
        assert all(w == 8 + 4 * g for (l, _, w, _) in ups if l == g)
    assert any(st > 0 for (_, _, _, st) in ups)  # interleaved finishers: staleness
    assert r0["max_err"] < 1e-5
    for r in range(world):
        res = json.load(open(tmp_path / f"coloc_{r}.json"))
        assert all(np.all(np.isfinite(f)) for f in res["finals"])


@exits_hard  # a finished rank skips interpreter finalisation (utils/launch.py)
def _secure_worker(rank, world, port, out_dir, per_rank, tasks):
    """Secure aggregation (CKKS PWA) with the asynchronous protocol: every
    learner records the plaintext model it submitted (test hook) so the test
    can recompute the PWA on the host."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig
    comm = Comm(backend="gloo")
    gids = [rank * per_rank + j for j in range(per_rank)]
    nets, dss = [], []
    for g in gids:
        net = HousingMLP(batch_size=4, device="cpu", seed=g + 1, optimizer=OptimizerSpec("vanilla_sgd", 0.01))
        rng = np.random.default_rng(g)
        n = 8 + 4 * g
        nets.append(net)
        dss.append(net.make_dataset(rng.standard_normal((n, 13)).astype(np.float32),
                                    rng.standard_normal(n).astype(np.float32), seed=g))
    owners = [g // per_rank for g in range(world * per_rank)]
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, staleness="polynomial",
                           secure_aggregation=True)
    fed = AsyncCollectiveFederation(comm, nets, dss, cfg, tasks_per_learner=tasks, gids=gids, owners=owners)
    submitted = {g: [] for g in gids}
    orig = fed._submit

    def spy(L, meta, _orig=orig):
        submitted[L.gid].append(L.net.state.model32.numpy().astype(np.float64).tolist())
        _orig(L, meta)
        # the learner now holds the decrypted community model
        submitted[L.gid].append(L.net.state.model32.numpy().astype(np.float64).tolist())
    fed._submit = spy
    ups = fed.run()
    res = {"rank": rank, "submitted": {str(g): v for g, v in submitted.items()}}
    if rank == 0:
        res["updates"] = [(u.learner, u.task, u.weight, u.staleness) for u in ups]
        res["community"] = fed.community().double().numpy().tolist()
        res["ref"] = fed.community_reference().tolist()
        res["ct_is_bytes"] = bool(fed.last[0].dtype == torch.uint8)
    with open(os.path.join(out_dir, f"secure_{rank}.json"), "w") as f:
        json.dump(res, f)
    comm.barrier()
    comm.close()


def test_async_secure_pwa_over_latest_ciphertexts(tmp_path):
    """asynchronous PWA on the collective plane.  2 ranks x 2
    learners submit CKKS ciphertexts; rank 0 keeps the latest one per learner
    and answers each finisher with the PWA ciphertext, which the finisher
    decrypts.  Replaying the updates on the host (each learner's latest
    submitted plaintext, its staleness-discounted weight) reproduces every
    community model a learner received, to CKKS precision."""
    world, per, tasks = 2, 2, 2
    mp.start_processes(_secure_worker, args=(world, _free_port(), str(tmp_path), per, tasks), nprocs=world,
                       join=True, start_method="spawn")
    res = [json.load(open(tmp_path / f"secure_{r}.json")) for r in range(world)]
    r0 = res[0]
    assert r0["ct_is_bytes"]  # the aggregator holds ciphertexts, not models
    sub = {}
    for r in res:
        sub.update({int(g): v for g, v in r["submitted"].items()})
    ups = r0["updates"]
    assert len(ups) == world * per * tasks
    latest, weights = {}, {}
    for (g, t, w, _) in ups:  # replay in aggregation order
        latest[g] = np.array(sub[g][2 * t])
        weights[g] = w
        ref = sum(weights[k] * latest[k] for k in latest) / sum(weights.values())
        got = np.array(sub[g][2 * t + 1])  # what the finisher decrypted
        assert np.abs(got - ref).max() <= 1e-5 * (np.abs(ref).max() + 1e-9), (g, t)
    final = np.array(r0["community"])
    assert np.abs(final - ref).max() <= 1e-5 * (np.abs(ref).max() + 1e-9)
    assert np.abs(np.array(r0["ref"]) - ref).max() <= 1e-5 * (np.abs(ref).max() + 1e-9)


def test_async_colocated_single_process():
    """World 1 (no process group): several co-located learners, all FedRec on
    rank 0's device path -- the on-one-GPU asynchronous configuration."""
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig
    comm = Comm(backend="gloo")  # no RANK / WORLD_SIZE here: world 1, no process group
    assert not comm.distributed
    nets, dss = [], []
    for g in range(3):
        net = HousingMLP(batch_size=4, device="cpu", seed=g + 1, optimizer=OptimizerSpec("vanilla_sgd", 0.01))
        rng = np.random.default_rng(g)
        nets.append(net)
        dss.append(net.make_dataset(rng.standard_normal((8 + 4 * g, 13)).astype(np.float32),
                                    rng.standard_normal(8 + 4 * g).astype(np.float32), seed=g))
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False)
    fed = AsyncCollectiveFederation(comm, nets, dss, cfg, tasks_per_learner=2)
    ups = fed.run()
    assert len(ups) == 6 and fed.version == 6
    assert sorted(u.learner for u in ups) == [0, 0, 1, 1, 2, 2]
    ref = fed.community_reference()
    assert np.abs(fed.community().double().numpy() - ref).max() <= 1e-5 * (np.abs(ref).max() + 1e-12)


def test_async_secure_checkpoint_resume_drops_lost_learner(tmp_path):
    """Secure asynchronous checkpoints hold every learner's latest CIPHERTEXT
    (no plaintext community model is written); a resume on fewer learners
    drops the lost learner's ciphertext from the PWA set and restarts the
    survivors from the PWA of the remaining ones (decrypted by the learners'
    host, rank 0), continuing the version count."""
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel import checkpoint as ck
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig

    def learners(gs):
        nets, dss = [], []
        for g in gs:
            net = HousingMLP(batch_size=4, device="cpu", seed=g + 1, optimizer=OptimizerSpec("vanilla_sgd", 0.01))
            rng = np.random.default_rng(g)
            nets.append(net)
            dss.append(net.make_dataset(rng.standard_normal((8 + 4 * g, 13)).astype(np.float32),
                                        rng.standard_normal(8 + 4 * g).astype(np.float32), seed=g))
        return nets, dss

    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, secure_aggregation=True)
    comm = Comm(backend="gloo")
    nets, dss = learners([0, 1, 2])
    fed = AsyncCollectiveFederation(comm, nets, dss, cfg, learner_ids=["L0", "L1", "L2"])
    fed.run_until(max_updates=6, checkpoint_dir=str(tmp_path / "ck"), checkpoint_every=1)
    assert fed.version >= 6
    d = ck.resolve(str(tmp_path / "ck"))
    meta = json.load(open(os.path.join(d, "federation.json")))
    assert meta["secure_aggregation"] and not os.path.exists(os.path.join(d, "community_model.pb"))
    plain = {lid: fed.he.decrypt_fresh(fed.last[g]) for g, lid in enumerate(["L0", "L1", "L2"])}
    w = dict(zip(["L0", "L1", "L2"], fed.last_w))
    # two learners come back (L1 is lost); they share the key pair
    nets2, dss2 = learners([0, 2])
    cfg2 = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, secure_aggregation=True,
                            he_key_dir=fed._he_dir)
    fed2 = AsyncCollectiveFederation(comm, nets2, dss2, cfg2, learner_ids=["L0", "L2"])
    fed2.resume(str(tmp_path / "ck"))
    assert fed2.version == meta["version"] and fed2.resumed["dropped"] == ["L1"]
    ref = (w["L0"] * plain["L0"] + w["L2"] * plain["L2"]) / (w["L0"] + w["L2"])
    for n in nets2:
        got = n.state.model32.double().numpy()
        assert np.abs(got - ref).max() <= 1e-5 * (np.abs(ref).max() + 1e-9)
    ups = fed2.run()
    assert len(ups) == 2 * fed2.tasks and fed2.version == meta["version"] + 2 * fed2.tasks


class _SlowLineageEngine:
    """Controller bridge stand-in: a lineage send takes 0.2 s, so most of the
    community versions' snapshots are skipped while one is in flight."""

    def __init__(self):
        self.versions, self.models = [], {}

    def snapshot_community(self, names, arrays, trainable, version):
        import time
        time.sleep(0.2)
        self.versions.append(int(version))
        self.models[int(version)] = np.concatenate([np.asarray(a).reshape(-1) for a in arrays])

    def record_async_update(self, *a):
        pass

    def record_async_evaluation(self, *a):
        pass

    def should_stop(self):
        return False


def test_async_final_community_version_reaches_the_lineage():
    """The asynchronous aggregator's lineage snapshots are best effort (skipped
    while the previous one is being sent), but the FINAL community version
    always reaches the controller (flush re-sends it)."""
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig
    comm = Comm(backend="gloo")
    nets, dss = [], []
    for g in range(3):
        net = HousingMLP(batch_size=4, device="cpu", seed=g + 1, optimizer=OptimizerSpec("vanilla_sgd", 0.01))
        rng = np.random.default_rng(g)
        nets.append(net)
        dss.append(net.make_dataset(rng.standard_normal((8, 13)).astype(np.float32),
                                    rng.standard_normal(8).astype(np.float32), seed=g))
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, snapshot_every=1)
    eng = _SlowLineageEngine()
    fed = AsyncCollectiveFederation(comm, nets, dss, cfg, engine=eng)
    fed.run_until(max_updates=12)
    assert fed.version >= 12
    assert len(eng.versions) < fed.version      # some versions were skipped ...
    assert eng.versions[-1] == fed.version      # ... but not the final one
    flat = fed.community().numpy()
    want = np.concatenate([flat[sp.offset: sp.offset + sp.numel] for sp in nets[0].state.specs])
    np.testing.assert_allclose(eng.models[fed.version], want, rtol=1e-6, atol=1e-7)


def _fedrec_drift(resum_every: int, versions: int = 5000) -> float:
    """Relative max error of the FedRec community after ``versions`` random
    submissions against the host fp64 average of every learner's latest
    contribution."""
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import FederationConfig
    comm = Comm(backend="gloo")
    nets, dss = [], []
    for g in range(4):
        net = HousingMLP(batch_size=4, device="cpu", seed=g + 1, optimizer=OptimizerSpec("vanilla_sgd", 0.01))
        rng = np.random.default_rng(g)
        nets.append(net)
        dss.append(net.make_dataset(rng.standard_normal((8, 13)).astype(np.float32),
                                    rng.standard_normal(8).astype(np.float32), seed=g))
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, fedrec_resum_every=resum_every)
    fed = AsyncCollectiveFederation(comm, nets, dss, cfg)
    n = nets[0].state.model32.numel()
    rng = np.random.default_rng(123)
    for v in range(versions):
        g = int(rng.integers(0, 4))
        # contributions of very different magnitude and weight: the running
        # sum's fp32 subtract / add rounding is what accumulates
        theta = torch.from_numpy((rng.standard_normal(n) * 10.0 ** rng.integers(-2, 3)).astype(np.float32))
        meta = {"task": v, "weight": float(rng.integers(1, 1000)), "loss": 0.0, "batches": 1,
                "base_version": fed.version}
        fed._fedrec(g, theta, meta)
    ref = fed.community_reference()
    got = fed._community().double().numpy()
    return float(np.abs(got - ref).max() / np.abs(ref).max())


def test_fedrec_running_sum_stays_exact_over_5000_versions():
    """VERDICT r5 #5c: 5,000 asynchronous FedRec versions stay within 1e-6 of
    the host fp64 recomputation over the learners' latest models (the
    aggregator re-sums S from them every ``fedrec_resum_every`` versions);
    the reference-style running sum alone drifts further."""
    err = _fedrec_drift(32)
    assert err <= 1e-6, err
    assert _fedrec_drift(0) > err
