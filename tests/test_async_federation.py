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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
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
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False)
    fed = AsyncCollectiveFederation(comm, net, ds, cfg, tasks_per_learner=3, poll_every=1)
    ups = fed.run()
    res = {"rank": rank, "final": net.state.model32.numpy().tolist()}
    if rank == 0:
        ref = fed.community_reference()
        got = fed._community().double().numpy()
        res["updates"] = [(u.learner, u.task, u.weight) for u in ups]
        res["max_err"] = float(np.abs(got - ref).max() / (np.abs(ref).max() + 1e-12))
    with open(os.path.join(out_dir, f"async_{rank}.json"), "w") as f:
        json.dump(res, f)
    comm.barrier()
    comm.close()


def test_async_fedrec_three_learners(tmp_path):
    world = 3
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [json.load(open(tmp_path / f"async_{r}.json")) for r in range(world)]
    ups = res[0]["updates"]
    assert len(ups) == world * 3
    for r in range(world):
        tasks = [t for (l, t, _) in ups if l == r]
        assert tasks == [0, 1, 2]  # every task of every learner applied, in order
        assert all(w == 8 + 4 * r for (l, _, w) in ups if l == r)  # NUM_TRAINING_EXAMPLES weights
    assert res[0]["max_err"] < 1e-5
    for r in res:
        assert np.all(np.isfinite(r["final"]))
