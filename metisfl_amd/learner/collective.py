"""One rank of an on-node collective federation, launched by
``DriverSession`` when the federation environment says ``DataPlane: rccl``
(one process per GPU, torch.distributed env from the driver).

Rank 0 fetches the driver's initial community model from the controller and
broadcasts it; every round the learners train their shards and average in
place with one RCCL all-reduce (parallel/federation.py); rank 0 reports each
round to the controller's collective bookkeeping service, so the driver's
``monitor_federation`` / ``get_federation_statistics`` see the rounds.  The
reference has no such data plane: its learners always ship models through
the controller (driver_session.py:529-582 launches them with their GPUs).

    python -m metisfl_amd.learner.collective <job.json>
"""
from __future__ import annotations

import json
import os
import sys


def _load_recipe(path):
    if not path:
        return None
    import cloudpickle  # the driver's own file (DriverSession._dump_recipe)
    with open(path, "rb") as f:
        return cloudpickle.load(f)


def main(argv=None) -> int:
    argv = argv if argv is not None else sys.argv[1:]
    with open(argv[0]) as f:
        job = json.load(f)
    import torch

    from metisfl_amd.learner.learner import resolve_dataset
    from metisfl_amd.models.model_def import StaticModelDef
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.engine_bridge import RemoteCollectiveController
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig
    from metisfl_amd.proto import metis_pb2, model_pb2
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient

    comm = Comm(backend=job.get("backend"))
    rank = comm.rank
    lcfg = job["learners"][rank]
    torch.manual_seed(job.get("seed", 0) + rank)
    opt = OptimizerSpec.from_proto(model_pb2.OptimizerConfig.FromString(bytes.fromhex(job["optimizer_hex"])))
    model_def = StaticModelDef.load(job["model_dir"])
    net = model_def.get_model(batch_size=job["batch_size"], device=comm.device, optimizer=opt,
                              seed=job.get("seed", 0))
    train = resolve_dataset(_load_recipe(job.get("train_recipe")), lcfg.get("train_path"))
    test = resolve_dataset(_load_recipe(job.get("test_recipe")), lcfg.get("test_path"))
    train_ds = net.make_dataset(train.get_x(), train.get_y(), seed=rank)
    test_ds = net.make_dataset(test.get_x(), test.get_y(), seed=rank, shuffle=False) if test is not None else None
    fcfg = FederationConfig(**job["federation"])
    fed = CollectiveFederation(comm, net, train_ds, fcfg, test_ds=test_ds, broadcast_initial=False)
    entity = metis_pb2.ServerEntity.FromString(bytes.fromhex(job["controller_hex"]))
    if rank == 0:
        client = GRPCControllerClient(entity, max_workers=1)
        try:
            lin = client.get_community_model_lineage(1)
            if len(lin.federated_models):
                fed.load_community_model(lin.federated_models[-1])
        finally:
            client.shutdown()
        fed.engine = RemoteCollectiveController(entity, fed.dataset_sizes,
                                                [(l["hostname"], l["port"]) for l in job["learners"]])
    fed.broadcast_initial_model()
    if job.get("resume_dir"):
        fed.resume(job["resume_dir"])
    for _ in range(int(job["rounds"])):
        rec = fed.run_round()
        if rank == 0:
            print(f"[collective] round {rec.global_iteration}: {rec.round_ms:.1f} ms "
                  f"(train {rec.train_ms:.1f}, aggregate {rec.aggregation_ms:.2f}) weights {rec.weights}",
                  flush=True)
    if job.get("checkpoint_dir"):
        fed.save_checkpoint(job["checkpoint_dir"])
    if rank == 0:
        st = net.state
        vals = st.to_numpy()
        fed.engine.snapshot_community([s.name for s in st.specs], [vals[s.name] for s in st.specs],
                                      [s.trainable for s in st.specs], fed.global_iteration)
        fed.engine.close()
    comm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
