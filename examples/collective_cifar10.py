"""On-node federation over RCCL (one learner process per GPU): CIFAR-10-shaped
IID shards, ResNet-18 (or CifarCNN), synchronous FedAvg by scaled all-reduce,
per-round metrics from the native controller, periodic checkpoints.

    torchrun --standalone --nproc-per-node 8 examples/collective_cifar10.py --rounds 10

Resume after a failure with --resume <checkpoint dir>.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from metisfl_amd.datasets import synthetic_classification  # noqa: E402
from metisfl_amd.models.model_def import StaticModelDef  # noqa: E402
from metisfl_amd.ops.optim import OptimizerSpec  # noqa: E402
from metisfl_amd.parallel.comm import Comm  # noqa: E402
from metisfl_amd.parallel.engine_bridge import CollectiveController  # noqa: E402
from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18", choices=["resnet18", "cifar_cnn"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--local-epochs", type=int, default=4)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--lr", type=float, default=0.005)
    ap.add_argument("--momentum", type=float, default=0.75)
    ap.add_argument("--protocol", default="synchronous", choices=["synchronous", "semi_synchronous"])
    ap.add_argument("--checkpoint-every", type=int, default=0)
    ap.add_argument("--checkpoint-dir", default="/tmp/metis_amd_ckpt")
    ap.add_argument("--resume", default="")
    ap.add_argument("--out", default="/tmp/metis_amd_collective.json")
    a = ap.parse_args()
    comm = Comm()
    n = comm.world
    sizes = [a.train_size // n + (1 if r < a.train_size % n else 0) for r in range(n)]
    x, y = synthetic_classification("cifar10", sizes[comm.rank], seed=comm.rank)
    xt, yt = synthetic_classification("cifar10", 1000, seed=10_000 + comm.rank)
    net = StaticModelDef(a.model).get_model(batch_size=a.batch, device=comm.device, seed=7,
                                            optimizer=OptimizerSpec("momentum_sgd", a.lr, momentum=a.momentum))
    train_ds = net.make_dataset(x, y, seed=comm.rank)
    test_ds = net.make_dataset(xt, yt, shuffle=False)
    cfg = FederationConfig(protocol=a.protocol, batch_size=a.batch, local_epochs=a.local_epochs)
    engine = CollectiveController(cfg, sizes) if comm.rank == 0 else None
    fed = CollectiveFederation(comm, net, train_ds, cfg, test_ds=test_ds, engine=engine)
    if a.resume:
        fed.resume(a.resume)
    while fed.global_iteration < a.rounds:
        rec = fed.run_round()
        if comm.rank == 0:
            test_acc = float(np.nanmean(rec.learner_meta[:, 9]))
            print(f"round {rec.global_iteration}: {rec.round_ms:.0f} ms, mean test accuracy {test_acc:.3f}",
                  flush=True)
        if a.checkpoint_every and fed.global_iteration % a.checkpoint_every == 0:
            # versioned: <dir>/round_<gi>/ + <dir>/LATEST (parallel/checkpoint.py); --resume <dir>
            fed.save_checkpoint(a.checkpoint_dir, block=False)
    fed.flush_checkpoints()
    if comm.rank == 0:
        from google.protobuf.json_format import MessageToDict
        with open(a.out, "w") as f:
            json.dump({"federation_runtime_metadata": MessageToDict(engine.runtime_metadata(0)),
                       "rounds": [r.to_json() for r in fed.history]}, f)
    comm.close()


if __name__ == "__main__":
    torch.set_num_threads(max(1, torch.get_num_threads()))
    main()
    from metisfl_amd.utils.launch import exit_process
    exit_process(0)  # no interpreter finalisation behind live c10d threads (utils/launch.py)
