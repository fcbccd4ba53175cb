"""CIFAR-10 federation through the driver (reference:
examples/keras/cifar10.py with examples/config/cifar10/*.yaml): IID shards
written to .npz, learners trained by the driver's learner processes (or, with
``DataPlane: rccl``, by the collective ranks), statistics dumped to
experiment.json.

    python examples/cifar10.py --env examples/config/cifar10/test_localhost_synchronous_fedprox_with_fhe.yaml
    python examples/cifar10.py --learners 4 --rounds 5 [--device cpu] [--model resnet18]

``--env`` runs a federation environment file as written (protocol,
aggregation rule, optimizer -- FedProx's proximal term included --, CKKS,
batch size, local epochs, learner count and placement); ports, dataset paths
and, with ``--rounds``, the round budget are set here.  ``--one-gpu`` places
every learner on GPU 0 (the files spread them over GPUs 0-7).

Data is synthetic with CIFAR-10 shapes (no network access here).
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from examples.utils.environment_generator import EnvGen  # noqa: E402
from metisfl_amd.datasets import DataPartitioning, synthetic_classification  # noqa: E402
from metisfl_amd.driver.driver_session import DriverSession, free_port  # noqa: E402
from metisfl_amd.models.model_dataset import ModelDatasetClassification  # noqa: E402
from metisfl_amd.models.model_def import StaticModelDef  # noqa: E402


def dataset_recipe(path):
    with np.load(path, allow_pickle=False) as z:
        return ModelDatasetClassification(z["x"], z["y"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="", help="federation environment YAML (examples/config/cifar10/*)")
    ap.add_argument("--learners", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--device", default=None)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--one-gpu", action="store_true", help="every learner on GPU 0")
    ap.add_argument("--model", default="cifar_cnn", choices=["cifar_cnn", "resnet18"])
    ap.add_argument("--width-mult", type=float, default=1.0, help="ResNet-18 width (resnet18 only)")
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--workdir", default="/tmp/metis_amd_cifar10")
    a = ap.parse_args()
    xtr, ytr = synthetic_classification("cifar10", a.train_size, seed=0)
    xte, yte = synthetic_classification("cifar10", a.test_size, seed=1)
    if a.env:
        from metisfl_amd.utils.fedenv_parser import FederationEnvironment
        env = FederationEnvironment(a.env)
        if "--rounds" in sys.argv:
            env.termination_signals.federation_rounds = a.rounds
    else:
        env = EnvGen(os.path.join(os.path.dirname(__file__), "config", "template.yaml")).generate_localhost(
            federation_rounds=a.rounds, learners_num=a.learners,
            gpu_devices=list(range(a.gpus)) if a.device != "cpu" else [-1])
    if a.one_gpu:
        for l in env.learners:
            l.devices = l.cuda_devices = [0]
    n = len(env.learners)
    xs, ys = DataPartitioning(xtr, ytr, n).iid_partition()
    d = a.workdir + "_data"
    os.makedirs(d, exist_ok=True)
    env.controller.grpc_servicer.port = free_port()
    test_p = os.path.join(d, "test.npz")
    np.savez(test_p, x=xte, y=yte)
    for i, l in enumerate(env.learners):
        p = os.path.join(d, f"train_{i}.npz")
        np.savez(p, x=xs[i], y=ys[i])
        l.dataset_configs.train_dataset_path = p
        l.dataset_configs.test_dataset_path = test_p
        l.grpc_servicer.port = free_port()
    kw = {"width_mult": a.width_mult} if a.model == "resnet18" and a.width_mult != 1.0 else {}
    sess = DriverSession(env, StaticModelDef(a.model, **kw), dataset_recipe, None, dataset_recipe,
                         working_dir=a.workdir, device=a.device)
    try:
        sess.initialize_federation()
        sess.monitor_federation(request_every_secs=1)
    finally:
        sess.shutdown_federation()
    stats = sess.get_federation_statistics()
    with open(os.path.join(a.workdir, "experiment.json"), "w") as f:
        json.dump(stats, f)
    print("statistics written to", os.path.join(a.workdir, "experiment.json"))


if __name__ == "__main__":
    main()
