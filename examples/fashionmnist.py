"""FashionMNIST federation through the driver (reference:
examples/keras/fashionmnist.py:17-97): IID shards written to .npz, one
learner process per shard (GPU round-robin), FashionMNIST FC on the static
HIP executor, statistics dumped to experiment.json.

    python examples/fashionmnist.py --learners 4 --rounds 5 [--device cpu]
    python examples/fashionmnist.py --env examples/config/fashionmnist/<config>.yaml [--rounds N]

``--env`` runs one of the federation environment files as written (protocol,
aggregation rule, CKKS, data plane, device placement, learner count); only
the ports, dataset paths and, with ``--rounds``, the round budget are set here.

Data is synthetic with FashionMNIST shapes (no network access here); pass
--npz path/with/x_train,y_train,x_test,y_test arrays to use real data.
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
    ap.add_argument("--learners", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--device", default=None)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--npz", default="")
    ap.add_argument("--workdir", default="/tmp/metis_amd_fashionmnist")
    ap.add_argument("--env", default="", help="federation environment YAML (examples/config/fashionmnist/*)")
    ap.add_argument("--train-size", type=int, default=6000)
    a = ap.parse_args()
    if a.npz:
        with np.load(a.npz, allow_pickle=False) as z:
            xtr, ytr, xte, yte = z["x_train"], z["y_train"], z["x_test"], z["y_test"]
    else:
        xtr, ytr = synthetic_classification("fashionmnist", a.train_size, seed=0)
        xte, yte = synthetic_classification("fashionmnist", 1000, seed=1)
    if a.env:
        from metisfl_amd.utils.fedenv_parser import FederationEnvironment
        env = FederationEnvironment(a.env)
        if "--rounds" in sys.argv:
            env.termination_signals.federation_rounds = a.rounds
    else:
        env = EnvGen(os.path.join(os.path.dirname(__file__), "config", "template.yaml")).generate_localhost(
            federation_rounds=a.rounds, learners_num=a.learners,
            gpu_devices=list(range(a.gpus)) if a.device != "cpu" else [-1])
    n = len(env.learners)
    xs, ys = DataPartitioning(xtr / max(1.0, float(np.abs(xtr).max())), ytr, n).iid_partition()
    os.makedirs(a.workdir + "_data", exist_ok=True)
    env.controller.grpc_servicer.port = free_port()
    test_p = os.path.join(a.workdir + "_data", "test.npz")
    np.savez(test_p, x=xte, y=yte)
    for i, l in enumerate(env.learners):
        p = os.path.join(a.workdir + "_data", f"train_{i}.npz")
        np.savez(p, x=xs[i], y=ys[i])
        l.dataset_configs.train_dataset_path = p
        l.dataset_configs.test_dataset_path = test_p
        l.grpc_servicer.port = free_port()
    sess = DriverSession(env, StaticModelDef("fashion_mnist_fc"), dataset_recipe, None, dataset_recipe,
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
