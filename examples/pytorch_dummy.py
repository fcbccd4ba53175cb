"""PyTorch user-model federation (reference: examples/pytorch/dummy.py:18-103,
the Ionosphere MLP of examples/pytorch/models/mlp.py): a user ``nn.Module``
(a TorchModelDef) federated through the driver.

    python examples/pytorch_dummy.py [--learners 3] [--rounds 5] [--protocol Asynchronous]
                                     [--data-plane rccl] [--device cpu]

``--data-plane grpc`` (the reference's path): learner processes train the
module and ship it through the controller every round.  ``--data-plane
rccl``: the collective ranks train it (models/torch_net.py: the module's
parameters and buffers are views of one flat buffer, the fused HIP optimizer
updates it, FedAvg is one weighted sum + all-reduce, the asynchronous
protocol FedRec over point-to-point transfers).

The reference downloads the 351-row Ionosphere CSV (34 radar features, a
good / bad label) and splits 10 % off for testing; with no network here the
rows are synthetic of the same shape: features in [-1, 1], the label a fixed
random linear rule of them.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from examples.models.torch_models import IonosphereMLP  # noqa: E402
from examples.utils.environment_generator import EnvGen  # noqa: E402
from metisfl_amd.driver.driver_session import DriverSession, free_port  # noqa: E402
from metisfl_amd.models.model_dataset import ModelDatasetClassification  # noqa: E402


def ionosphere_like(n: int = 351, seed: int = 0):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1.0, 1.0, (n, 34)).astype(np.float32)
    w = np.random.default_rng(1234).standard_normal(34)
    y = (x @ w > 0).astype(np.int64)
    return x, y


def dataset_recipe(path):
    with np.load(path, allow_pickle=False) as z:
        return ModelDatasetClassification(z["x"], z["y"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--learners", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--protocol", default="Synchronous", choices=["Synchronous", "SemiSynchronous", "Asynchronous"])
    ap.add_argument("--data-plane", default="rccl", choices=["grpc", "rccl"])
    ap.add_argument("--device", default=None)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--workdir", default="/tmp/metis_amd_pytorch_dummy")
    a = ap.parse_args()
    env = EnvGen(os.path.join(os.path.dirname(__file__), "config", "template.yaml")).generate_localhost(
        federation_rounds=a.rounds, learners_num=a.learners,
        gpu_devices=list(range(a.gpus)) if a.device != "cpu" else [-1])
    env.data_plane = a.data_plane
    env.communication_protocol.name = a.protocol
    env.communication_protocol.is_asynchronous = a.protocol == "Asynchronous"
    env.communication_protocol.is_synchronous = a.protocol == "Synchronous"
    env.communication_protocol.is_semi_synchronous = a.protocol == "SemiSynchronous"
    env.local_model_config.batch_size = 32
    env.local_model_config.local_epochs = 1
    env.controller.grpc_servicer.port = free_port()
    x, y = ionosphere_like()
    n_test = round(0.1 * len(x))
    d = a.workdir + "_data"
    os.makedirs(d, exist_ok=True)
    test_p = os.path.join(d, "test.npz")
    np.savez(test_p, x=x[:n_test], y=y[:n_test])
    parts = np.array_split(np.arange(n_test, len(x)), a.learners)  # IID shards of the training rows
    for i, l in enumerate(env.learners):
        p = os.path.join(d, f"train_{i}.npz")
        np.savez(p, x=x[parts[i]], y=y[parts[i]])
        l.dataset_configs.train_dataset_path = p
        l.dataset_configs.test_dataset_path = test_p
        l.grpc_servicer.port = free_port()
    sess = DriverSession(env, IonosphereMLP(), dataset_recipe, None, dataset_recipe, working_dir=a.workdir,
                         device=a.device)
    try:
        sess.initialize_federation()
        sess.monitor_federation(request_every_secs=1)
    finally:
        sess.shutdown_federation()
    with open(os.path.join(a.workdir, "experiment.json"), "w") as f:
        json.dump(sess.get_federation_statistics(), f)
    print("statistics written to", os.path.join(a.workdir, "experiment.json"))


if __name__ == "__main__":
    main()
