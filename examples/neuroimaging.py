"""Neuroimaging federation (reference: examples/keras/neuroimaging.py:32-362,
BrainAge / Alzheimer's CNNs on TFRecord MRI volumes): brain-age regression
with the 3D CNN as a user PyTorch model (TorchModelDef), trained by learner
processes through the driver with the fused HIP optimizer.

    python examples/neuroimaging.py --learners 2 --rounds 3 [--device cpu] [--dims 2]

Volumes are synthetic with MRI-like shapes (no network / UK Biobank access);
--shape 91 109 91 gives the reference's full resolution.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from examples.models.torch_models import BrainAge2DCNN, BrainAge3DCNN, synthetic_volumes  # noqa: E402
from examples.utils.environment_generator import EnvGen  # noqa: E402
from metisfl_amd.driver.driver_session import DriverSession, free_port  # noqa: E402
from metisfl_amd.models.model_dataset import ModelDatasetRegression  # noqa: E402


def dataset_recipe(path):
    with np.load(path, allow_pickle=False) as z:
        return ModelDatasetRegression(z["x"], z["y"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--learners", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dims", type=int, default=3, choices=(2, 3))
    ap.add_argument("--shape", type=int, nargs="+", default=None)
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--device", default=None)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--workdir", default="/tmp/metis_amd_neuroimaging")
    a = ap.parse_args()
    shape = tuple(a.shape or ((32, 32, 32) if a.dims == 3 else (96, 96)))
    model = BrainAge3DCNN() if a.dims == 3 else BrainAge2DCNN()
    env = EnvGen(os.path.join(os.path.dirname(__file__), "config", "template.yaml")).generate_localhost(
        federation_rounds=a.rounds, learners_num=a.learners,
        gpu_devices=list(range(a.gpus)) if a.device != "cpu" else [-1])
    env.controller.grpc_servicer.port = free_port()
    env.local_model_config.batch_size = 8
    env.local_model_config.local_epochs = 1
    d = a.workdir + "_data"
    os.makedirs(d, exist_ok=True)
    xte, yte = synthetic_volumes(16, shape, seed=999)
    test_p = os.path.join(d, "test.npz")
    np.savez(test_p, x=xte, y=yte)
    for i, l in enumerate(env.learners):
        x, y = synthetic_volumes(a.samples, shape, seed=i)
        p = os.path.join(d, f"train_{i}.npz")
        np.savez(p, x=x, y=y)
        l.dataset_configs.train_dataset_path = p
        l.dataset_configs.test_dataset_path = test_p
        l.grpc_servicer.port = free_port()
    sess = DriverSession(env, model, dataset_recipe, None, dataset_recipe, working_dir=a.workdir, device=a.device)
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
