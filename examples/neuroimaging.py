"""Neuroimaging federation (reference: examples/keras/neuroimaging.py:32-362,
BrainAge / Alzheimer's CNNs on TFRecord MRI volumes): brain-age regression
with the 3D CNN as a user PyTorch model (TorchModelDef), trained by learner
processes through the driver with the fused HIP optimizer.

    python examples/neuroimaging.py --learners 2 --rounds 3 [--device cpu] [--dims 2]
    python examples/neuroimaging.py --env examples/config/brainage/<config>.yaml [--rounds N] [--data-plane rccl]

``--env`` runs a federation environment file as written (protocol, rule,
batch size, local epochs, learner count and placement); ports, dataset paths
and, with ``--rounds``, the round budget are set here.

Volumes are synthetic with MRI-like shapes (no network / UK Biobank access);
--shape 91 109 91 gives the reference's full resolution.  As in the
reference (MRIScanGen.generate_tfrecord / load_dataset), every learner's
shard is serialized once to a TFRecord file of tf.train.Example rows
(image + label as raw bytes features) and the dataset recipe decodes it --
here through the framework's native TFRecord reader (datasets/tfrecord.py),
with ``--npz`` as the plain-numpy alternative.
"""
import argparse
import collections
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

from examples.models.torch_models import BrainAge2DCNN, BrainAge3DCNN, synthetic_volumes  # noqa: E402
from examples.utils.environment_generator import EnvGen  # noqa: E402
from metisfl_amd.driver.driver_session import DriverSession, free_port  # noqa: E402
from metisfl_amd.datasets import tfrecord  # noqa: E402
from metisfl_amd.models.model_dataset import ModelDatasetRegression  # noqa: E402

IMAGE_COLUMN, LABEL_COLUMN = "9dof_2mm_vol", "age_at_scan"  # the reference's BrainAge columns


def dataset_recipe(path):
    if path.endswith(".tfrecord"):
        cols = tfrecord.read_examples(path)
        return ModelDatasetRegression(cols[IMAGE_COLUMN], cols[LABEL_COLUMN])
    with np.load(path, allow_pickle=False) as z:
        return ModelDatasetRegression(z["x"], z["y"])


def save_shard(path_base: str, x, y, use_tfrecord: bool) -> str:
    if use_tfrecord:
        p = path_base + ".tfrecord"
        tfrecord.write_examples(p, collections.OrderedDict(
            [(IMAGE_COLUMN, x.astype(np.float32)), (LABEL_COLUMN, y.astype(np.float64))]))
        return p
    p = path_base + ".npz"
    np.savez(p, x=x, y=y)
    return p


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
    ap.add_argument("--npz", action="store_true", help="plain .npz shards instead of TFRecords")
    ap.add_argument("--env", default="", help="federation environment YAML (examples/config/brainage/*, ...)")
    ap.add_argument("--data-plane", default=None, choices=["grpc", "rccl"],
                    help="override the file's DataPlane: rccl trains the user model on the collective ranks "
                         "(models/torch_net.py)")
    a = ap.parse_args()
    shape = tuple(a.shape or ((32, 32, 32) if a.dims == 3 else (96, 96)))
    model = BrainAge3DCNN() if a.dims == 3 else BrainAge2DCNN()
    if a.env:
        from metisfl_amd.utils.fedenv_parser import FederationEnvironment
        env = FederationEnvironment(a.env)
        if "--rounds" in sys.argv:
            env.termination_signals.federation_rounds = a.rounds
    else:
        env = EnvGen(os.path.join(os.path.dirname(__file__), "config", "template.yaml")).generate_localhost(
            federation_rounds=a.rounds, learners_num=a.learners,
            gpu_devices=list(range(a.gpus)) if a.device != "cpu" else [-1])
        env.local_model_config.batch_size = 8
        env.local_model_config.local_epochs = 1
    if a.data_plane:
        env.data_plane = a.data_plane
    env.controller.grpc_servicer.port = free_port()
    d = a.workdir + "_data"
    os.makedirs(d, exist_ok=True)
    xte, yte = synthetic_volumes(16, shape, seed=999)
    test_p = save_shard(os.path.join(d, "test"), xte, yte, not a.npz)
    for i, l in enumerate(env.learners):
        x, y = synthetic_volumes(a.samples, shape, seed=i)
        p = save_shard(os.path.join(d, f"train_{i}"), x, y, not a.npz)
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
