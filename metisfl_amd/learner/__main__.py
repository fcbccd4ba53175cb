"""``python -m metisfl_amd.learner`` -- learner process entry point (reference:
metisfl/learner/__main__.py:10-137; same hex-encoded proto arguments).

  -e/--neural_engine   "static" (built-in family from <model_dir>/model_definition.json,
                       hipGraph executor), "torch" (cloudpickled TorchModelDef in
                       <model_dir>/model_def.pkl) or "fake" (echo learner, no compute)
  -t/-v/-s             .npz dataset files (x, y); loaded with allow_pickle=False
  -u/-w/-z             dataset recipes written by the driver (cloudpickle)
  --device             cuda (default when a GPU is visible) or cpu
"""
from __future__ import annotations

import argparse
import os

from metisfl_amd.learner.learner import Learner
from metisfl_amd.learner.learner_servicer import LearnerServicer
from metisfl_amd.proto import metis_pb2


def _pb(hexstr, cls):
    pb = cls()
    if hexstr:
        pb.ParseFromString(bytes.fromhex(hexstr))
    return pb


def _recipe(path):
    if not path:
        return None
    import cloudpickle  # recipes are produced by our own driver
    with open(path, "rb") as f:
        return cloudpickle.load(f)


def build_model_ops(engine: str, model_dir: str, device: str, seed: int = 0, fake_delay: float = 0.0):
    if engine == "fake":
        from metisfl_amd.learner.fake import EchoModelOps
        return EchoModelOps(fake_delay)
    if engine == "torch":
        from metisfl_amd.models.torch_ops import TorchModelOps
        import cloudpickle
        with open(os.path.join(model_dir, "model_def.pkl"), "rb") as f:
            model_def = cloudpickle.load(f)
        return TorchModelOps(model_def, device=device, seed=seed)
    from metisfl_amd.models.model_def import StaticModelDef
    from metisfl_amd.models.model_ops import StaticModelOps
    return StaticModelOps(StaticModelDef.load(model_dir), device=device, seed=seed)


def main(argv=None):
    p = argparse.ArgumentParser(prog="metisfl_amd.learner")
    p.add_argument("-l", "--learner_server_entity_protobuff_serialized_hexadecimal", default="")
    p.add_argument("-c", "--controller_server_entity_protobuff_serialized_hexadecimal", default="")
    p.add_argument("-f", "--he_scheme_protobuff_serialized_hexadecimal", default="")
    p.add_argument("-e", "--neural_engine", default="static")
    p.add_argument("-m", "--model_dir", default="")
    p.add_argument("-t", "--train_dataset", default="")
    p.add_argument("-v", "--validation_dataset", default="")
    p.add_argument("-s", "--test_dataset", default="")
    p.add_argument("-u", "--train_dataset_recipe", default="")
    p.add_argument("-w", "--validation_dataset_recipe", default="")
    p.add_argument("-z", "--test_dataset_recipe", default="")
    p.add_argument("--device", default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--credentials_dir", default=None)
    p.add_argument("--fake_train_delay", type=float, default=0.0)
    a = p.parse_args(argv)

    device = a.device
    if device is None:
        import torch
        device = "cuda" if torch.cuda.is_available() else "cpu"
    learner_entity = _pb(a.learner_server_entity_protobuff_serialized_hexadecimal, metis_pb2.ServerEntity)
    controller_entity = _pb(a.controller_server_entity_protobuff_serialized_hexadecimal, metis_pb2.ServerEntity)
    he_pb = _pb(a.he_scheme_protobuff_serialized_hexadecimal, metis_pb2.HESchemeConfig)
    ops = build_model_ops(a.neural_engine, a.model_dir, device, a.seed, a.fake_train_delay)
    learner = Learner(learner_entity, controller_entity, ops,
                      train_dataset=_recipe(a.train_dataset_recipe) or a.train_dataset or None,
                      validation_dataset=_recipe(a.validation_dataset_recipe) or a.validation_dataset or None,
                      test_dataset=_recipe(a.test_dataset_recipe) or a.test_dataset or None,
                      he_scheme_pb=he_pb, learner_credentials_fp=a.credentials_dir,
                      dataset_paths={"train": a.train_dataset, "validation": a.validation_dataset,
                                     "test": a.test_dataset})
    servicer = LearnerServicer(learner, servicer_workers=5)
    servicer.init_servicer()
    servicer.wait_servicer()


if __name__ == "__main__":
    main()
