"""Command lines that start the controller / learner processes (reference:
metisfl/utils/init_services_factory.py:4-85): every proto argument is
serialized and hex-encoded, exactly the CLI contract of
``python -m metisfl_amd.controller`` / ``python -m metisfl_amd.learner``."""
from __future__ import annotations

import sys


def _hex(pb) -> str:
    return pb.SerializeToString().hex()


class MetisInitServicesCmdFactory:

    def __init__(self, python: str | None = None):
        self.python = python or sys.executable

    def init_controller_target(self, controller_server_entity_pb, global_model_specs_pb,
                               communication_specs_pb, model_hyperparameters_pb, model_store_config_pb):
        return [self.python, "-m", "metisfl_amd.controller",
                "-e", _hex(controller_server_entity_pb),
                "-g", _hex(global_model_specs_pb),
                "-c", _hex(communication_specs_pb),
                "-m", _hex(model_hyperparameters_pb),
                "-s", _hex(model_store_config_pb)]

    def init_learner_target(self, learner_server_entity_pb, controller_server_entity_pb, he_scheme_pb,
                            model_dir, train_dataset="", validation_dataset="", test_dataset="",
                            train_dataset_recipe_pkl="", validation_dataset_recipe_pkl="",
                            test_dataset_recipe_pkl="", neural_engine="static", device=None,
                            credentials_dir=None, seed=0, fake_train_delay=0.0):
        cmd = [self.python, "-m", "metisfl_amd.learner",
               "-l", _hex(learner_server_entity_pb),
               "-c", _hex(controller_server_entity_pb),
               "-f", _hex(he_scheme_pb),
               "-e", neural_engine, "-m", model_dir,
               "-t", train_dataset or "", "-v", validation_dataset or "", "-s", test_dataset or "",
               "-u", train_dataset_recipe_pkl or "", "-w", validation_dataset_recipe_pkl or "",
               "-z", test_dataset_recipe_pkl or "", "--seed", str(seed)]
        if device:
            cmd += ["--device", device]
        if credentials_dir:
            cmd += ["--credentials_dir", credentials_dir]
        if fake_train_delay:
            cmd += ["--fake_train_delay", str(fake_train_delay)]
        return cmd
