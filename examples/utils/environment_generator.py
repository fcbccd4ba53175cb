"""Localhost federation environments (reference:
examples/utils/environment_generator.py:8-37): N learners on consecutive
ports, GPUs assigned round-robin."""
from __future__ import annotations

import copy
import itertools
import os

from metisfl_amd.utils.fedenv_parser import FederationEnvironment


class EnvGen:
    def __init__(self, template_filepath: str | None = None):
        self.template_filepath = template_filepath or os.path.join(
            os.path.dirname(__file__), "..", "config", "template.yaml")

    def generate_localhost(self, federation_rounds=10, learners_num=10, gpu_devices=(0,),
                           gpu_assignment="round_robin") -> FederationEnvironment:
        if gpu_assignment != "round_robin":
            raise RuntimeError("Only round-robin GPU assignment is supported.")
        env = FederationEnvironment(self.template_filepath)
        env.termination_signals.federation_rounds = federation_rounds
        tmpl = env.learners.learners[0]
        devs = itertools.cycle(gpu_devices)
        env.learners.learners = []
        for k in range(learners_num):
            l = copy.deepcopy(tmpl)
            l.learner_id = f"localhost:{k}"
            d = next(devs)
            l.devices = l.cuda_devices = [] if d is None or d < 0 else [int(d)]
            l.grpc_servicer.port = int(tmpl.grpc_servicer.port + k)
            env.learners.learners.append(l)
        return env
