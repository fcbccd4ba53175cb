"""FakeLearner model ops: no training, no evaluation -- echo the received
model back after a delay with fixed synthetic metadata (reference:
test/learner_notrain_noeval.py:16-198, metadata 1, 100, 1, 100.0, 100.0).
Used to test controller orchestration at scale on CPU."""
from __future__ import annotations

import time

from metisfl_amd.models.model_ops import ModelOps, TaskCancelled
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M


class EchoModelOps(ModelOps):
    def __init__(self, train_delay_s: float = 0.0):
        super().__init__(None)
        self.delay = train_delay_s
        self.model_pb = None

    def set_model_from_pb(self, model_pb):
        self.model_pb = model_pb

    def get_model_weights(self):
        return [], [], []

    def set_model_weights(self, names, arrays):
        pass

    def train_model(self, train_dataset, learning_task_pb, hyperparameters_pb, validation_dataset=None,
                    test_dataset=None, verbose=False, cancel_event=None):
        end = time.time() + self.delay
        while time.time() < end:
            if cancel_event is not None and cancel_event.is_set():
                raise TaskCancelled()
            time.sleep(min(0.01, max(0.0, end - time.time())))
        meta = M.construct_task_execution_metadata_pb(learning_task_pb.global_iteration, None, 1, 100, 1,
                                                      100.0, 100.0)
        return M.construct_completed_learning_task_pb(self.model_pb, meta, "")

    def evaluate_model(self, dataset, batch_size, metrics=(), verbose=False, model_pb=None):
        return {}
