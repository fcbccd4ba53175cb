"""CompletedLearningTask / ModelEvaluation builders (reference:
metisfl/models/model_proto_factory.py:9-114).  Per-epoch evaluations are
emitted when there is one value per completed epoch, otherwise only the last
one (same convention as the reference)."""
from __future__ import annotations

import math

from metisfl_amd.utils.formatting import DictionaryFormatter
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
from metisfl_amd.utils.proto_messages_factory import ModelProtoMessages as MM


def _epoch_evaluations(collection: dict, completed_epochs: float):
    n_ep = int(math.ceil(completed_epochs))
    lens = [len(v) for v in collection.values()]
    out = []
    if all(n == n_ep for n in lens):
        for e in range(n_ep):
            stats = DictionaryFormatter.stringify({k: v[e] for k, v in collection.items()})
            out.append(M.construct_epoch_evaluation_pb(e + 1, M.construct_model_evaluation_pb(stats)))
    else:
        stats = DictionaryFormatter.stringify({k: v[-1] for k, v in collection.items()})
        out.append(M.construct_epoch_evaluation_pb(n_ep, M.construct_model_evaluation_pb(stats)))
    return out


class ModelProtoFactory:

    class CompletedLearningTaskProtoMessage:
        def __init__(self, weights_names, weights_trainable, weights_values, train_stats,
                     completed_epochs, global_iteration, validation_stats=None, test_stats=None,
                     completes_batches=0, batch_size=0, processing_ms_per_epoch=0.0,
                     processing_ms_per_batch=0.0):
            self.names, self.trainable, self.values = weights_names, weights_trainable, weights_values
            self.train_stats = DictionaryFormatter.listify_values(train_stats or {})
            self.validation_stats = DictionaryFormatter.listify_values(validation_stats or {})
            self.test_stats = DictionaryFormatter.listify_values(test_stats or {})
            self.completed_epochs = completed_epochs
            self.global_iteration = global_iteration
            self.completed_batches = completes_batches
            self.batch_size = batch_size
            self.ms_per_epoch = processing_ms_per_epoch
            self.ms_per_batch = processing_ms_per_batch

        def construct_task_execution_metadata_pb(self):
            ev = M.construct_task_evaluation_pb(
                _epoch_evaluations(self.train_stats, self.completed_epochs),
                _epoch_evaluations(self.validation_stats, self.completed_epochs),
                _epoch_evaluations(self.test_stats, self.completed_epochs))
            return M.construct_task_execution_metadata_pb(
                self.global_iteration, ev, self.completed_epochs, self.completed_batches,
                self.batch_size, self.ms_per_epoch, self.ms_per_batch)

        def construct_completed_learning_task_pb(self, aux_metadata="", he_scheme=None):
            model_pb = MM.construct_model_pb_from_np(self.values, self.names, self.trainable, he_scheme)
            return M.construct_completed_learning_task_pb(
                model_pb, self.construct_task_execution_metadata_pb(), aux_metadata)

    class ModelEvaluationProtoMessage:
        def __init__(self, metric_values):
            self.metric_values = metric_values

        def construct_model_evaluation_pb(self):
            return M.construct_model_evaluation_pb(DictionaryFormatter.stringify(self.metric_values))
