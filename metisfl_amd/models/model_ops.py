"""Learner-side model operations: weights <-> Model proto, local training
task, evaluation (reference: metisfl/models/model_ops.py:18-144 and
keras/keras_model_ops.py:15-283).

Differences by design (MI355X-first):
  * the model is PERSISTENT in device memory across rounds -- no SavedModel
    reload per task, no subprocess per task (keras_model_ops.py:117-197
    reloads and re-saves the model every task);
  * a training task is ``num_local_updates`` replays of the captured step
    graph (exact step budget; the reference's StepCounter runs total+1
    batches, callbacks/step_counter.py:39-45) and ``completed_batches`` is
    what actually ran;
  * evaluation of a received community model runs on a separate eval-only
    instance, so it can overlap with training on the same GPU.
"""
from __future__ import annotations

import abc
import math
import threading
import time

import numpy as np
import torch

from metisfl_amd.models.model_dataset import ModelDataset
from metisfl_amd.models.model_proto_factory import ModelProtoFactory
from metisfl_amd.ops.optim import OptimizerSpec
from metisfl_amd.utils.formatting import DictionaryFormatter
from metisfl_amd.utils.metis_logger import MetisLogger
from metisfl_amd.utils.tensor_codec import model_to_arrays


class TaskCancelled(Exception):
    pass


class ModelOps(abc.ABC):
    def __init__(self, he_scheme=None):
        self.he_scheme = he_scheme

    # -- weights -----------------------------------------------------------------
    def get_model_weights_from_variables_pb(self, model_pb):
        names, arrays, _ = model_to_arrays(model_pb, self.he_scheme)
        return names, arrays

    @abc.abstractmethod
    def get_model_weights(self):
        """-> (names, trainables, arrays)"""

    @abc.abstractmethod
    def set_model_weights(self, names, arrays):
        ...

    def set_model_from_pb(self, model_pb):
        names, arrays = self.get_model_weights_from_variables_pb(model_pb)
        if names:
            self.set_model_weights(names, arrays)

    # -- tasks ---------------------------------------------------------------------
    @abc.abstractmethod
    def train_model(self, train_dataset: ModelDataset, learning_task_pb, hyperparameters_pb,
                    validation_dataset=None, test_dataset=None, verbose=False, cancel_event=None):
        """-> CompletedLearningTask proto"""

    @abc.abstractmethod
    def evaluate_model(self, dataset: ModelDataset, batch_size: int, metrics=(), verbose=False) -> dict:
        ...

    def infer_model(self, dataset: ModelDataset, batch_size: int, verbose=False):
        raise NotImplementedError

    def cleanup(self):
        pass


class StaticModelOps(ModelOps):
    """ModelOps over a static-graph network (models/net.py)."""

    def __init__(self, model_def, device="cuda", seed: int = 0, he_scheme=None,
                 eval_steps_cap: int | None = None):
        super().__init__(he_scheme)
        self.model_def = model_def
        self.device = torch.device(device)
        self.seed = seed
        self.nets: dict[int, object] = {}      # training instances by batch size
        self.eval_nets: dict[int, object] = {}  # eval-only instances by batch size
        self.datasets: dict[tuple, object] = {}
        self.current = None
        self.eval_steps_cap = eval_steps_cap
        self.lock = threading.Lock()

    # -- instances -------------------------------------------------------------------------
    def _net(self, batch_size: int, eval_only=False):
        pool = self.eval_nets if eval_only else self.nets
        if batch_size not in pool:
            net = self.model_def.get_model(batch_size=batch_size, device=self.device, seed=self.seed)
            if not eval_only and self.current is not None:
                net.state.model32.copy_(self.current.state.model32)
                net.state.refresh_bf16()
            pool[batch_size] = net
        return pool[batch_size]

    def _model(self):
        if self.current is None:
            self.current = self._net(getattr(self.model_def, "default_batch", 32))
        return self.current

    def _device_dataset(self, net, ds: ModelDataset, key: str, shuffle: bool):
        k = (id(net), key, id(ds))
        if k not in self.datasets:
            y = ds.get_y()
            self.datasets[k] = net.make_dataset(np.asarray(ds.get_x()), np.asarray(y), seed=self.seed,
                                                shuffle=shuffle)
        return self.datasets[k]

    # -- weights ---------------------------------------------------------------------------------
    def get_model_weights(self):
        st = self._model().state
        vals = st.to_numpy()
        names = [s.name for s in st.specs]
        return names, [s.trainable for s in st.specs], [vals[n] for n in names]

    def _load(self, net, names, arrays):
        st = net.state
        if set(names) == set(st.by_name):
            st.load_numpy(dict(zip(names, arrays)))
        elif len(names) == len(st.specs):  # positional (models exported by other frameworks)
            st.load_numpy({s.name: a for s, a in zip(st.specs, arrays)})
        else:
            raise ValueError(f"model has {len(names)} variables, expected {len(st.specs)}")

    def set_model_weights(self, names, arrays):
        net = self._model()
        self._load(net, names, arrays)
        net.state.set_anchor()  # FedProx proximal anchor = received community model

    # -- training -----------------------------------------------------------------------------------
    def train_model(self, train_dataset, learning_task_pb, hyperparameters_pb, validation_dataset=None,
                    test_dataset=None, verbose=False, cancel_event=None):
        B = int(hyperparameters_pb.batch_size) or 32
        with self.lock:
            prev = self._model()
            net = self._net(B)
            if net is not prev:
                net.state.model32.copy_(prev.state.model32)
                net.state.refresh_bf16()
                net.state.set_anchor()
                self.current = net
            if hyperparameters_pb.HasField("optimizer"):
                net.state.set_optimizer(OptimizerSpec.from_proto(hyperparameters_pb.optimizer))
            ds = self._device_dataset(net, train_dataset, "train", shuffle=True)
            total = int(learning_task_pb.num_local_updates)
            spe = ds.steps_per_epoch
            train_stats = {"loss": [], "accuracy": []}
            done = 0
            t0 = time.perf_counter()
            while done < total:
                if cancel_event is not None and cancel_event.is_set():
                    raise TaskCancelled()
                chunk = min(spe - (done % spe), total - done)
                net.reset_train_stats()
                net.train_steps(ds, chunk, step_offset=done)
                done += chunk
                if done % spe == 0 or done == total:
                    s = net.train_stats()
                    train_stats["loss"].append(s["loss"])
                    train_stats["accuracy"].append(s["accuracy"])
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            train_ms = (time.perf_counter() - t0) * 1e3
            val_stats = self.evaluate_model(validation_dataset, B) if _nonempty(validation_dataset) else {}
            test_stats = self.evaluate_model(test_dataset, B) if _nonempty(test_dataset) else {}
            names, trainable, values = self.get_model_weights()
        ms_batch = train_ms / max(1, done)
        msg = ModelProtoFactory.CompletedLearningTaskProtoMessage(
            names, trainable, values, train_stats, completed_epochs=done / spe,
            global_iteration=learning_task_pb.global_iteration, validation_stats=val_stats,
            test_stats=test_stats, completes_batches=done, batch_size=B,
            processing_ms_per_epoch=ms_batch * spe, processing_ms_per_batch=ms_batch)
        if verbose:
            MetisLogger.info("trained %d steps in %.1f ms (%.3f ms/step)", done, train_ms, ms_batch)
        return msg.construct_completed_learning_task_pb(he_scheme=self.he_scheme)

    # -- evaluation ------------------------------------------------------------------------------------
    def evaluate_model(self, dataset, batch_size: int, metrics=(), verbose=False, model_pb=None) -> dict:
        """Loss / accuracy of the current model (or of ``model_pb`` on the
        eval-only instance) on ``dataset``."""
        if not _nonempty(dataset):
            return {}
        B = int(batch_size) or 32
        if model_pb is not None:
            net = self._net(B, eval_only=True)
            names, arrays = self.get_model_weights_from_variables_pb(model_pb)
            self._load(net, names, arrays)
        else:
            net = self._model()
        ds = self._device_dataset(net, dataset, "eval", shuffle=False)
        res = net.evaluate(ds, self.eval_steps_cap)
        if metrics:
            keep = {m.lower() for m in metrics} | {"loss"}
            res = {k: v for k, v in res.items() if k in keep}
        return res


def _nonempty(ds) -> bool:
    return ds is not None and ds.get_x() is not None and ds.get_size() > 0
