"""The learner runtime (reference: metisfl/learner/learner.py:21-417).

One persistent learner per GPU.  The reference runs every train / eval task
in a freshly spawned process that reloads the model from disk
(learner.py:77-89, 338-354); here the model, optimizer state and the data
shard stay resident in device memory for the learner's whole life, and a
task is a sequence of hipGraph replays on a worker thread:

  * ``run_learning_task`` cancels the in-flight task (reference semantics:
    a new RunTask preempts, learner.py:376-396), loads the community model,
    trains, and reports the CompletedLearningTask to the controller from the
    completion callback (MarkTaskCompleted, non-blocking);
  * ``run_evaluation_task`` evaluates the received model on an eval-only
    instance (concurrent with training) and blocks until done;
  * credentials (learner id / auth token) are persisted so a restarted
    learner rejoins with ALREADY_EXISTS (learner.py:96-103).
"""
from __future__ import annotations

import os
import threading
from concurrent import futures
from inspect import signature

from metisfl_amd.learner.he import he_scheme_from_config
from metisfl_amd.models.model_dataset import ModelDataset, ModelDatasetClassification, ModelDatasetRegression
from metisfl_amd.models.model_ops import ModelOps, TaskCancelled
from metisfl_amd.proto import learner_pb2, metis_pb2
from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
from metisfl_amd.utils.metis_logger import MetisLogger
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M


def resolve_dataset(spec, path=None, default_class=None) -> ModelDataset | None:
    """A dataset given as a ModelDataset, a recipe callable (``recipe()`` or
    ``recipe(path)``), an ``.npz`` path (x, y; loaded with allow_pickle=False)
    or None (-> ``default_class()`` if given)."""
    if isinstance(spec, ModelDataset):
        return spec
    if callable(spec):
        ds = spec(path) if len(signature(spec).parameters) > 0 and path else spec()
        assert isinstance(ds, ModelDataset), "dataset recipes must return a ModelDataset"
        return ds
    if isinstance(spec, str) and spec.endswith(".npz"):
        import numpy as np
        with np.load(spec, allow_pickle=False) as z:
            return ModelDatasetClassification(z["x"], z["y"])
    return default_class() if default_class is not None else None


class Learner:

    def __init__(self, learner_server_entity, controller_server_entity, model_ops: ModelOps,
                 train_dataset, validation_dataset=None, test_dataset=None, he_scheme_pb=None,
                 learner_credentials_fp: str | None = None, dataset_paths: dict | None = None):
        self.learner_server_entity = learner_server_entity
        self.controller_server_entity = controller_server_entity
        self.model_ops = model_ops
        if he_scheme_pb is not None and getattr(he_scheme_pb, "enabled", False):
            self.model_ops.he_scheme = he_scheme_from_config(he_scheme_pb)
        paths = dataset_paths or {}
        self.train_dataset = resolve_dataset(train_dataset, paths.get("train"))
        cls = type(self.train_dataset) if self.train_dataset is not None else ModelDataset
        self.validation_dataset = resolve_dataset(validation_dataset, paths.get("validation"), cls)
        self.test_dataset = resolve_dataset(test_dataset, paths.get("test"), cls)
        self._client = GRPCControllerClient(controller_server_entity, max_workers=1)
        self._client.retry_sleep_s = 1.0
        self.completion_retries = 60
        cred = learner_credentials_fp or os.path.join(
            "/tmp/metis_amd", f"learner_{learner_server_entity.port}_credentials")
        os.makedirs(cred, exist_ok=True)
        self._id_fp = os.path.join(cred, "learner_id.txt")
        self._token_fp = os.path.join(cred, "auth_token.txt")
        self.learner_id: str | None = None
        self.auth_token: str | None = None
        self._train_pool = futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="train")
        self._eval_pool = futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="eval")
        self._train_future: futures.Future | None = None
        self._cancel = threading.Event()
        self._lock = threading.Lock()
        self._joined = threading.Event()
        self.completed_tasks = 0

    def host_port_identifier(self) -> str:
        return f"{self.learner_server_entity.hostname}:{self.learner_server_entity.port}"

    # -- membership -----------------------------------------------------------------------
    def _spec(self, ds):
        return (ds.get_size(), ds.get_model_dataset_specifications()) if ds is not None else (0, {})

    def join_federation(self):
        tr, va, te = self._spec(self.train_dataset), self._spec(self.validation_dataset), \
            self._spec(self.test_dataset)
        is_cls = isinstance(self.train_dataset, ModelDatasetClassification)
        is_reg = isinstance(self.train_dataset, ModelDatasetRegression)
        self.learner_id, self.auth_token, status = self._client.join_federation(
            self.learner_server_entity, self._id_fp, self._token_fp, tr[0], tr[1], va[0], va[1], te[0], te[1],
            is_cls, is_reg, request_retries=3)
        self._joined.set()
        return status

    def leave_federation(self):
        if self.learner_id is None:
            return False
        try:
            return self._client.leave_federation(self.learner_id, self.auth_token)
        finally:
            self._client.shutdown()

    # -- tasks ---------------------------------------------------------------------------------
    def model_train(self, learning_task_pb, hyperparameters_pb, model_pb, cancel_event, verbose=False):
        self.model_ops.set_model_from_pb(model_pb)
        return self.model_ops.train_model(self.train_dataset, learning_task_pb, hyperparameters_pb,
                                          self.validation_dataset, self.test_dataset, verbose,
                                          cancel_event=cancel_event)

    def _on_trained(self, fut: futures.Future):
        if fut.cancelled():
            return
        exc = fut.exception()
        if isinstance(exc, TaskCancelled):
            MetisLogger.info("learner %s: training task preempted", self.host_port_identifier())
            return
        if exc is not None:
            MetisLogger.error("learner %s: training task failed: %r", self.host_port_identifier(), exc)
            return
        self.completed_tasks += 1
        # The controller dispatches a joining learner's first task from inside
        # JoinFederation, so a fast task can finish before the join response
        # (our id / token) has arrived: report only once it has.
        if not self._joined.wait(timeout=120.0):
            MetisLogger.error("learner %s: completed a task but never joined; result dropped",
                              self.host_port_identifier())
            return
        # A completed task must survive a controller restart (the
        # restored controller waits for this round's results): retry while the
        # controller is UNAVAILABLE, for up to ~1 minute.
        self._client.mark_task_completed(self.learner_id, self.auth_token, fut.result(),
                                         request_retries=self.completion_retries, block=False)

    def run_learning_task(self, learning_task_pb, hyperparameters_pb, model_pb,
                          cancel_running_tasks=True, block=False, verbose=False) -> bool:
        with self._lock:
            if self._train_future is not None and not self._train_future.done():
                if cancel_running_tasks:
                    self._cancel.set()
                self._train_future.cancel()
                try:
                    self._train_future.result()
                except BaseException:  # noqa: BLE001 - the preempted task's outcome is irrelevant
                    pass
            self._cancel = threading.Event()
            fut = self._train_pool.submit(self.model_train, learning_task_pb, hyperparameters_pb, model_pb,
                                          self._cancel, verbose)
            fut.add_done_callback(self._on_trained)
            self._train_future = fut
        if block:
            futures.wait([fut])
        return True

    def model_evaluate(self, model_pb, batch_size, evaluation_datasets, metrics_pb, verbose=False):
        metrics = list(metrics_pb.metric) if metrics_pb is not None else []
        E = learner_pb2.EvaluateModelRequest
        out = {}
        for which, ds in ((E.TRAINING, self.train_dataset), (E.VALIDATION, self.validation_dataset),
                          (E.TEST, self.test_dataset)):
            if which in evaluation_datasets and ds is not None:
                out[which] = self.model_ops.evaluate_model(ds, batch_size, metrics, verbose, model_pb=model_pb)
        ev = lambda w: M.construct_model_evaluation_pb(
            {k: str(v) for k, v in out.get(w, {}).items()})
        return M.construct_model_evaluations_pb(ev(E.TRAINING), ev(E.VALIDATION), ev(E.TEST))

    def run_evaluation_task(self, model_pb, batch_size, evaluation_dataset_pb, metrics_pb,
                            cancel_running_tasks=False, block=True, verbose=False):
        fut = self._eval_pool.submit(self.model_evaluate, model_pb, batch_size, list(evaluation_dataset_pb),
                                     metrics_pb, verbose)
        if block:
            return fut.result()
        return metis_pb2.ModelEvaluations()

    def run_inference_task(self):
        raise NotImplementedError("inference tasks are not part of the reference protocol either")

    def wait_idle(self, timeout=None) -> None:
        if self._train_future is not None:
            futures.wait([self._train_future], timeout=timeout)

    def shutdown(self, cancel_train_running_tasks=True, cancel_eval_running_tasks=False,
                 cancel_infer_running_tasks=True):
        if cancel_train_running_tasks:
            self._cancel.set()
        self._client.cancel_retries()
        self._train_pool.shutdown(wait=True, cancel_futures=cancel_train_running_tasks)
        self._eval_pool.shutdown(wait=not cancel_eval_running_tasks, cancel_futures=cancel_eval_running_tasks)
        self.model_ops.cleanup()
