"""LearnerService over gRPC (reference: metisfl/learner/learner_servicer.py:14-139).

RunTask is non-blocking (the task preempts any running one); EvaluateModel
blocks until the metrics are ready; ShutDown stops serving, cancels
training, leaves the federation and releases ``wait_servicer``."""
from __future__ import annotations

import threading

import grpc
from google.protobuf.timestamp_pb2 import Timestamp

from metisfl_amd.learner.learner import Learner
from metisfl_amd.proto import learner_pb2, service_common_pb2
from metisfl_amd.proto.grpc_api import learner_pb2_grpc
from metisfl_amd.utils.grpc_services import GRPCServerMaxMsgLength
from metisfl_amd.utils.metis_logger import MetisLogger


def _ack(status=True):
    ts = Timestamp()
    ts.GetCurrentTime()
    return service_common_pb2.Ack(status=status, timestamp=ts)


class LearnerServicer(learner_pb2_grpc.LearnerServiceServicer):

    def __init__(self, learner: Learner, servicer_workers: int = 10):
        self.learner = learner
        self.servicer_workers = servicer_workers
        self.community_models_received = 0
        self.model_evaluation_requests = 0
        self._not_serving = threading.Event()
        self._shutdown = threading.Event()
        self._server: GRPCServerMaxMsgLength | None = None

    def init_servicer(self, join: bool = True) -> int:
        self._server = GRPCServerMaxMsgLength(max_workers=self.servicer_workers,
                                              server_entity=self.learner.learner_server_entity)
        learner_pb2_grpc.add_LearnerServiceServicer_to_server(self, self._server.server)
        self._server.server.start()
        if self.learner.learner_server_entity.port == 0:  # OS-assigned port (tests)
            self.learner.learner_server_entity.port = self._server.port
        MetisLogger.info("Learner servicer listening on %s", self._server.grpc_endpoint.listening_endpoint)
        if join:
            self.learner.join_federation()
        return self._server.port

    def wait_servicer(self) -> None:
        self._shutdown.wait()
        self._server.server.stop(None)

    def stop(self) -> None:
        self._not_serving.set()
        self._shutdown.set()
        if self._server is not None:
            self._server.server.stop(0.5)

    # -- RPCs ----------------------------------------------------------------------------
    def EvaluateModel(self, request, context):
        if self._not_serving.is_set():
            context.abort(grpc.StatusCode.UNAVAILABLE, "learner is shutting down")
        self.model_evaluation_requests += 1
        evals = self.learner.run_evaluation_task(request.model, request.batch_size, request.evaluation_dataset,
                                                 request.metrics, cancel_running_tasks=False, block=True)
        return learner_pb2.EvaluateModelResponse(evaluations=evals)

    def GetServicesHealthStatus(self, request, context):
        if self._not_serving.is_set():
            context.abort(grpc.StatusCode.UNAVAILABLE, "learner is shutting down")
        resp = service_common_pb2.GetServicesHealthStatusResponse()
        resp.services_status["server"] = self._server is not None
        return resp

    def RunTask(self, request, context):
        if self._not_serving.is_set():
            context.abort(grpc.StatusCode.UNAVAILABLE, "learner is shutting down")
        self.community_models_received += 1
        ok = self.learner.run_learning_task(request.task, request.hyperparameters, request.federated_model.model,
                                            cancel_running_tasks=True, block=False)
        return learner_pb2.RunTaskResponse(ack=_ack(ok))

    def ShutDown(self, request, context):
        MetisLogger.info("Learner %s received a shutdown request.", self.learner.host_port_identifier())
        self._not_serving.set()
        self.learner.shutdown(cancel_train_running_tasks=True, cancel_eval_running_tasks=False,
                              cancel_infer_running_tasks=True)
        self.learner.leave_federation()
        self._shutdown.set()
        return service_common_pb2.ShutDownResponse(ack=_ack(True))
