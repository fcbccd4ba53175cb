"""Driver -> learner client (reference: metisfl/utils/grpc_learner_client.py:8-58):
health check and shutdown, plus direct RunTask / EvaluateModel calls used by
tests and tools."""
from __future__ import annotations

from metisfl_amd.proto.grpc_api import learner_pb2_grpc
from metisfl_amd.utils import proto_messages_factory as pf
from metisfl_amd.utils.grpc_services import GRPCServerClient


class GRPCLearnerClient(GRPCServerClient):

    def __init__(self, learner_server_entity, max_workers: int = 1):
        super().__init__(learner_server_entity, max_workers)
        self._stub = learner_pb2_grpc.LearnerServiceStub(self._channel)

    def check_health_status(self, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.GetServicesHealthStatus(
                pf.ServiceCommonProtoMessages.construct_get_services_health_status_request_pb(), timeout=t)
        return self._schedule(_req, request_retries, request_timeout, block)

    def run_task(self, run_task_request_pb, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.RunTask(run_task_request_pb, timeout=t)
        return self._schedule(_req, request_retries, request_timeout, block)

    def evaluate_model(self, evaluate_model_request_pb, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.EvaluateModel(evaluate_model_request_pb, timeout=t)
        return self._schedule(_req, request_retries, request_timeout, block)

    def shutdown_learner(self, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            resp = self._stub.ShutDown(pf.ServiceCommonProtoMessages.construct_shutdown_request_pb(), timeout=t)
            return resp.ack.status
        return self._schedule(_req, request_retries, request_timeout, block)
