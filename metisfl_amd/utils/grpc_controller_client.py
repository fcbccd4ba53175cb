"""Learner / driver -> controller client (reference:
metisfl/utils/grpc_controller_client.py:11-297).  Same method names and
blocking / non-blocking / retry semantics; adds the two lineage getters the
reference's controller never served (community models, learner local
models)."""
from __future__ import annotations

import grpc

from metisfl_amd.proto.grpc_api import controller_pb2_grpc
from metisfl_amd.utils import proto_messages_factory as pf
from metisfl_amd.utils.grpc_services import GRPCServerClient
from metisfl_amd.utils.metis_logger import MetisLogger
from metisfl_amd.utils.ssl_configurator import SSLConfigurator

C = pf.ControllerServiceProtoMessages


class GRPCControllerClient(GRPCServerClient):

    def __init__(self, controller_server_entity, max_workers: int = 1):
        super().__init__(controller_server_entity, max_workers)
        self._stub = controller_pb2_grpc.ControllerServiceStub(self._channel)

    def _call(self, fn, request_retries, request_timeout, block):
        return self._schedule(fn, request_retries, request_timeout, block)

    def check_health_status(self, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            resp = self._stub.GetServicesHealthStatus(
                pf.ServiceCommonProtoMessages.construct_get_services_health_status_request_pb(), timeout=t)
            MetisLogger.info("Controller health %s: %s", self.grpc_endpoint.listening_endpoint,
                             dict(resp.services_status))
            return resp
        return self._call(_req, request_retries, request_timeout, block)

    def join_federation(self, learner_server_entity, learner_id_fp, auth_token_fp, train_dataset_size,
                        train_dataset_specs, validation_dataset_size, validation_dataset_specs,
                        test_dataset_size, test_dataset_specs, is_classification, is_regression,
                        request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            # never ship the learner's private key: public certificate only
            public = SSLConfigurator.gen_public_ssl_config_pb_as_stream(learner_server_entity.ssl_config)
            entity = pf.MetisProtoMessages.construct_server_entity_pb(
                learner_server_entity.hostname, learner_server_entity.port, public)
            spec = pf.MetisProtoMessages.construct_dataset_spec_pb(
                train_dataset_size, validation_dataset_size, test_dataset_size, train_dataset_specs,
                validation_dataset_specs, test_dataset_specs, is_classification, is_regression)
            try:
                resp = self._stub.JoinFederation(C.construct_join_federation_request_pb(entity, spec), timeout=t)
                lid, tok, status = resp.learner_id, resp.auth_token, resp.ack.status
                with open(learner_id_fp, "w") as f:
                    f.write(lid.strip())
                with open(auth_token_fp, "w") as f:
                    f.write(tok.strip())
                MetisLogger.info("Joined federation with id %s", lid)
            except grpc.RpcError as err:
                if err.code() != grpc.StatusCode.ALREADY_EXISTS:
                    raise RuntimeError(f"Unhandled grpc error: {err}") from err
                # rejoin: credentials persisted by the earlier join
                with open(learner_id_fp) as f:
                    lid = f.read().strip()
                with open(auth_token_fp) as f:
                    tok = f.read().strip()
                status = True
                MetisLogger.info("Learner re-joined federation with id %s", lid)
            return lid, tok, status
        return self._call(_req, request_retries, request_timeout, block)

    def leave_federation(self, learner_id, auth_token, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.LeaveFederation(C.construct_leave_federation_request_pb(learner_id, auth_token),
                                              timeout=t)
        return self._call(_req, request_retries, request_timeout, block)

    def mark_task_completed(self, learner_id, auth_token, completed_task_pb, request_retries=1,
                            request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.MarkTaskCompleted(
                C.construct_mark_task_completed_request_pb(learner_id, auth_token, completed_task_pb), timeout=t)
        # not idempotent: retried on transport failures only (the controller
        # ignores a duplicate completion of a task it already recorded)
        return self._schedule(_req, request_retries, request_timeout, block, retry_codes=self.TRANSIENT_CODES)

    def get_community_model_evaluation_lineage(self, num_backtracks, request_retries=1, request_timeout=None,
                                               block=True):
        def _req(t=None):
            return self._stub.GetCommunityModelEvaluationLineage(
                C.construct_get_community_model_evaluation_lineage_request_pb(num_backtracks), timeout=t)
        return self._call(_req, request_retries, request_timeout, block)

    def get_community_model_lineage(self, num_backtracks, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.GetCommunityModelLineage(
                C.construct_get_community_model_lineage_request_pb(num_backtracks), timeout=t)
        return self._call(_req, request_retries, request_timeout, block)

    def get_learner_local_model_lineage(self, num_backtracks, server_entities, request_retries=1,
                                        request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.GetLearnerLocalModelLineage(
                C.construct_get_learner_local_model_lineage_request_pb(num_backtracks, server_entities),
                timeout=t)
        return self._call(_req, request_retries, request_timeout, block)

    def get_local_task_lineage(self, num_backtracks, learner_ids, request_retries=1, request_timeout=None,
                               block=True):
        def _req(t=None):
            return self._stub.GetLocalTaskLineage(
                C.construct_get_local_task_lineage_request_pb(num_backtracks, learner_ids), timeout=t)
        return self._call(_req, request_retries, request_timeout, block)

    def get_participating_learners(self, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.GetParticipatingLearners(
                C.construct_get_participating_learners_request_pb(), timeout=t)
        return self._call(_req, request_retries, request_timeout, block)

    def get_runtime_metadata(self, num_backtracks, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            return self._stub.GetRuntimeMetadataLineage(
                C.construct_get_runtime_metadata_lineage_request_pb(num_backtracks), timeout=t)
        return self._call(_req, request_retries, request_timeout, block)

    def replace_community_model(self, num_contributors, model_pb, request_retries=1, request_timeout=None,
                                block=True, global_iteration: int = 0):
        def _req(t=None):
            fm = pf.ModelProtoMessages.construct_federated_model_pb(num_contributors, model_pb, global_iteration)
            resp = self._stub.ReplaceCommunityModel(C.construct_replace_community_model_request_pb(fm),
                                                    timeout=t)
            return resp.ack.status
        return self._call(_req, request_retries, request_timeout, block)

    def shutdown_controller(self, request_retries=1, request_timeout=None, block=True):
        def _req(t=None):
            resp = self._stub.ShutDown(pf.ServiceCommonProtoMessages.construct_shutdown_request_pb(), timeout=t)
            return resp.ack.status
        return self._call(_req, request_retries, request_timeout, block)
