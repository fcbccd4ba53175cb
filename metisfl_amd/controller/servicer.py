"""ControllerService over gRPC, backed by the native controller engine.

Reference: metisfl/controller/core/controller_servicer.cc:110-388 (RPC ->
Controller mapping and status codes) and controller.cc:349-793 (the async
RunTask / EvaluateModel fan-out with one channel per request).

Structure here:
  * every RPC is a thin call into ``metisfl_amd._engine.Controller`` (C++);
    the engine never blocks on the network -- it returns a *dispatch* of
    serialized RunTask / EvaluateModel requests;
  * ``LearnerDispatcher`` delivers those on a thread pool, with a fresh
    channel per request like the reference (its FIXME measured channel reuse
    5-10x slower for ~100 MB messages), and feeds evaluation results back
    into the engine;
  * MarkTaskCompleted / ReplaceCommunityModel are registered with RAW
    request bytes: the (large) model inside is handed to the engine without
    being parsed into Python objects;
  * all 12 RPCs are served, including GetCommunityModelLineage and
    GetLearnerLocalModelLineage, which the reference declares
    (controller.proto:15,19) but never implements.
"""
from __future__ import annotations

import os
import threading
from concurrent import futures

import grpc
from google.protobuf import json_format
from google.protobuf.timestamp_pb2 import Timestamp

from metisfl_amd import _engine as E
from metisfl_amd.proto import controller_pb2, learner_pb2, metis_pb2, service_common_pb2
from metisfl_amd.proto.grpc_api import LEARNER_SERVICE, controller_pb2_grpc, raw_unary, split_fields
from metisfl_amd.utils.grpc_services import GRPCServerMaxMsgLength, make_channel
from metisfl_amd.utils.metis_logger import MetisLogger

_CODES = {c.value[0]: c for c in grpc.StatusCode}


def _ack(status: bool, message: str = "") -> service_common_pb2.Ack:
    ts = Timestamp()
    ts.GetCurrentTime()
    return service_common_pb2.Ack(status=status, timestamp=ts, message=message)


class LearnerDispatcher:
    """Delivers the engine's dispatches to learners (RunTask is fire-and-
    forget on the learner side; EvaluateModel blocks until the metrics come
    back and is recorded into the engine)."""

    def __init__(self, engine, max_workers: int = 16, rpc_timeout: float | None = None):
        self.engine = engine
        self.pool = futures.ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="dispatch")
        self.entities: dict[str, metis_pb2.ServerEntity] = {}
        self.rpc_timeout = rpc_timeout
        self.lock = threading.Lock()
        self.failures = 0

    def register(self, learner_id: str, entity: metis_pb2.ServerEntity) -> None:
        with self.lock:
            self.entities[learner_id] = entity

    def forget(self, learner_id: str) -> None:
        with self.lock:
            self.entities.pop(learner_id, None)

    def _entity(self, learner_id):
        with self.lock:
            return self.entities.get(learner_id)

    def submit(self, dispatch) -> list:
        futs = []
        for lid, req in dispatch["run_tasks"]:
            futs.append(self.pool.submit(self._run_task, lid, req))
        for lid, req, ce_idx, md_idx in dispatch["eval_tasks"]:
            futs.append(self.pool.submit(self._evaluate, lid, req, ce_idx, md_idx))
        return futs

    def _run_task(self, lid: str, req: bytes) -> None:
        ent = self._entity(lid)
        if ent is None:
            return
        ch = make_channel(ent)
        try:
            resp = raw_unary(ch, LEARNER_SERVICE, "RunTask")(req, timeout=self.rpc_timeout)
            if not resp.ack.status:
                MetisLogger.warning("learner %s did not accept the task", lid)
        except grpc.RpcError as e:
            self.failures += 1
            MetisLogger.error("RunTask to %s failed: %s", lid, e.code())
        finally:
            ch.close()

    def _evaluate(self, lid: str, req: bytes, ce_idx: int, md_idx: int) -> None:
        ent = self._entity(lid)
        if ent is None:
            return
        ch = make_channel(ent)
        try:
            resp = raw_unary(ch, LEARNER_SERVICE, "EvaluateModel")(req, timeout=self.rpc_timeout)
            self.engine.record_evaluation(lid, ce_idx, md_idx, resp.evaluations.SerializeToString())
        except grpc.RpcError as e:
            self.failures += 1
            MetisLogger.error("EvaluateModel to %s failed: %s", lid, e.code())
        finally:
            ch.close()

    def shutdown(self) -> None:
        self.pool.shutdown(wait=True, cancel_futures=True)


class LearnerHealthMonitor:
    """Failure detector (the reference has no learner heartbeat
    and a dead learner stalls the synchronous barrier forever).  Every
    ``interval_s`` each registered learner gets a GetServicesHealthStatus
    probe; after ``threshold`` consecutive failures it is evicted from the
    engine, which re-checks the barrier and may release the pending round."""

    def __init__(self, servicer, interval_s: float = 5.0, threshold: int = 3, timeout_s: float = 2.0):
        self.srv = servicer
        self.interval = interval_s
        self.threshold = threshold
        self.timeout = timeout_s
        self.failures: dict[str, int] = {}
        self.evicted: list[str] = []
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="learner-health", daemon=True)

    def start(self):
        self._thread.start()

    def stop(self):
        self._stop.set()

    def probe(self, lid: str, entity) -> bool:
        ch = make_channel(entity)
        try:
            raw_unary(ch, LEARNER_SERVICE, "GetServicesHealthStatus")(b"", timeout=self.timeout)
            return True
        except grpc.RpcError:
            return False
        finally:
            ch.close()

    def check_once(self) -> None:
        with self.srv.dispatcher.lock:
            entities = dict(self.srv.dispatcher.entities)
        for lid, ent in entities.items():
            if self.probe(lid, ent):
                self.failures[lid] = 0
                continue
            self.failures[lid] = self.failures.get(lid, 0) + 1
            if self.failures[lid] >= self.threshold:
                MetisLogger.warning("learner %s failed %d health checks: evicting", lid, self.failures[lid])
                try:
                    dispatch = self.srv.engine.evict_learner(lid)
                except E.EngineStatusError:
                    dispatch = None  # already gone
                self.srv.dispatcher.forget(lid)
                self.failures.pop(lid, None)
                self.evicted.append(lid)
                if dispatch:
                    self.srv.dispatcher.submit(dispatch)

    def _loop(self):
        while not self._stop.wait(self.interval):
            try:
                self.check_once()
            except Exception as e:  # noqa: BLE001 - the monitor must survive anything
                MetisLogger.error("health monitor error: %r", e)


class ControllerServicer(controller_pb2_grpc.ControllerServiceServicer):

    def __init__(self, controller_params_pb, dispatch_workers: int = 16,
                 heartbeat_interval_s: float | None = 5.0, heartbeat_threshold: int = 3,
                 checkpoint_dir: str | None = None):
        self.params = controller_params_pb
        self.engine = E.Controller(controller_params_pb.SerializeToString())
        self.dispatcher = LearnerDispatcher(self.engine, dispatch_workers)
        # the engine state is snapshotted after every membership
        # change and every completed round; a controller started on an
        # existing checkpoint restores it and re-dispatches the round
        self.checkpoint_dir = checkpoint_dir
        # the learner ids of the on-node collective federation currently
        # registered through the collective service (collective_service.py)
        self.collective_members: list[str] = []
        self._ckpt_lock = threading.Lock()
        self._ckpt_gi = -1
        self.resumed = False
        if checkpoint_dir and os.path.exists(self._ckpt_path()):
            with open(self._ckpt_path(), "rb") as f:
                self.engine.restore(f.read())
            self.resumed = True
            self._ckpt_gi = self.engine.global_iteration()
            MetisLogger.info("Controller restored from %s (round %d, %d learners)", self._ckpt_path(),
                             self._ckpt_gi, self.engine.num_learners())
        self._shutdown = threading.Event()
        self._server: GRPCServerMaxMsgLength | None = None
        self._stop_thread: threading.Thread | None = None
        self.monitor = LearnerHealthMonitor(self, heartbeat_interval_s or 5.0, heartbeat_threshold) \
            if heartbeat_interval_s else None

    # -- lifecycle --------------------------------------------------------------
    def start(self) -> int:
        self._server = GRPCServerMaxMsgLength(max_workers=32, server_entity=self.params.server_entity)
        controller_pb2_grpc.add_ControllerServiceServicer_to_server(
            self, self._server.server, raw_requests=("MarkTaskCompleted", "ReplaceCommunityModel"))
        # rank 0 of an on-node collective (RCCL) federation reports its rounds here
        from metisfl_amd.controller.collective_service import add_collective_service
        add_collective_service(self, self._server.server)
        self._server.server.start()
        if self.monitor is not None:
            self.monitor.start()
        MetisLogger.info("Controller servicer listening on %s (port %d)",
                         self._server.grpc_endpoint.listening_endpoint, self._server.port)
        if self.resumed:  # re-broadcast the current round to the restored learners
            for d in controller_pb2.GetParticipatingLearnersResponse.FromString(
                    self.engine.participating_learners()).learner:
                self.dispatcher.register(d.id, d.server_entity)
            self.dispatcher.submit(self.engine.resume_dispatch())
        return self._server.port

    # -- checkpoint ------------------------------------------------------
    def _ckpt_path(self) -> str:
        return os.path.join(self.checkpoint_dir, "controller.ckpt")

    def checkpoint(self, force: bool = False) -> bool:
        """Write the engine snapshot (atomic rename) if the round advanced."""
        if not self.checkpoint_dir:
            return False
        with self._ckpt_lock:
            gi = self.engine.global_iteration()
            if not force and gi == self._ckpt_gi:
                return False
            os.makedirs(self.checkpoint_dir, exist_ok=True)
            tmp = self._ckpt_path() + ".tmp"
            with open(tmp, "wb") as f:
                f.write(self.engine.checkpoint())
            os.replace(tmp, self._ckpt_path())
            self._ckpt_gi = gi
            return True

    @property
    def port(self) -> int:
        return self._server.port if self._server else 0

    def shutdown_request_received(self) -> bool:
        return self._shutdown.is_set()

    def stop(self, grace: float = 0.5) -> None:
        self._shutdown.set()
        if self.monitor is not None:
            self.monitor.stop()
        if self._server is not None:
            self._server.server.stop(grace).wait()
        self.dispatcher.shutdown()

    def wait(self) -> None:
        if self._stop_thread is not None:
            self._stop_thread.join()
        elif self._server is not None:
            self._server.server.wait_for_termination()

    # -- helpers -------------------------------------------------------------------
    @staticmethod
    def _abort(context, code: int, msg: str):
        context.abort(_CODES.get(code, grpc.StatusCode.INTERNAL), msg)

    # -- queries -----------------------------------------------------------------------
    def GetCommunityModelEvaluationLineage(self, request, context):
        return controller_pb2.GetCommunityModelEvaluationLineageResponse.FromString(
            self.engine.community_evaluation_lineage(request.num_backtracks))

    def GetCommunityModelLineage(self, request, context):
        return controller_pb2.GetCommunityModelLineageResponse.FromString(
            self.engine.community_model_lineage(request.num_backtracks))

    def GetLearnerLocalModelLineage(self, request, context):
        ses = [se.SerializeToString() for se in request.server_entity]
        return controller_pb2.GetLearnerLocalModelLineageResponse.FromString(
            self.engine.learner_local_model_lineage(request.num_backtracks, ses))

    def GetLocalTaskLineage(self, request, context):
        return controller_pb2.GetLocalTaskLineageResponse.FromString(
            self.engine.local_task_lineage(request.num_backtracks, list(request.learner_ids)))

    def GetRuntimeMetadataLineage(self, request, context):
        resp = controller_pb2.GetRuntimeMetadataLineageResponse.FromString(
            self.engine.runtime_metadata_lineage(request.num_backtracks))
        resp.json_metadata = json_format.MessageToJson(resp)
        return resp

    def GetParticipatingLearners(self, request, context):
        return controller_pb2.GetParticipatingLearnersResponse.FromString(
            self.engine.participating_learners())

    def GetServicesHealthStatus(self, request, context):
        resp = service_common_pb2.GetServicesHealthStatusResponse()
        resp.services_status["controller"] = self.engine is not None
        return resp

    # -- membership --------------------------------------------------------------------
    def JoinFederation(self, request, context):
        if not request.HasField("server_entity") and not request.HasField("local_dataset_spec"):
            self._abort(context, 3, "Server entity and local dataset cannot be empty.")
        try:
            lid, tok, dispatch = self.engine.add_learner(request.server_entity.SerializeToString(),
                                                         request.local_dataset_spec.SerializeToString())
        except E.EngineStatusError as e:
            code, msg = e.args
            self._abort(context, 6 if code == 6 else 3, msg)
        self.dispatcher.register(lid, request.server_entity)
        MetisLogger.info("Learner %s joined the federation.", lid)
        self.checkpoint(force=True)
        self.dispatcher.submit(dispatch)
        return controller_pb2.JoinFederationResponse(ack=_ack(True), learner_id=lid, auth_token=tok)

    def LeaveFederation(self, request, context):
        if not request.learner_id or not request.auth_token:
            self._abort(context, 3, "Learner id and authentication token cannot be empty.")
        dispatch = None
        try:
            dispatch = self.engine.remove_learner(request.learner_id, request.auth_token)
        except E.EngineStatusError as e:
            self._abort(context, grpc.StatusCode.CANCELLED.value[0], e.args[1])
        self.dispatcher.forget(request.learner_id)
        MetisLogger.info("Learner %s left the federation.", request.learner_id)
        self.checkpoint(force=True)
        if dispatch:  # the sync barrier was waiting only for the leaver
            self.dispatcher.submit(dispatch)
        return controller_pb2.LeaveFederationResponse(ack=_ack(True))

    # -- task flow ---------------------------------------------------------------------------
    def MarkTaskCompleted(self, request: bytes, context):
        f = split_fields(request)
        lid = bytes(f.get(1, [b""])[0]).decode()
        tok = bytes(f.get(2, [b""])[0]).decode()
        task = bytes(f.get(3, [b""])[0])
        try:
            dispatch = self.engine.learner_completed_task(lid, tok, task)
        except E.EngineStatusError as e:
            code, msg = e.args
            self._abort(context, code if code in (3, 5, 7, 16) else 13, msg)
        self.checkpoint()
        self.dispatcher.submit(dispatch)
        return controller_pb2.MarkTaskCompletedResponse(ack=_ack(True))

    def ReplaceCommunityModel(self, request: bytes, context):
        f = split_fields(request)
        try:
            self.engine.replace_community_model(bytes(f.get(1, [b""])[0]))
        except (E.EngineStatusError, RuntimeError, ValueError) as e:
            self._abort(context, grpc.StatusCode.UNAUTHENTICATED.value[0], str(e))
        MetisLogger.info("Replaced the community model.")
        self.checkpoint(force=True)
        return controller_pb2.ReplaceCommunityModelResponse(ack=_ack(True))

    def ShutDown(self, request, context):
        self._shutdown.set()
        # stop asynchronously so this response still goes out (reference:
        # controller_servicer.cc:364-379 schedules Stop on a 1-thread pool)
        self._stop_thread = threading.Thread(target=self.stop, daemon=True)
        self._stop_thread.start()
        return service_common_pb2.ShutDownResponse(ack=_ack(True))
