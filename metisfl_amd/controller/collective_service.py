"""Collective-round bookkeeping service on the controller's gRPC server.

On one MI355X node the learners average their models with an RCCL
all-reduce (parallel/federation.py); no model crosses the controller.  The
controller still owns the federation's record: the learners, the scaling
factors, one ``FederatedTaskRuntimeMetadata`` per round, the local task
lineages and the community-model lineage -- so the driver's
``monitor_federation`` / ``get_federation_statistics`` and every
``metisfl.ControllerService`` query work unchanged for a collective
federation.

Rank 0 of the collective job reports through this small service.  It is a
SEPARATE gRPC service (``metisfl_amd.CollectiveService``, JSON payloads) on
the same server, so the reference's ``metisfl.ControllerService`` schema
(controller.proto) stays byte-identical.  The learners it registers have no
gRPC server of their own: they are not health-probed and never receive
RunTask dispatches.
"""
from __future__ import annotations

import base64
import json

import grpc

from metisfl_amd.utils.metis_logger import MetisLogger
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M

SERVICE = "metisfl_amd.CollectiveService"
METHODS = ("RegisterLearners", "ScalingFactors", "RecordRound")


def add_collective_service(servicer, server: grpc.Server) -> None:
    eng = servicer.engine

    def register(req: bytes, ctx) -> bytes:
        d = json.loads(req)
        ids, toks = [], []
        for l in d["learners"]:
            se = M.construct_server_entity_pb(l.get("hostname", "localhost"), int(l.get("port", 0)))
            ds = M.construct_dataset_spec_pb(int(l["num_training_examples"]), 0, int(l.get("num_test_examples", 0)))
            lid, tok, _ = eng.add_learner(se.SerializeToString(), ds.SerializeToString())
            ids.append(lid)
            toks.append(tok)
        MetisLogger.info("Collective federation registered %d learners.", len(ids))
        servicer.checkpoint(force=True)
        return json.dumps({"ids": ids, "tokens": toks}).encode()

    def scaling(req: bytes, ctx) -> bytes:
        d = json.loads(req)
        f = eng.scaling_factors(d["ids"], [float(x) for x in d["num_train"]], [float(x) for x in d["batches"]])
        return json.dumps({"factors": [float(f[i]) for i in d["ids"]]}).encode()

    def record(req: bytes, ctx) -> bytes:
        d = json.loads(req)
        metas = [base64.b64decode(m) for m in d["metas"]]
        eng.record_collective_round(int(d["global_iteration"]), d["ids"], int(d["started_ns"]),
                                    int(d["completed_ns"]), int(d["agg_started_ns"]), int(d["agg_completed_ns"]),
                                    metas, d.get("zeros", []), d.get("sizes", []), d.get("lengths", []))
        servicer.checkpoint()
        return b"{}"

    fns = {"RegisterLearners": register, "ScalingFactors": scaling, "RecordRound": record}
    handlers = {name: grpc.unary_unary_rpc_method_handler(fn) for name, fn in fns.items()}
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))


def call(channel: grpc.Channel, method: str, payload: dict, timeout: float = 60.0) -> dict:
    fn = channel.unary_unary(f"/{SERVICE}/{method}")
    return json.loads(fn(json.dumps(payload).encode(), timeout=timeout) or b"{}")
