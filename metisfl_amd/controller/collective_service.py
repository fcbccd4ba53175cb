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
METHODS = ("RegisterLearners", "ScalingFactors", "RecordRound", "RecordAsyncUpdate", "RecordEvaluation",
           "RequestStop", "ShouldStop", "RequestRegroup")


def add_collective_service(servicer, server: grpc.Server) -> None:
    eng = servicer.engine
    # stop: leave after the current round; regroup: checkpoint after the
    # current round and exit for a relaunch on a new membership (learners
    # joining a running collective federation, driver_session.py)
    state = {"stop": False, "regroup": False}

    def register(req: bytes, ctx) -> bytes:
        """(Re-)register the collective ranks.  A relaunch (after a lost rank,
        or to admit joining learners: driver_session.py) registers the new
        membership: the collective learners of the previous one that are not
        in it leave the federation (the reference's LeaveFederation,
        controller.cc:171-199), the others re-join with fresh specs and
        tokens.  The previous membership is the engine's own (collective
        learners have no gRPC server, port < 1024 or the "collective-rank"
        host), so it survives a controller restart from its checkpoint; the
        removals are membership changes, not failure-detector evictions."""
        d = json.loads(req)
        want = {f"{l.get('hostname', 'localhost')}:{int(l.get('port', 0))}" for l in d["learners"]}
        prev = set(servicer.collective_members) | want
        for lid in eng.learner_ids():
            if lid in prev:  # leaving, or re-joining with fresh specs / token
                eng.evict_learner(lid, False)
                if lid not in want:
                    MetisLogger.info("Collective learner %s left the federation.", lid)
        registered = servicer.collective_members
        registered.clear()
        state["regroup"] = False  # a requested membership change is now in effect
        ids, toks = [], []
        for l in d["learners"]:
            se = M.construct_server_entity_pb(l.get("hostname", "localhost"), int(l.get("port", 0)))
            ds = M.construct_dataset_spec_pb(int(l["num_training_examples"]), 0, int(l.get("num_test_examples", 0)))
            lid, tok, _ = eng.add_learner(se.SerializeToString(), ds.SerializeToString(), False)
            ids.append(lid)
            toks.append(tok)
            registered.append(lid)
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
        if d.get("eval_ids"):  # the learners' evaluations of the new community model
            eng.record_community_evaluation(int(d["global_iteration"]), d["eval_ids"],
                                            [base64.b64decode(e) for e in d["evaluations"]])
        servicer.checkpoint()
        return json.dumps({"stop": state["stop"], "regroup": state["regroup"]}).encode()

    def record_async(req: bytes, ctx) -> bytes:
        """One FedRec update of an asynchronous collective federation: the
        finisher's task metadata (local task lineage) and the update's
        FederatedTaskRuntimeMetadata (one community version)."""
        d = json.loads(req)
        eng.record_collective_round(int(d["global_iteration"]), [d["id"]], int(d["started_ns"]),
                                    int(d["completed_ns"]), int(d["agg_started_ns"]), int(d["agg_completed_ns"]),
                                    [base64.b64decode(d["meta"])], [], [], [])
        servicer.checkpoint()
        return json.dumps({"stop": state["stop"]}).encode()

    def record_eval(req: bytes, ctx) -> bytes:
        d = json.loads(req)
        eng.record_community_evaluation(int(d["global_iteration"]), d["ids"],
                                        [base64.b64decode(e) for e in d["evaluations"]])
        return json.dumps({"stop": state["stop"]}).encode()

    def request_stop(req: bytes, ctx) -> bytes:
        state["stop"] = True
        MetisLogger.info("Collective federation: stop requested.")
        return b"{}"

    def should_stop(req: bytes, ctx) -> bytes:
        return json.dumps({"stop": state["stop"]}).encode()

    def request_regroup(req: bytes, ctx) -> bytes:
        state["regroup"] = True
        MetisLogger.info("Collective federation: membership change requested (regroup after this round).")
        return b"{}"

    fns = {"RegisterLearners": register, "ScalingFactors": scaling, "RecordRound": record,
           "RecordAsyncUpdate": record_async, "RecordEvaluation": record_eval, "RequestStop": request_stop,
           "ShouldStop": should_stop, "RequestRegroup": request_regroup}
    handlers = {name: grpc.unary_unary_rpc_method_handler(fn) for name, fn in fns.items()}
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))


def call(channel: grpc.Channel, method: str, payload: dict, timeout: float = 60.0) -> dict:
    fn = channel.unary_unary(f"/{SERVICE}/{method}")
    return json.loads(fn(json.dumps(payload).encode(), timeout=timeout) or b"{}")
