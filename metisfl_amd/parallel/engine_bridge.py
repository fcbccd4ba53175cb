"""The native controller engine on the collective (RCCL) data plane.

On one node the models never travel through the controller: they are
averaged in place by an all-reduce.  Rank 0 still runs the SAME native
controller state machine as the gRPC path, so a collective federation has the
reference's bookkeeping and queries: learners registered with their dataset
specs, scaling factors from the configured scaler (controller.cc:809-830),
FederatedTaskRuntimeMetadata per round (the benchmark record, metis.proto
342-365), local task lineages, per-variable model quantifiers
(controller.cc:952-1004, computed on device by the count-zeros kernel) and
community-model lineage snapshots.
"""
from __future__ import annotations

import time

import numpy as np

from metisfl_amd.proto import controller_pb2, metis_pb2
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
from metisfl_amd.utils.proto_messages_factory import ModelProtoMessages as MM

_SCALING_NAMES = {"NUM_TRAINING_EXAMPLES": "NumTrainingExamples", "NUM_COMPLETED_BATCHES": "NumCompletedBatches",
                  "NUM_PARTICIPANTS": "NumParticipants"}
_RULES = {"fed_avg": "FedAvg", "fed_stride": "FedStride", "fed_rec": "FedRec"}


def controller_params_for(cfg, optimizer_pb=None):
    """ControllerParams equivalent of a FederationConfig."""
    rule = M.construct_aggregation_rule_pb(_RULES.get(cfg.aggregation, cfg.aggregation),
                                           _SCALING_NAMES.get(cfg.scaling_factor.upper(), cfg.scaling_factor),
                                           cfg.stride_length or None)
    opt = optimizer_pb or MM.construct_optimizer_config_pb(MM.construct_vanilla_sgd_optimizer_pb(0.01))
    return M.construct_controller_params_pb(
        M.construct_server_entity_pb("localhost", 50051),
        M.construct_global_model_specs(rule, 1.0),
        M.construct_communication_specs_pb(cfg.protocol.upper(), cfg.semi_sync_lambda, cfg.semi_sync_recompute),
        M.construct_model_store_config_pb("InMemory", "LineageLengthEviction", 1),
        M.construct_controller_modelhyperparams_pb(cfg.batch_size, cfg.local_epochs, opt, 0.0))


class CollectiveController:
    """Rank-0 wrapper around ``_engine.Controller`` for collective rounds."""

    def __init__(self, cfg, dataset_sizes: list[int], optimizer_pb=None):
        from metisfl_amd import _engine
        self.engine = _engine.Controller(controller_params_for(cfg, optimizer_pb).SerializeToString())
        self.ids, self.tokens = [], []
        for r, n in enumerate(dataset_sizes):
            se = M.construct_server_entity_pb("localhost", 50052 + r).SerializeToString()
            ds = M.construct_dataset_spec_pb(int(n), 0, 0).SerializeToString()
            lid, tok, _ = self.engine.add_learner(se, ds, False)
            self.ids.append(lid)
            self.tokens.append(tok)

    # -- aggregation weights ------------------------------------------------------
    def weights(self, num_train, completed_batches) -> list[float]:
        f = self.engine.scaling_factors(self.ids, [float(x) for x in num_train],
                                        [float(x) for x in completed_batches])
        return [float(f[i]) for i in self.ids]

    # -- bookkeeping ------------------------------------------------------------------
    @staticmethod
    def _task_meta(row, batch_size: int) -> bytes:
        n, batches, ms_b, ms_e, loss, acc, epochs, gi = row[:8]
        ev = M.construct_task_evaluation_pb([M.construct_epoch_evaluation_pb(
            max(1, int(np.ceil(epochs))), M.construct_model_evaluation_pb({"loss": loss, "accuracy": acc}))])
        return M.construct_task_execution_metadata_pb(int(gi), ev, float(epochs), int(batches), batch_size,
                                                      float(ms_e), float(ms_b)).SerializeToString()

    @staticmethod
    def _model_evaluations(ev: dict) -> bytes:
        """A learner's evaluation of the community model as the reference's
        ModelEvaluations (test set; metric values are strings)."""
        test = M.construct_model_evaluation_pb({"loss": ev["loss"], "accuracy": ev["accuracy"]})
        return M.construct_model_evaluations_pb(M.construct_model_evaluation_pb({}),
                                                M.construct_model_evaluation_pb({}), test).SerializeToString()

    def _evals(self, rec):
        if not rec.community_eval:
            return [], []
        ids = [self.ids[i] for i, e in enumerate(rec.community_eval) if e.get("num_examples") and i < len(self.ids)]
        evs = [self._model_evaluations(e) for e in rec.community_eval if e.get("num_examples")]
        return ids, evs

    def record_round(self, rec, batch_size: int, quantifiers=None) -> bool:
        ns = lambda t: int(t * 1e9)
        zeros, sizes, lengths = quantifiers or ([], [], [])
        metas = [self._task_meta(rec.learner_meta[i], batch_size) for i in range(len(self.ids))]
        self.engine.record_collective_round(rec.global_iteration, self.ids, ns(rec.started_at),
                                            ns(rec.completed_at), ns(rec.aggregation_started_at),
                                            ns(rec.aggregation_completed_at), metas, zeros, sizes, lengths)
        ids, evs = self._evals(rec)
        if ids:
            self.engine.record_community_evaluation(rec.global_iteration, ids, evs)
        return False

    def record_evaluations(self, global_iteration: int, community_eval: list) -> None:
        """A round's community-model evaluations recorded after the round (the
        deferred evaluation, FederationConfig.defer_community_eval)."""
        ids = [self.ids[i] for i, e in enumerate(community_eval) if e.get("num_examples") and i < len(self.ids)]
        evs = [self._model_evaluations(e) for e in community_eval if e.get("num_examples")]
        if ids:
            self._record_evaluations(int(global_iteration), ids, evs)

    def _record_evaluations(self, gi: int, ids: list, evs: list) -> None:
        self.engine.record_community_evaluation(gi, ids, evs)

    # -- asynchronous collective federation (async_federation.run_until) ---------------
    def _async_args(self, version: int, r: int, meta: dict, up):
        row = [meta.get("n_train", 0), meta["batches"], meta.get("ms_per_batch", 0.0), meta.get("ms_per_epoch", 0.0),
               meta["loss"], meta.get("accuracy", float("nan")), meta.get("epochs", 0.0), version]
        agg_done = up.received_at
        agg_start = agg_done - up.aggregation_ms / 1e3
        return row, int(meta.get("started_at", agg_start) * 1e9), int(agg_start * 1e9), int(agg_done * 1e9)

    def record_async_update(self, version: int, r: int, meta: dict, up, batch_size: int = 0) -> None:
        """One FedRec update: the finisher's task metadata and one runtime
        metadata record (global iteration = community version)."""
        row, st, ag0, ag1 = self._async_args(version, r, meta, up)
        self.engine.record_collective_round(version, [self.ids[r]], st, ag0, ag0, ag1,
                                            [self._task_meta(row, batch_size)], [], [], [])

    def record_async_evaluation(self, ev: dict) -> None:
        self.engine.record_community_evaluation(ev["version"], [self.ids[ev["learner"]]],
                                                [self._model_evaluations(ev)])

    def should_stop(self) -> bool:
        return False

    def community_evaluation_lineage(self, n: int = 0):
        return controller_pb2.GetCommunityModelEvaluationLineageResponse.FromString(
            self.engine.community_evaluation_lineage(n))

    def snapshot_community(self, names, arrays, trainable, global_iteration: int) -> None:
        """Community-model lineage entry (an explicit D2H copy: done on
        checkpoints / on request, not every round)."""
        from metisfl_amd.utils.tensor_codec import model_from_arrays
        fm = MM.construct_federated_model_pb(len(self.ids), model_from_arrays(names, arrays, trainable),
                                             global_iteration)
        self.engine.replace_community_model(fm.SerializeToString())

    # -- queries (same responses as the gRPC controller) -------------------------------
    def runtime_metadata(self, n: int = 0):
        return controller_pb2.GetRuntimeMetadataLineageResponse.FromString(self.engine.runtime_metadata_lineage(n))

    def local_task_lineage(self, n: int = 0):
        return controller_pb2.GetLocalTaskLineageResponse.FromString(self.engine.local_task_lineage(n, self.ids))

    def participating_learners(self):
        return controller_pb2.GetParticipatingLearnersResponse.FromString(self.engine.participating_learners())

    def community_model_lineage(self, n: int = 1):
        return controller_pb2.GetCommunityModelLineageResponse.FromString(self.engine.community_model_lineage(n))


class RemoteCollectiveController(CollectiveController):
    """Rank 0's bookkeeping sent to a RUNNING gRPC controller (the driver's,
    controller/collective_service.py) instead of an in-process engine: the
    same ``weights`` / ``record_round`` / ``snapshot_community`` interface,
    so ``CollectiveFederation`` is unchanged, and the driver's monitoring
    and statistics RPCs see the collective rounds."""

    def __init__(self, controller_entity, dataset_sizes: list[int], endpoints=None):  # no local engine
        """``endpoints``: (hostname, port) identities of the learners (the
        federation environment's; learner ids are derived from them)."""
        from metisfl_amd.controller import collective_service as cs
        from metisfl_amd.utils.grpc_services import make_channel
        self._cs = cs
        self._entity = controller_entity
        self._ch = make_channel(controller_entity)
        endpoints = endpoints or [("collective-rank", r + 1) for r in range(len(dataset_sizes))]
        r = cs.call(self._ch, "RegisterLearners",
                    {"learners": [{"hostname": h, "port": int(p), "num_training_examples": int(n)}
                                  for (h, p), n in zip(endpoints, dataset_sizes)]})
        self.ids, self.tokens = r["ids"], r["tokens"]

    def weights(self, num_train, completed_batches) -> list[float]:
        r = self._cs.call(self._ch, "ScalingFactors", {"ids": self.ids, "num_train": [float(x) for x in num_train],
                                                        "batches": [float(x) for x in completed_batches]})
        return r["factors"]

    def record_round(self, rec, batch_size: int, quantifiers=None) -> bool:
        """-> True when the driver asked the federation to stop."""
        import base64
        ns = lambda t: int(t * 1e9)
        zeros, sizes, lengths = quantifiers or ([], [], [])
        metas = [base64.b64encode(self._task_meta(rec.learner_meta[i], batch_size)).decode()
                 for i in range(len(self.ids))]
        ids, evs = self._evals(rec)
        r = self._cs.call(self._ch, "RecordRound", {
            "global_iteration": rec.global_iteration, "ids": self.ids, "started_ns": ns(rec.started_at),
            "completed_ns": ns(rec.completed_at), "agg_started_ns": ns(rec.aggregation_started_at),
            "agg_completed_ns": ns(rec.aggregation_completed_at), "metas": metas,
            "zeros": [int(z) for z in zeros], "sizes": [int(z) for z in sizes], "lengths": [int(z) for z in lengths],
            "eval_ids": ids, "evaluations": [base64.b64encode(e).decode() for e in evs]})
        self.regroup_requested = bool(r.get("regroup", False))
        return bool(r.get("stop", False))

    def should_stop(self) -> bool:
        if getattr(self, "_stop_seen", False):
            return True
        self._stop_seen = bool(self._cs.call(self._ch, "ShouldStop", {}).get("stop", False))
        return self._stop_seen

    def record_async_update(self, version: int, r: int, meta: dict, up, batch_size: int = 0) -> None:
        import base64
        row, st, ag0, ag1 = self._async_args(version, r, meta, up)
        resp = self._cs.call(self._ch, "RecordAsyncUpdate", {
            "global_iteration": version, "id": self.ids[r], "started_ns": st, "completed_ns": ag0,
            "agg_started_ns": ag0, "agg_completed_ns": ag1,
            "meta": base64.b64encode(self._task_meta(row, batch_size)).decode()})
        self._stop_seen = getattr(self, "_stop_seen", False) or bool(resp.get("stop", False))

    def _record_evaluations(self, gi: int, ids: list, evs: list) -> None:
        import base64
        self._cs.call(self._ch, "RecordEvaluation", {"global_iteration": gi, "ids": list(ids),
                                                     "evaluations": [base64.b64encode(e).decode() for e in evs]})

    def record_async_evaluation(self, ev: dict) -> None:
        import base64
        self._cs.call(self._ch, "RecordEvaluation", {
            "global_iteration": ev["version"], "ids": [self.ids[ev["learner"]]],
            "evaluations": [base64.b64encode(self._model_evaluations(ev)).decode()]})

    def snapshot_community(self, names, arrays, trainable, global_iteration: int) -> None:
        """Called from the lineage writer thread (one at a time): one client,
        and its channel, reused for every round's ReplaceCommunityModel."""
        from metisfl_amd.utils.tensor_codec import model_from_arrays
        if getattr(self, "_lineage_client", None) is None:
            from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
            self._lineage_client = GRPCControllerClient(self._entity, max_workers=1)
        self._lineage_client.replace_community_model(len(self.ids), model_from_arrays(names, arrays, trainable),
                                                     request_retries=2, global_iteration=int(global_iteration))

    def close(self) -> None:
        c, self._lineage_client = getattr(self, "_lineage_client", None), None
        if c is not None:
            c.shutdown()
        self._ch.close()
