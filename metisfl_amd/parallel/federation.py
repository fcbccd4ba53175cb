"""Collective (single-node, one learner per GPU) federation engine.

Each process hosts ONE persistent learner whose model, optimizer state and
data shard stay resident in HBM across rounds.  A synchronous FedAvg round is

  1. local training: ``num_local_updates`` graph-replayed steps,
  2. all-gather of a few scalars per learner (dataset size, completed
     batches, per-batch / per-epoch time, train metrics) -- the payload of the
     reference's MarkTaskCompleted metadata (learner.py:197-206),
  3. scaling factors from the controller's scaler (C++ engine) -- identical
     on every rank, so no broadcast is needed,
  4. in-place pre-scale ``theta_i *= w_i`` (K1) and ONE RCCL all-reduce of the
     flat model buffer: every learner now holds the community model, which is
     the reference's gather -> FedAvg -> RunTask broadcast
     (controller.cc:428-518, 795-950) collapsed into one collective.

Semi-synchronous rounds use the same barrier with per-learner step budgets
recomputed from the measured per-batch times (controller.cc:520-569).
Asynchronous rounds are served by parallel/async_fed.py.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from metisfl_amd.ops import optim as opt_ops
from metisfl_amd.parallel.comm import Comm
from metisfl_amd.parallel import scaling

META_FIELDS = ("num_training_examples", "completed_batches", "ms_per_batch", "ms_per_epoch",
               "train_loss", "train_accuracy", "completed_epochs", "global_iteration")


@dataclass
class FederationConfig:
    protocol: str = "synchronous"          # synchronous | semi_synchronous | asynchronous
    aggregation: str = "fed_avg"           # fed_avg | fed_stride | fed_rec
    scaling_factor: str = "NUM_TRAINING_EXAMPLES"
    stride_length: int = 0
    batch_size: int = 32
    local_epochs: int = 4
    semi_sync_lambda: float = 2.0
    semi_sync_recompute: bool = False
    evaluate_test: bool = True             # learner test-set eval at task end
    eval_max_steps: int | None = None
    extra: dict = field(default_factory=dict)


@dataclass
class RoundRecord:
    global_iteration: int
    started_at: float
    completed_at: float
    aggregation_started_at: float
    aggregation_completed_at: float
    round_ms: float
    train_ms: float
    aggregation_ms: float
    learner_meta: np.ndarray
    weights: list
    num_local_updates: list
    test_metrics: dict | None = None


class CollectiveFederation:
    """Drives rounds for the learner hosted by this rank."""

    def __init__(self, comm: Comm, net, train_ds, cfg: FederationConfig, test_ds=None,
                 learner_ids: list[str] | None = None, engine=None):
        self.comm = comm
        self.net = net
        self.train_ds = train_ds
        self.test_ds = test_ds
        self.cfg = cfg
        self.engine = engine
        self.world = comm.world
        self.rank = comm.rank
        self.learner_ids = learner_ids or [f"learner_{r}" for r in range(self.world)]
        spe = train_ds.steps_per_epoch
        # reference: num_local_updates = epochs * ceil(N_train / batch) (controller.cc:148-153)
        n_updates = cfg.local_epochs * max(1, math.ceil(train_ds.n / cfg.batch_size))
        self.num_local_updates = [n_updates] * self.world
        self.steps_done = 0
        self.global_iteration = 0
        self.history: list[RoundRecord] = []
        self._spe = spe
        dev = comm.device
        self._ev0 = torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else None
        self._ev1 = torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else None
        self.broadcast_initial_model()

    # ------------------------------------------------------------------------
    def broadcast_initial_model(self) -> None:
        """ReplaceCommunityModel equivalent: rank 0's model becomes everyone's."""
        st = self.net.state
        self.comm.broadcast_(st.model32, src=0)
        st.refresh_bf16()
        st.set_anchor()

    def _sync(self):
        if self.comm.device.type == "cuda":
            torch.cuda.synchronize(self.comm.device)

    def local_train(self, nsteps: int) -> dict:
        net = self.net
        net.reset_train_stats()
        t0 = time.perf_counter()
        if self._ev0 is not None:
            self._ev0.record()
        net.train_steps(self.train_ds, nsteps, step_offset=self.steps_done)
        if self._ev1 is not None:
            self._ev1.record()
            self._ev1.synchronize()
            ms = self._ev0.elapsed_time(self._ev1)
        else:
            ms = (time.perf_counter() - t0) * 1e3
        self.steps_done += nsteps
        tr = net.train_stats()
        out = {"ms": ms, "ms_per_batch": ms / max(1, nsteps),
               "ms_per_epoch": ms / max(1, nsteps) * self._spe,
               "completed_batches": nsteps, "completed_epochs": nsteps / self._spe,
               "train_loss": tr["loss"], "train_accuracy": tr["accuracy"]}
        if self.cfg.evaluate_test and self.test_ds is not None:
            out["test"] = net.evaluate(self.test_ds, self.cfg.eval_max_steps)
        return out

    def aggregate(self, meta: np.ndarray) -> tuple[list[float], float]:
        """Scale + all-reduce; returns (weights, ms)."""
        t0 = time.perf_counter()
        ids = self.learner_ids
        if self.engine is not None:
            weights = self.engine.scaling_factors(self.cfg.scaling_factor, ids,
                                                  meta[:, 0].tolist(), meta[:, 1].tolist(),
                                                  self.world)
        else:
            weights = scaling.compute(self.cfg.scaling_factor, meta[:, 0], meta[:, 1], self.world)
        st = self.net.state
        if self.world > 1:
            opt_ops.scale_(st.model32, weights[self.rank])
            self.comm.all_reduce_(st.model32)
        st.refresh_bf16()
        st.set_anchor()
        self._sync()
        return weights, (time.perf_counter() - t0) * 1e3

    def update_templates(self, meta: np.ndarray) -> None:
        """Semi-synchronous step budgets (controller.cc:520-569): after round 1
        (or every round with recompute) each learner gets
        ceil(lambda * max_i(ms_per_epoch_i) / ms_per_batch_self) updates."""
        if self.cfg.protocol != "semi_synchronous":
            return
        if not (self.global_iteration == 2 or self.cfg.semi_sync_recompute):
            return
        t_max = self.cfg.semi_sync_lambda * float(meta[:, 3].max())
        self.num_local_updates = [max(1, int(math.ceil(t_max / max(1e-6, float(mpb)))))
                                  for mpb in meta[:, 2]]

    def run_round(self) -> RoundRecord:
        self.global_iteration += 1
        started = time.time()
        n = self.num_local_updates[self.rank]
        res = self.local_train(n)
        row = torch.tensor([self.train_ds.n, res["completed_batches"], res["ms_per_batch"],
                            res["ms_per_epoch"], res["train_loss"], res["train_accuracy"],
                            res["completed_epochs"], self.global_iteration],
                           dtype=torch.float64, device=self.comm.device)
        meta = self.comm.all_gather_rows(row).cpu().numpy()
        completed = time.time()
        weights, agg_ms = self.aggregate(meta)
        agg_done = time.time()
        rec = RoundRecord(self.global_iteration, started, completed, completed, agg_done,
                          (agg_done - started) * 1e3, res["ms"], agg_ms, meta, weights,
                          list(self.num_local_updates), res.get("test"))
        if self.engine is not None and self.rank == 0:
            self.engine.record_collective_round(rec, self.learner_ids)
        self.update_templates(meta)
        self.history.append(rec)
        return rec
