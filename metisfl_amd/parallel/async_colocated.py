"""Asynchronous federation of learners co-located on one GPU (FedRec).

The reference's asynchronous protocol (AsynchronousScheduler,
scheduling/asynchronous_scheduler.h:12-18) re-dispatches a learner the
moment its task completes, after folding its model into the community model
with the recency rule FedRec (aggregation/federated_recency.cc:8-100: the
finisher's previous contribution is replaced in a running weighted sum);
only the finisher receives the new community model.

Here the learners of one GPU (models/colocated.py) run their tasks
concurrently on their own HIP streams and the aggregation never leaves the
device: when a learner's last launch of a task has completed (a HIP event,
polled by the host without blocking), the FedRec update runs on the
aggregator stream with the K2 rolling kernels --

    S -= w_old * theta_old ; S += w_new * theta_new ; Z += w_new - w_old
    theta_finisher <- S / Z

-- and the finisher's stream waits for it before its next task starts; the
other learners keep training throughout.  Community versions count FedRec
updates (the reference's global iterations); a learner's staleness is the
number of versions applied since the version it started its task from, with
the same staleness-aware weighting as the cross-GPU asynchronous plane
(async_federation.staleness_discount).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np
import torch

from metisfl_amd.ops import aggregate as agg
from metisfl_amd.parallel.async_federation import AsyncUpdate, staleness_discount


@dataclass
class _Slot:
    gen: object = None
    done_ev: object = None
    task: int = 0
    base_version: int = 0
    started: float = 0.0
    nsteps: int = 0


class CoLocatedAsyncFederation:
    """L learners on one device, FedRec over their latest models."""

    def __init__(self, group, cfg, num_local_updates: list[int] | None = None):
        self.group = group
        self.cfg = cfg
        nets = group.nets
        self.L = len(nets)
        self.nums = num_local_updates or [cfg.local_epochs * max(1, -(-d.n // cfg.batch_size))
                                          for d in group.train_dss]
        st0 = nets[0].state
        self.device = st0.model32.device
        self.cuda = self.device.type == "cuda"
        self.S = torch.zeros_like(st0.model32)
        self.Z = 0.0
        self.last = [None] * self.L
        self.last_w = [0.0] * self.L
        self.version = 0
        self.updates: list[AsyncUpdate] = []
        self.steps_done = [0] * self.L
        self.agg_stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self._stats: list[torch.Tensor] = []
        # every learner starts from learner 0's model (the initial community model)
        for net in nets[1:]:
            net.state.model32.copy_(st0.model32)
        for net in nets:
            net.state.refresh_bf16()
            net.state.set_anchor()

    def _weight(self, j: int) -> float:
        sf = self.cfg.scaling_factor
        if sf == "NUM_TRAINING_EXAMPLES":
            return float(self.group.train_dss[j].n)
        if sf == "NUM_COMPLETED_BATCHES":
            return float(self.nums[j])
        return 1.0

    def community(self) -> torch.Tensor:
        c = self.S.clone()
        agg.rolling_op(c, None, agg.SCALE_DIV, self.Z)
        return c

    def community_reference(self) -> np.ndarray:
        """Host recomputation over the latest contributions (tests)."""
        xs = [x.double().cpu().numpy() for x in self.last if x is not None]
        ws = [w for x, w in zip(self.last, self.last_w) if x is not None]
        return sum(w * x for w, x in zip(ws, xs)) / sum(ws)

    def _start(self, j: int, slot: _Slot) -> None:
        net, ds = self.group.nets[j], self.group.train_dss[j]
        with self.group._ctx(j):  # ordered after the previous FedRec's read of the statistics
            net.reset_train_stats()
        slot.nsteps = self.nums[j]
        slot.gen = net.train_steps_iter(ds, slot.nsteps, self.steps_done[j])
        slot.started = time.perf_counter()
        slot.base_version = self.version

    def _fedrec(self, j: int, slot: _Slot) -> None:
        """On the aggregator stream, after learner j's task: FedRec update,
        the new community model into learner j."""
        t0 = time.perf_counter()
        net = self.group.nets[j]
        theta = net.state.model32
        stale = self.version - slot.base_version
        w0 = self._weight(j)
        w = w0 * staleness_discount(self.cfg.staleness, stale, self.cfg.staleness_a, self.cfg.staleness_b)
        ctx = torch.cuda.stream(self.agg_stream) if self.cuda else _null()
        with ctx:
            if self.cuda:
                self.agg_stream.wait_event(slot.done_ev)
            if self.last[j] is not None:
                agg.rolling_op(self.S, self.last[j], agg.MERGE_SUB, self.last_w[j])
                self.Z -= self.last_w[j]
            else:
                self.last[j] = torch.empty_like(theta)
            agg.rolling_op(self.S, theta, agg.MERGE_ADD, w)
            self.Z += w
            self.last[j].copy_(theta)
            self.last_w[j] = w
            theta.copy_(self.S)
            agg.rolling_op(theta, None, agg.SCALE_DIV, self.Z)
            net.state.refresh_bf16()
            net.state.set_anchor()
            stats = net.stats.clone()  # the task's loss sums, read after the run (no host sync here)
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(self.agg_stream)
                self.group.streams[j].wait_event(ev)
        self.version += 1
        self._stats.append(stats)
        self.updates.append(AsyncUpdate(j, slot.task, w, time.time(), (time.perf_counter() - t0) * 1e3,
                                        float("nan"), slot.nsteps, stale, w0))
        self.steps_done[j] += slot.nsteps
        slot.task += 1

    def run(self, tasks_per_learner: int) -> list[AsyncUpdate]:
        """Every learner runs ``tasks_per_learner`` tasks; returns the FedRec
        updates applied (one per task, in completion order)."""
        group = self.group
        for net, ds, n in zip(group.nets, group.train_dss, self.nums):
            net.prepare_graphs(ds, n)
        group._fork()
        if self.cuda:
            self.agg_stream.wait_stream(torch.cuda.current_stream(self.device))
        slots = [_Slot() for _ in range(self.L)]
        for j, s in enumerate(slots):
            self._start(j, s)
        live = set(range(self.L))
        pending = {}  # j -> slot whose last launch is issued, completion not yet seen
        while live or pending:
            progressed = False
            for j in list(live):
                s = slots[j]
                with group._ctx(j):
                    try:
                        next(s.gen)
                        progressed = True
                        continue
                    except StopIteration:
                        pass
                    if self.cuda:
                        s.done_ev = torch.cuda.Event()
                        s.done_ev.record(group.streams[j])
                live.discard(j)
                pending[j] = s
            for j in list(pending):
                s = pending[j]
                if self.cuda and not s.done_ev.query():
                    continue
                del pending[j]
                self._fedrec(j, s)
                progressed = True
                if s.task < tasks_per_learner:
                    self._start(j, s)
                    live.add(j)
            if not progressed:
                time.sleep(0.0002)
        group._join()
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.agg_stream)
        for u, st in zip(self.updates[len(self.updates) - len(self._stats):], self._stats):
            v = st.cpu().numpy()
            u.train_loss = float(v[0] / max(1.0, float(v[2])))
        self._stats = []
        return self.updates


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
