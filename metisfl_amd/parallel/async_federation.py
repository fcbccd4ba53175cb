"""Asynchronous collective federation: FedRec over point-to-point RCCL.

The reference's asynchronous protocol re-dispatches every learner the moment
its task completes (AsynchronousScheduler, scheduling/asynchronous_scheduler.h:
12-18), aggregates over the latest model of every active learner
(ScheduledCardinality selector, selection/scheduled_cardinality.h:21-29) with
the recency rule FedRec (aggregation/federated_recency.cc:8-100: replace the
finisher's previous contribution in a running weighted sum) and sends the new
community model to the finisher only.  All models cross the controller as
serialized gRPC messages.

Here one process per GPU hosts a learner; rank 0
is also the aggregator.  A finished learner posts its task metadata to the
process group's key-value store (the control channel), then ``send``s its
flat fp32 model to rank 0 and ``recv``s the community model back -- one
point-to-point RCCL transfer each way over xGMI, nothing through the host.
Rank 0 keeps, in HBM, the running sum S = sum_i w_i theta_i, Z = sum_i w_i
and every learner's last contribution, and applies the FedRec update with
the K2 rolling kernels:

    S -= w_old * theta_old ; Z -= w_old        (learner seen before)
    S += w_new * theta_new ; Z += w_new
    community = S / Z

Staleness-aware weighting (the reference's FedRec has
none): rank 0 versions the community model (+1 per applied update) and
answers every submission with the new version through the store; a
learner's next submission carries the version it trained from, and its
FedRec weight is multiplied by cfg.staleness's discount of
t = version_now - version_base (``staleness_discount``).

Rank 0's aggregator runs in a service thread with its own process group
(point-to-point transfers) and its own HIP stream, so a finisher is served
the moment it posts -- rank 0's own training never blocks it (and is not
chunked).  ``serve_in_thread=False`` keeps the single-threaded variant: rank
0 trains in chunks of ``poll_every`` local steps and serves between chunks,
so a finisher waits up to one chunk.  The weights are the
NUM_TRAINING_EXAMPLES (or batch / participant) scaling inputs,
un-normalised, as FedRec consumes them.
"""
from __future__ import annotations

import json
import threading
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from metisfl_amd.ops import aggregate as agg
from metisfl_amd.parallel.comm import Comm
from metisfl_amd.parallel.federation import FederationConfig

_KEY = "metisfl_async/{}/{}/{}"
_VER = "metisfl_async/ver/{}/{}/{}"
_STOP = "metisfl_async/stop/{}"
_DONE = "metisfl_async/done/{}/{}"
_INSTANCES = [0]  # federations built so far in this process (identical on every rank)


def staleness_discount(kind: str, t: int, a: float = 0.5, b: int = 4) -> float:
    """FedAsync staleness functions (Xie et al. 2019): none / polynomial / hinge."""
    t = max(0, int(t))
    if kind in ("none", "", None):
        return 1.0
    if kind == "polynomial":
        return float((1.0 + t) ** (-a))
    if kind == "hinge":
        return 1.0 if t <= b else 1.0 / (a * (t - b) + 1.0)
    raise ValueError(f"unknown staleness function {kind!r}")


@dataclass
class AsyncUpdate:
    learner: int
    task: int
    weight: float
    received_at: float
    aggregation_ms: float
    train_loss: float
    completed_batches: int
    staleness: int = 0
    base_weight: float = 0.0


class AsyncCollectiveFederation:
    def __init__(self, comm: Comm, net, train_ds, cfg: FederationConfig, tasks_per_learner: int = 2,
                 poll_every: int = 16, store=None, broadcast_initial: bool = True,
                 serve_in_thread: bool = True, test_ds=None, engine=None):
        self.comm, self.net, self.train_ds, self.cfg = comm, net, train_ds, cfg
        self.test_ds = test_ds
        # rank 0: the controller bridge (engine_bridge.py) every FedRec update
        # and community evaluation is recorded with (runtime metadata, local
        # task lineage, community-model evaluations)
        self.engine = engine if comm.rank == 0 else None
        self.evaluations: list[dict] = []  # rank 0: {"version", "learner", "loss", "accuracy"}
        self._stop_flag = False            # termination mode (run_until)
        self._done: set[int] = set()
        self.rank, self.world = comm.rank, comm.world
        _INSTANCES[0] += 1
        self.tag = _INSTANCES[0]  # store-key namespace: repeated federations never see old keys
        self.tasks = tasks_per_learner
        self.poll_every = max(1, poll_every)
        self.threaded = bool(serve_in_thread) and comm.distributed
        # point-to-point model transfers on their own group (created on every
        # rank, a collective call): the service thread's sends / receives never
        # interleave with the default group's collectives
        self.p2p = dist.new_group(backend=comm.backend) if comm.distributed else None
        self._lock = threading.Lock()     # rank 0: FedRec state (S, Z, last, version)
        self._svc_error: BaseException | None = None
        self.store = store if store is not None else (
            dist.distributed_c10d._get_default_store() if comm.distributed else None)
        n = int(train_ds.n)
        self.num_local_updates = cfg.local_epochs * max(1, -(-n // cfg.batch_size))
        self.steps_done = 0
        self.updates: list[AsyncUpdate] = []   # rank 0: every FedRec update applied
        self.version = 0                       # rank 0: community model version
        self.base_version = 0                  # version this learner's current task started from
        st = net.state
        if broadcast_initial and comm.distributed:
            comm.broadcast_(st.model32, src=0)
            st.refresh_bf16()
            st.set_anchor()
        if self.rank == 0:
            dev = st.model32.device
            self.S = torch.zeros_like(st.model32)
            self.Z = 0.0
            self.last = [None] * self.world        # each learner's last contribution (HBM)
            self.last_w = [0.0] * self.world
            self.next_task = [0] * self.world       # next expected task per learner
            self.rbuf = torch.empty_like(st.model32, device=dev)

    # ---- learner side ------------------------------------------------------------
    def _weight(self, completed_batches: int) -> float:
        sf = self.cfg.scaling_factor
        if sf == "NUM_TRAINING_EXAMPLES":
            return float(self.train_ds.n)
        if sf == "NUM_COMPLETED_BATCHES":
            return float(completed_batches)
        return 1.0  # NUM_PARTICIPANTS

    def _train(self, nsteps: int) -> None:
        self.net.train_steps(self.train_ds, nsteps, step_offset=self.steps_done)
        self.steps_done += nsteps

    def _pending(self) -> bool:
        if self._until:
            return len(self._done) < self.world - 1
        return any(self.next_task[r] < self.tasks for r in range(1, self.world))

    _until = False

    def _serve_loop(self) -> None:
        """Rank 0 service thread: serve submissions as they arrive."""
        try:
            st = self.net.state
            if st.model32.is_cuda:
                torch.cuda.set_device(st.model32.device)
                stream = torch.cuda.Stream(device=st.model32.device)
                ctx = torch.cuda.stream(stream)
            else:
                import contextlib
                ctx = contextlib.nullcontext()
            with ctx:
                while self._pending():
                    if not self.serve(block=False):
                        time.sleep(0.0005)
        except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
            self._svc_error = e

    def run(self, debug_delay_s: float = 0.0) -> list[AsyncUpdate]:
        """Run ``tasks_per_learner`` asynchronous tasks on this learner; rank 0
        also serves every other learner's submissions until all are done.
        ``debug_delay_s``: sleep after each task (uneven learner speeds)."""
        svc = None
        if self.rank == 0 and self.threaded:
            svc = threading.Thread(target=self._serve_loop, name="metisfl-async-aggregator", daemon=True)
            svc.start()
        for task in range(self.tasks):
            self.net.reset_train_stats()
            left = self.num_local_updates
            while left > 0:
                k = min(left, self.poll_every) if (self.rank == 0 and not self.threaded) else left
                self._train(k)
                left -= k
                if self.rank == 0 and not self.threaded:
                    self.serve(block=False)
            if debug_delay_s:
                self._sync_stream()
                time.sleep(debug_delay_s)
            meta = {"task": task, "weight": self._weight(self.num_local_updates),
                    "loss": self.net.train_stats()["loss"], "batches": self.num_local_updates,
                    "base_version": self.base_version}
            if self.rank == 0:
                with self._lock:
                    self._fedrec(0, self.net.state.model32, meta)
                    self.net.state.model32.copy_(self._community())
                    self._sync_stream()
                    self.base_version = self.version
                self._install()
            else:
                self.store.set(_KEY.format(self.tag, self.rank, task), json.dumps(meta))
                dist.send(self.net.state.model32, dst=0, group=self.p2p)
                dist.recv(self.net.state.model32, src=0, group=self.p2p)
                self.base_version = int(self.store.get(_VER.format(self.tag, self.rank, task)))
                self._install()
        if self.rank == 0:
            if svc is not None:
                svc.join()
                if self._svc_error is not None:
                    raise RuntimeError("async aggregator thread failed") from self._svc_error
            else:
                while self._pending():
                    if not self.serve(block=False):
                        time.sleep(0.001)
        return self.updates

    def _sync_stream(self) -> None:
        t = self.net.state.model32
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()

    def _install(self) -> None:
        st = self.net.state
        st.refresh_bf16()
        st.set_anchor()

    # ---- aggregator side (rank 0) ---------------------------------------------------
    def serve(self, block: bool = False) -> int:
        """Apply every pending submission (FedRec) and answer it with the
        community model.  Returns the number served."""
        served = 0
        for r in range(1, self.world):
            t = self.next_task[r]
            if (not self._until and t >= self.tasks) or r in self._done:
                continue
            key = _KEY.format(self.tag, r, t)
            if not block and not self.store.check([key]):
                if self._until:
                    dkey = _DONE.format(self.tag, r)
                    if self.store.check([dkey]):  # its last submission was served
                        self._record_eval(r, json.loads(self.store.get(dkey)).get("eval"))
                        self._done.add(r)
                continue
            meta = json.loads(self.store.get(key))
            self._record_eval(r, meta.get("eval"))
            dist.recv(self.rbuf, src=r, group=self.p2p)
            with self._lock:
                self._fedrec(r, self.rbuf, meta)
                comm_model = self._community()
                ver = self.version
                self._sync_stream()
            self.store.set(_VER.format(self.tag, r, t), str(ver))
            dist.send(comm_model, dst=r, group=self.p2p)
            self.next_task[r] = t + 1
            served += 1
            self._after_update()
        return served

    def _fedrec(self, r: int, theta: torch.Tensor, meta: dict) -> None:
        t0 = time.perf_counter()
        stale = self.version - int(meta.get("base_version", self.version))
        w0 = float(meta["weight"])
        w = w0 * staleness_discount(self.cfg.staleness, stale, self.cfg.staleness_a, self.cfg.staleness_b)
        if self.last[r] is not None:
            agg.rolling_op(self.S, self.last[r], agg.MERGE_SUB, self.last_w[r])
            self.Z -= self.last_w[r]
        else:
            self.last[r] = torch.empty_like(theta)
        agg.rolling_op(self.S, theta, agg.MERGE_ADD, w)
        self.Z += w
        self.last[r].copy_(theta)
        self.last_w[r] = w
        self.version += 1
        if theta.is_cuda:  # this stream only: rank 0's training keeps running on its own
            torch.cuda.current_stream(theta.device).synchronize()
        up = AsyncUpdate(r, int(meta["task"]), w, time.time(), (time.perf_counter() - t0) * 1e3,
                         float(meta["loss"]), int(meta["batches"]), stale, w0)
        self.updates.append(up)
        if self.engine is not None:
            # one FederatedTaskRuntimeMetadata per community version + the
            # finisher's local task lineage (the reference's async controller
            # records both per completion, controller.cc:201-259, 428-518)
            self.engine.record_async_update(self.version, r, meta, up)

    def _community(self) -> torch.Tensor:
        c = self.S.clone()
        agg.rolling_op(c, None, agg.SCALE_DIV, self.Z)
        return c

    def community_reference(self) -> np.ndarray:
        """Host recomputation of sum_i w_i theta_i / sum_i w_i over the latest
        contributions (tests)."""
        xs = [x.double().cpu().numpy() for x in self.last if x is not None]
        ws = [w for x, w in zip(self.last, self.last_w) if x is not None]
        return sum(w * x for w, x in zip(ws, xs)) / sum(ws)


    # ---- termination-driven mode (the driver-launched asynchronous protocol) ------------
    def _record_eval(self, r: int, ev) -> None:
        """A learner's evaluation of the community model version it received
        (it rides in its next submission / its done message)."""
        if not ev:
            return
        rec = {"version": int(ev["version"]), "learner": r, "loss": float(ev["loss"]),
               "accuracy": float(ev["accuracy"]), "num_examples": int(ev.get("n", 0))}
        self.evaluations.append(rec)
        if self.engine is not None:
            self.engine.record_async_evaluation(rec)

    def _after_update(self) -> None:
        """Rank 0, after every FedRec update: the termination signals."""
        if not self._until or self._stop_flag:
            return
        why = None
        if self._max_updates and self.version >= self._max_updates:
            why = "rounds"
        elif self._deadline is not None and time.time() > self._deadline:
            why = "time"
        elif self._metric_cutoff is not None and self.evaluations:
            last = [e for e in self.evaluations if e["num_examples"]][-self.world:]
            vals = [e.get(self._metric) for e in last if e.get(self._metric) is not None]
            if vals and float(np.mean(vals)) >= self._metric_cutoff:
                why = "metric"
        if why is None and self.engine is not None and self.engine.should_stop():
            why = "driver"
        if why is not None:
            self._stop_flag = True
            self.stop_reason = why
            self.store.set(_STOP.format(self.tag), why)

    def _stopped(self) -> bool:
        if self.rank == 0:
            return self._stop_flag
        return bool(self.store.check([_STOP.format(self.tag)]))

    def _evaluate_received(self) -> dict | None:
        if self.test_ds is None or not self.cfg.evaluate_community:
            return None
        ev = self.net.evaluate(self.test_ds, self.cfg.eval_max_steps)
        return {"version": self.base_version, "loss": ev["loss"], "accuracy": ev["accuracy"], "n": self.test_ds.n}

    def run_until(self, max_updates: int | None = None, cutoff_s: float | None = None,
                  metric: str | None = None, metric_cutoff: float | None = None,
                  debug_delay_s: float = 0.0) -> list[AsyncUpdate]:
        """Asynchronous tasks until a termination signal: ``max_updates``
        community versions (FedRec updates -- the reference's global
        iterations), the wall-clock cutoff, the mean community-model test
        metric of the learners' latest evaluations, or the driver's stop
        request.  Every learner finishes the task it is running, is served,
        and leaves; rank 0 serves until all have left."""
        self._until = True
        self._max_updates = max_updates
        self._deadline = time.time() + cutoff_s if cutoff_s else None
        self._metric, self._metric_cutoff = metric, metric_cutoff
        self.stop_reason = None
        svc = None
        if self.rank == 0 and self.world > 1:
            if not self.threaded:
                raise RuntimeError("run_until needs the threaded aggregator (serve_in_thread=True)")
            svc = threading.Thread(target=self._serve_loop, name="metisfl-async-aggregator", daemon=True)
            svc.start()
        task, last_eval = 0, None
        spe = self.train_ds.steps_per_epoch
        while not self._stopped():
            self.net.reset_train_stats()
            t_task = time.time()
            self._train(self.num_local_updates)
            self._sync_stream()
            if debug_delay_s:
                time.sleep(debug_delay_s)  # test hook: uneven learner speeds
            ms_b = (time.time() - t_task) * 1e3 / max(1, self.num_local_updates)
            tr = self.net.train_stats()
            meta = {"task": task, "weight": self._weight(self.num_local_updates),
                    "loss": tr["loss"], "accuracy": tr["accuracy"], "batches": self.num_local_updates,
                    "base_version": self.base_version, "eval": last_eval, "started_at": t_task,
                    "n_train": int(self.train_ds.n), "ms_per_batch": ms_b, "ms_per_epoch": ms_b * spe,
                    "epochs": self.num_local_updates / spe}
            if self.rank == 0:
                with self._lock:
                    self._record_eval(0, last_eval)
                    self._fedrec(0, self.net.state.model32, meta)
                    self.net.state.model32.copy_(self._community())
                    self._sync_stream()
                    self.base_version = self.version
                    self._after_update()
                self._install()
            else:
                self.store.set(_KEY.format(self.tag, self.rank, task), json.dumps(meta))
                dist.send(self.net.state.model32, dst=0, group=self.p2p)
                dist.recv(self.net.state.model32, src=0, group=self.p2p)
                self.base_version = int(self.store.get(_VER.format(self.tag, self.rank, task)))
                self._install()
            last_eval = self._evaluate_received()
            task += 1
        if self.rank == 0:
            with self._lock:
                self._record_eval(0, last_eval)
            if svc is not None:
                svc.join()
                if self._svc_error is not None:
                    raise RuntimeError("async aggregator thread failed") from self._svc_error
        else:
            self.store.set(_DONE.format(self.tag, self.rank), json.dumps({"eval": last_eval}))
        self.tasks_run = task
        return self.updates
