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

Failure handling (in the reference one lost learner never ends
an asynchronous federation: controller.cc:171-199 removes it and the
asynchronous scheduler keeps serving the others).  ``run_until`` with a
checkpoint directory writes, every ``checkpoint_every`` community versions,
the aggregator's FedRec state (S, Z, every learner's last contribution and
weight, the version) plus the community model as a ``FederatedModel``
(``<dir>/round_<version>/``, LATEST), and every learner's local state after
its tasks (``<dir>/async_learner_rank<r>.pt``) -- staged on the device and
written by background threads (parallel/checkpoint.py).  After a lost rank
the driver relaunches the survivors; ``resume`` restores the FedRec state,
drops the lost learners' contributions from S and Z, restarts every survivor
from the restored community model and continues the version count.
The controller bookkeeping (runtime metadata per version, the driver's stop
request) goes through a queue served by its own thread, never under the
aggregator lock.
"""
from __future__ import annotations

import json
import os
import queue
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
        self.task_index = 0                    # tasks this learner completed (kept across a resume)
        self.ckpt_dir: str | None = None
        self.ckpt_every = 0
        self.snapshot_every = int(getattr(cfg, "snapshot_every", 0) or 0)
        self._ckpt = self._lckpt = self._lineage = None
        self._bk_q: queue.Queue | None = None
        self._bk_thread = None
        self._driver_stop = False
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
        self._close_bookkeeping()
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
            # records both per completion, controller.cc:201-259, 428-518);
            # sent by the bookkeeping thread, not under the aggregator lock
            self._bookkeep("update", self.version, r, meta, up)
        self._after_fedrec()

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
            self._bookkeep("eval", rec)

    # ---- controller bookkeeping off the aggregator's path -----------------
    STOP_POLL_S = 0.5

    def _bookkeep(self, kind: str, *args) -> None:
        if self._bk_q is None:
            self._bk_q = queue.Queue()
            self._bk_thread = threading.Thread(target=self._bookkeeping_loop, name="metisfl-async-bookkeeping",
                                               daemon=True)
            self._bk_thread.start()
        self._bk_q.put((kind, args))

    def _bookkeeping_loop(self) -> None:
        last_poll = 0.0
        while True:
            try:
                item = self._bk_q.get(timeout=self.STOP_POLL_S)
            except queue.Empty:
                item = None
            if item is not None:
                kind, args = item
                if kind == "close":
                    return
                try:
                    if kind == "update":
                        self.engine.record_async_update(*args)
                    elif kind == "eval":
                        self.engine.record_async_evaluation(*args)
                except Exception as e:  # noqa: BLE001 - bookkeeping must not kill the aggregator
                    print(f"[async] controller bookkeeping failed: {e!r}", flush=True)
            if self._until and time.time() - last_poll >= self.STOP_POLL_S:
                last_poll = time.time()
                try:
                    if self.engine.should_stop():
                        self._driver_stop = True
                except Exception:  # noqa: BLE001
                    pass

    def _close_bookkeeping(self) -> None:
        if self._bk_thread is not None:
            self._bk_q.put(("close", ()))
            self._bk_thread.join(timeout=30)
            self._bk_thread = None
            self._bk_q = None

    # ---- checkpoints / lineage snapshots / resume ------------------------------------
    def _after_fedrec(self) -> None:
        """Rank 0, under the lock, after a FedRec update: the periodic
        aggregator checkpoint and the controller's community-model lineage
        (both staged device-to-device and written in the background; skipped
        while the previous one is still being written)."""
        v = self.version
        if self.ckpt_dir and self.ckpt_every and v % self.ckpt_every == 0:
            self._checkpoint_aggregator(block=False)
        if self.engine is not None and self.snapshot_every and v % self.snapshot_every == 0 \
                and hasattr(self.engine, "snapshot_community"):
            from metisfl_amd.parallel import checkpoint as ck
            if self._lineage is None:
                self._lineage = ck.AsyncSnapshot(self.S.device, "metisfl-async-lineage")
            st, engine, z = self.net.state, self.engine, float(self.Z)

            def write(h):
                flat = (h["S"].double() / z).float().numpy()
                engine.snapshot_community([sp.name for sp in st.specs],
                                          [flat[sp.offset: sp.offset + sp.numel].reshape(sp.shape) for sp in st.specs],
                                          [sp.trainable for sp in st.specs], v)
            self._lineage.try_submit({"S": self.S}, write)

    def _checkpoint_aggregator(self, block: bool = False) -> None:
        from metisfl_amd.parallel import checkpoint as ck
        if self._ckpt is None:
            self._ckpt = ck.AsyncSnapshot(self.S.device, "metisfl-async-checkpoint")
        if self._ckpt.busy() and not block:
            return
        v, root = self.version, self.ckpt_dir
        tensors = {"S": self.S}
        for r, x in enumerate(self.last):
            if x is not None:
                tensors[f"last{r}"] = x
        meta = {"Z": float(self.Z), "last_w": list(self.last_w), "version": v, "world": self.world,
                "learner_ids": list(getattr(self, "learner_ids", [f"learner_{r}" for r in range(self.world)])),
                "protocol": "asynchronous", "global_iteration": v,
                "updates": [{"learner": u.learner, "task": u.task, "weight": u.weight, "staleness": u.staleness}
                            for u in self.updates[-1000:]]}
        st = self.net.state
        n_contrib = sum(1 for x in self.last if x is not None)

        def write(h):
            d = os.path.join(root, f"round_{v}")
            os.makedirs(d, exist_ok=True)
            state = {k: t.clone() for k, t in h.items()}
            ck.atomic_torch_save(state, os.path.join(d, "async_state.pt"))
            from metisfl_amd.proto import model_pb2
            from metisfl_amd.utils.tensor_codec import model_from_arrays
            flat = (h["S"].double() / meta["Z"]).float().numpy() if meta["Z"] else h["S"].numpy()
            fm = model_pb2.FederatedModel()
            fm.num_contributors = n_contrib
            fm.global_iteration = v
            fm.model.CopyFrom(model_from_arrays([sp.name for sp in st.specs],
                                                [flat[sp.offset: sp.offset + sp.numel].reshape(sp.shape)
                                                 for sp in st.specs], [sp.trainable for sp in st.specs]))
            ck.atomic_write(os.path.join(d, "community_model.pb"), fm.SerializeToString())
            ck.atomic_write(os.path.join(d, "federation.json"), json.dumps(meta).encode())
            ck.publish(root, f"round_{v}")

        os.makedirs(root, exist_ok=True)
        self._ckpt.submit(tensors, write)
        if block:
            self._ckpt.wait()

    def _checkpoint_learner(self, block: bool = False) -> None:
        """This learner's local state after a task (any rank)."""
        from metisfl_amd.parallel import checkpoint as ck
        if self._lckpt is None:
            self._lckpt = ck.AsyncSnapshot(self.net.state.model32.device, "metisfl-async-learner")
        st = self.net.state
        tensors = {"step": st.step, "perm": self.train_ds.perm}
        for k in ("m", "v", "anchor"):
            t = getattr(st, k)
            if t is not None:
                tensors[k] = t
        host = {"steps_done": self.steps_done, "base_version": self.base_version, "task": self.task_index}
        path = os.path.join(self.ckpt_dir, f"async_learner_rank{self.rank}.pt")

        def write(h):
            d = {k: t.clone() for k, t in h.items()}
            d.update({k: torch.tensor(v) for k, v in host.items()})
            ck.atomic_torch_save(d, path)

        os.makedirs(self.ckpt_dir, exist_ok=True)
        if block:
            self._lckpt.submit(tensors, write)
            self._lckpt.wait()
        else:
            self._lckpt.try_submit(tensors, write)

    def flush(self) -> None:
        for w in (self._ckpt, self._lckpt, self._lineage):
            if w is not None:
                w.wait()

    def resume(self, path: str, prev_rank: int | None = None) -> None:
        """Collective.  Continue an asynchronous federation from its last
        checkpoint on (possibly) fewer learners: rank 0 restores the FedRec
        state with the contributions of the learners still present (old rank
        ``prev_rank`` of each new rank) and without the lost ones, every
        learner restores its local state and starts from the restored
        community model; the version count continues."""
        from metisfl_amd.parallel import checkpoint as ck
        prev = self.rank if prev_rank is None else int(prev_rank)
        dev = self.net.state.model32.device
        prevs = self.comm.all_gather_rows(torch.tensor([float(prev)], dtype=torch.float64, device=dev))
        prevs = [int(x) for x in prevs.cpu().numpy()[:, 0]]
        st = self.net.state
        lpath = os.path.join(path, f"async_learner_rank{prev}.pt")
        if os.path.exists(lpath):
            d = torch.load(lpath, weights_only=True)
            st.step.copy_(d["step"].to(dev))
            for k in ("m", "v"):
                if k in d and getattr(st, k) is not None and d[k].numel() == getattr(st, k).numel():
                    getattr(st, k).copy_(d[k].to(dev))
            if d["perm"].numel() == self.train_ds.perm.numel():
                self.train_ds.perm.copy_(d["perm"].to(dev))
                self.steps_done = int(d["steps_done"])
            self.task_index = int(d["task"])
        found = ck.resolve(path)
        ver = torch.zeros(1, dtype=torch.float64, device=dev)
        if self.rank == 0 and found is not None:
            with open(os.path.join(found, "federation.json")) as f:
                meta = json.load(f)
            state = torch.load(os.path.join(found, "async_state.pt"), weights_only=True)
            S = state["S"].to(dev)
            Z = float(meta["Z"])
            old_w = list(meta["last_w"])
            self.last = [None] * self.world
            self.last_w = [0.0] * self.world
            keep = set()
            for r, p in enumerate(prevs):
                x = state.get(f"last{p}")
                if x is not None:
                    self.last[r] = x.to(dev)
                    self.last_w[r] = float(old_w[p])
                    keep.add(p)
            for p in range(int(meta["world"])):  # the lost learners leave the running sum
                x = state.get(f"last{p}")
                if p not in keep and x is not None:
                    agg.rolling_op(S, x.to(dev), agg.MERGE_SUB, float(old_w[p]))
                    Z -= float(old_w[p])
            self.S.copy_(S)
            self.Z = Z
            self.version = int(meta["version"])
            self.resumed = {"version": self.version, "dropped": sorted(set(range(int(meta["world"]))) - keep)}
            st.model32.copy_(self._community())
            ver[0] = self.version
        self.comm.broadcast_(ver, src=0)
        self.comm.broadcast_(st.model32, src=0)
        self.base_version = int(ver.item())
        st.refresh_bf16()
        st.set_anchor()

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
        if why is None and self._driver_stop:
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
                  debug_delay_s: float = 0.0, checkpoint_dir: str | None = None,
                  checkpoint_every: int = 0, fault_task: int | None = None,
                  on_fault=None) -> list[AsyncUpdate]:
        """Asynchronous tasks until a termination signal: ``max_updates``
        community versions (FedRec updates -- the reference's global
        iterations), the wall-clock cutoff, the mean community-model test
        metric of the learners' latest evaluations, or the driver's stop
        request.  Every learner finishes the task it is running, is served,
        and leaves; rank 0 serves until all have left.  ``checkpoint_dir`` /
        ``checkpoint_every``: see the module docstring; ``fault_task``: this
        learner calls ``on_fault`` when it is about to start that task (1 =
        its first; fault injection for tests)."""
        self._until = True
        self.ckpt_dir, self.ckpt_every = checkpoint_dir, int(checkpoint_every or 0)
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
        task, last_eval = self.task_index, None
        # submission keys count this run's tasks from 0 (rank 0's next_task
        # does): a resumed learner's task_index continues its lifetime count
        sub = 0
        spe = self.train_ds.steps_per_epoch
        while not self._stopped():
            if fault_task is not None and task + 1 == int(fault_task) and on_fault is not None:
                self.flush()
                on_fault(task + 1)
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
                self.store.set(_KEY.format(self.tag, self.rank, sub), json.dumps(meta))
                dist.send(self.net.state.model32, dst=0, group=self.p2p)
                dist.recv(self.net.state.model32, src=0, group=self.p2p)
                self.base_version = int(self.store.get(_VER.format(self.tag, self.rank, sub)))
                self._install()
            last_eval = self._evaluate_received()
            sub += 1
            task += 1
            self.task_index = task
            if self.ckpt_dir and self.ckpt_every and task % self.ckpt_every == 0:
                self._checkpoint_learner()
        if self.rank == 0:
            with self._lock:
                self._record_eval(0, last_eval)
            if svc is not None:
                svc.join()
                if self._svc_error is not None:
                    raise RuntimeError("async aggregator thread failed") from self._svc_error
            if self.ckpt_dir:
                self._checkpoint_aggregator(block=True)
        else:
            self.store.set(_DONE.format(self.tag, self.rank), json.dumps({"eval": last_eval}))
        if self.ckpt_dir:
            self._checkpoint_learner(block=True)
        self.flush()
        self._close_bookkeeping()
        self.tasks_run = task
        return self.updates
