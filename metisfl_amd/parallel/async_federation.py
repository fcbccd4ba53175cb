"""Asynchronous collective federation: ONE FedRec core for every placement.

The reference's asynchronous protocol re-dispatches every learner the moment
its task completes (AsynchronousScheduler, scheduling/asynchronous_scheduler.h:
12-18), aggregates over the latest model of every active learner
(ScheduledCardinality selector, selection/scheduled_cardinality.h:21-29) with
the recency rule FedRec (aggregation/federated_recency.cc:8-100: replace the
finisher's previous contribution in a running weighted sum) and sends the new
community model to the finisher only.  Scheduling is per learner, whatever
the placement -- its own asynchronous configs put all 10 learners on GPU 0
(examples/config/fashionmnist/test_localhost_asynchronous_vanillasgd.yaml).
All models cross the controller as serialized gRPC messages.

Here one process per GPU hosts that GPU's learners (``nets``: one or several,
co-located on their own HIP streams as in models/colocated.py); rank 0 is
also the aggregator.  Every learner -- global id ``g`` in the job's learner
order -- is its own FedRec participant:

* a learner hosted by rank 0 folds its model into the running sum on the
  device, under the aggregator lock, the moment its task's last launch has
  completed (a HIP event polled without blocking the other learners);
* a learner hosted by another rank posts its task metadata to the process
  group's key-value store (the control channel), ``send``s its flat fp32
  model to rank 0 and ``recv``s the community model back -- one point-to-point
  RCCL transfer each way over xGMI, nothing through the host.  Rank 0's
  service thread (own process group, own HIP stream) serves those.

Rank 0 keeps, in HBM, S = sum_g w_g theta_g, Z = sum_g w_g and every
learner's last contribution, and applies the FedRec update with the K2
rolling kernels:

    S -= w_old * theta_old ; Z -= w_old        (learner seen before)
    S += w_new * theta_new ; Z += w_new
    community = S / Z

Staleness-aware weighting (the reference's FedRec has
none): rank 0 versions the community model (+1 per applied update); a
learner's next submission carries the version it trained from, and its
FedRec weight is multiplied by cfg.staleness's discount of
t = version_now - version_base (``staleness_discount``).

Failure handling (in the reference one lost learner never ends
an asynchronous federation: controller.cc:171-199 removes it and the
asynchronous scheduler keeps serving the others).  ``run_until`` with a
checkpoint directory writes, every ``checkpoint_every`` community versions,
the aggregator's FedRec state (S, Z, every learner's last contribution and
weight -- keyed by STABLE learner id, ``last:<id>`` -- and the version) plus
the community model as a ``FederatedModel`` (``<dir>/round_<version>/``,
LATEST), and every learner's local state after its tasks
(``<dir>/async_learner_<id>.pt``) -- staged on the device and written by
background threads (parallel/checkpoint.py).  After a lost rank the driver
relaunches the survivors (possibly regrouped onto fewer ranks); ``resume``
restores the FedRec state of the learner ids still present, drops the lost
ones' contributions from S and Z, restarts every survivor from the restored
community model and continues the version count.  The controller
bookkeeping (runtime metadata per version, the driver's stop request) goes
through a queue served by its own thread, never under the aggregator lock.

Secure aggregation (``cfg.secure_aggregation``; the reference's
test_localhost_asynchronous_vanillasgd_with_fhe.yaml): learners submit CKKS
ciphertexts instead of models and rank 0 keeps each learner's latest
ciphertext and answers with the private weighted average over them
(``AsyncPWA``); checkpoints then hold ciphertexts only.
"""
from __future__ import annotations

import contextlib
import json
import os
import queue
import threading
import time
from dataclasses import dataclass, field

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


class AsyncPWA:
    """The encrypted side of the asynchronous protocol (secure aggregation).

    The reference's controller keeps every learner's latest encrypted model
    and computes the private weighted average over them when a learner
    completes (aggregation/private_weighted_average.cc:24-82 over the
    ScheduledCardinality selection); only learners hold the private key.
    Here a finishing learner encrypts its flat model where it lives (device
    RNS-CKKS, kernels/ckks.hip), the ciphertext crosses to rank 0 over the
    process group (point-to-point), rank 0 keeps the latest ciphertext of
    every learner in HBM and runs the PWA over them (K9, one launch over all
    learners, weights normalised to sum 1), and the finisher decrypts the
    community ciphertext it gets back.  The aggregator never decrypts.  On a
    CPU process group the host scheme (csrc/he/ckks.cc) does the same on
    MCK1 byte blobs carried as uint8 tensors."""

    def __init__(self, scheme, device: torch.device, n: int):
        from metisfl_amd.encryption.fhe import WEIGHT_BITS
        self.scheme, self.n, self.device = scheme, int(n), torch.device(device)
        self.wbits = WEIGHT_BITS
        self.dev = None
        if self.device.type == "cuda":
            from metisfl_amd.encryption.device import DeviceCKKS
            self.dev = DeviceCKKS(scheme, self.device)
            self.numel, self.dtype = self.dev.ct_numel(self.n), torch.int64
            self.nct = self.dev.num_ciphertexts(self.n)
        else:
            self.numel, self.dtype = len(scheme.encrypt(np.zeros(self.n))), torch.uint8

    def buffer(self) -> torch.Tensor:
        return torch.empty(self.numel, dtype=self.dtype, device=self.device)

    def encrypt(self, flat: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if self.dev is not None:
            return self.dev.encrypt(flat, out=out)
        b = self.scheme.encrypt(flat.detach().double().reshape(-1).numpy())
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        if out is None:
            return t
        out.copy_(t)
        return out

    def pwa(self, cts: list, weights: list[float], out: torch.Tensor | None = None) -> torch.Tensor:
        """Enc(sum_i w_i theta_i / sum_i w_i) from the learners' ciphertexts."""
        z = float(sum(weights))
        ws = [float(w) / z for w in weights]
        if self.dev is None:
            b = self.scheme.compute_weighted_average([bytes(c.numpy().tobytes()) for c in cts], ws)
            t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
            return t if out is None else out.copy_(t)
        from metisfl_amd.ops._native import ops
        d = self.dev
        if out is None:
            out = self.buffer()
        wq = np.zeros((len(ws), d.L, 2), dtype=np.uint64)
        for i, w in enumerate(ws):
            wi = int(round(w * (1 << self.wbits)))
            for j, qj in enumerate(d.q):
                r = wi % qj
                wq[i, j] = (r, (r << 64) // qj)  # Shoup precomputation
        ptrs = torch.tensor([c.data_ptr() for c in cts], dtype=torch.int64).to(self.device)
        wqt = torch.from_numpy(wq.view(np.int64).reshape(-1)).to(self.device)
        ops().ckks_pwa(ptrs, wqt, out, d.tables[0], d.L, d.N, self.nct)
        return out

    def decrypt_into(self, ct: torch.Tensor, flat: torch.Tensor) -> None:
        """flat <- Dec(community ciphertext) (the PWA's scale: 2^(bits + 30))."""
        if self.dev is not None:
            self.dev.decrypt(ct, self.n, self.dev.bits + self.wbits, out=flat.view(-1))
            return
        v = self.scheme.decrypt(bytes(ct.numpy().tobytes()), self.n)
        flat.view(-1).copy_(torch.from_numpy(np.asarray(v)).to(flat.dtype))

    def decrypt_fresh(self, ct: torch.Tensor) -> np.ndarray:
        """A learner's own (unweighted) ciphertext -> host fp64 (tests)."""
        if self.dev is not None:
            return self.dev.decrypt(ct, self.n, dtype=torch.float64).cpu().numpy()
        return np.asarray(self.scheme.decrypt(bytes(ct.numpy().tobytes()), self.n), dtype=np.float64)


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


@dataclass
class _Local:
    """One learner hosted by this rank."""
    j: int                      # index among this rank's learners
    gid: int                    # global learner index (the job's learner order)
    lid: str                    # stable learner id (checkpoint keys)
    net: object
    train_ds: object
    test_ds: object
    num_local_updates: int
    steps_done: int = 0
    base_version: int = 0       # community version its current task started from
    task_index: int = 0         # tasks completed (kept across a resume)
    sub: int = 0                # this run's submissions (store keys)
    last_eval: dict | None = None
    gen: object = None          # the running task's launch generator
    done_ev: object = None
    started: float = 0.0
    finished: bool = False
    lckpt: object = None
    tasks_run: int = 0
    extra: dict = field(default_factory=dict)


class AsyncCollectiveFederation:
    """``nets`` / ``train_dss`` / ``test_ds``: this rank's learner(s) (a model or
    a list).  ``gids``: their global learner indices and ``owners[g]``: the
    rank hosting learner g (default: one learner per rank, learner g on rank
    g).  ``learner_ids``: stable ids of all learners, by global index."""

    def __init__(self, comm: Comm, nets, train_dss, cfg: FederationConfig, tasks_per_learner: int = 2,
                 poll_every: int = 16, store=None, broadcast_initial: bool = True,
                 serve_in_thread: bool = True, test_ds=None, engine=None, gids=None, owners=None,
                 learner_ids=None, streams=None):
        single = not isinstance(nets, (list, tuple))
        nets = [nets] if single else list(nets)
        train_dss = [train_dss] if single else list(train_dss)
        test_dss = ([test_ds] if single else list(test_ds)) if test_ds is not None else [None] * len(nets)
        self.comm, self.cfg = comm, cfg
        self.rank, self.world = comm.rank, comm.world
        if owners is None:
            owners = list(range(self.world)) if len(nets) == 1 else [0] * len(nets)
        self.owners = [int(o) for o in owners]
        self.G = len(self.owners)
        if gids is None:
            gids = [g for g, o in enumerate(self.owners) if o == self.rank]
        assert len(gids) == len(nets), (gids, len(nets))
        self.learner_ids = list(learner_ids) if learner_ids else [f"learner_{g}" for g in range(self.G)]
        self.engine = engine if comm.rank == 0 else None
        self.evaluations: list[dict] = []  # rank 0: {"version", "learner", "loss", "accuracy"}
        self._stop_flag = False            # termination mode (run_until)
        self._done: set[int] = set()       # rank 0: remote learners that left (global ids)
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
        self.learners = [
            _Local(j, int(g), self.learner_ids[int(g)], n, d, t,
                   cfg.local_epochs * max(1, -(-int(d.n) // cfg.batch_size)))
            for j, (g, n, d, t) in enumerate(zip(gids, nets, train_dss, test_dss))]
        self.updates: list[AsyncUpdate] = []   # rank 0: every FedRec update applied
        self.version = 0                       # rank 0: community model version
        self.ckpt_dir: str | None = None
        self.ckpt_every = 0
        self.snapshot_every = int(getattr(cfg, "snapshot_every", 0) or 0)
        self._ckpt = self._lineage = None
        self._bk_q: queue.Queue | None = None
        self._bk_thread = None
        self._driver_stop = False
        st = self.net.state
        self.cuda = st.model32.is_cuda
        # the host-side reads and the rank-0 FedRec of local learners run on a
        # high-priority stream: a hardware queue of its own (HIP keeps queues
        # per priority), so they never wait in FIFO order behind the learner
        # graphs queued on a shared in-order queue (8 learner streams share 4)
        self._hp = None
        if st.model32.is_cuda and os.environ.get("MFL_ASYNC_HP", "1") == "1":  # (=0: A/B runs only)
            lo, hi = torch.cuda.Stream.priority_range()
            self._hp = torch.cuda.Stream(device=st.model32.device, priority=hi)
        # co-located learners replay their step graphs on their own streams
        if streams is not None:
            self.streams = list(streams)
        elif self.cuda and len(nets) > 1:
            self.streams = [torch.cuda.Stream(device=st.model32.device) for _ in nets]
        else:
            self.streams = [None] * len(nets)
        if broadcast_initial and comm.distributed:
            comm.broadcast_(st.model32, src=0)
        for L in self.learners[1:]:  # every learner starts from the community model
            L.net.state.model32.copy_(st.model32)
        for L in self.learners:
            self._install(L)
        # secure aggregation: learners submit CKKS ciphertexts, rank 0 runs the
        # private weighted average over the latest ones (AsyncPWA)
        self.secure = bool(getattr(cfg, "secure_aggregation", False))
        self.he = None
        self._ct_buf = None
        if self.secure:
            from metisfl_amd.parallel.federation import setup_ckks
            scheme, self._he_dir = setup_ckks(comm, cfg)
            self.he = AsyncPWA(scheme, st.model32.device, st.model32.numel())
        if self.rank == 0:
            self.S = torch.zeros_like(st.model32)
            self.Z = 0.0
            # each learner's last contribution (HBM): its flat model, or its
            # ciphertext under secure aggregation
            self.last = [None] * self.G
            self.last_w = [0.0] * self.G
            self.next_task = [0] * self.G       # next expected submission per remote learner
            self.rbuf = self.he.buffer() if self.secure else torch.empty_like(st.model32)
        self.remote = [g for g, o in enumerate(self.owners) if o != 0]

    # ---- compatibility: the first hosted learner ----------------------------------
    @property
    def net(self):
        return self.learners[0].net

    @property
    def train_ds(self):
        return self.learners[0].train_ds

    @property
    def num_local_updates(self) -> int:
        return self.learners[0].num_local_updates

    @property
    def steps_done(self) -> int:
        return self.learners[0].steps_done

    @property
    def base_version(self) -> int:
        return self.learners[0].base_version

    @property
    def task_index(self) -> int:
        return self.learners[0].task_index

    # ---- learner side ------------------------------------------------------------
    def _weight(self, L: _Local, completed_batches: int) -> float:
        sf = self.cfg.scaling_factor
        if sf == "NUM_TRAINING_EXAMPLES":
            return float(L.train_ds.n)
        if sf == "NUM_COMPLETED_BATCHES":
            return float(completed_batches)
        return 1.0  # NUM_PARTICIPANTS

    def _ctx(self, L: _Local):
        s = self.streams[L.j]
        return torch.cuda.stream(s) if s is not None else contextlib.nullcontext()

    def _hp_after(self, ev):
        """The high-priority stream, ordered after event ``ev`` (a learner's
        task-end or evaluation-end marker), as a stream context."""
        if self._hp is None:
            return contextlib.nullcontext()
        if ev is not None:
            self._hp.wait_event(ev)
        return torch.cuda.stream(self._hp)

    def _sync_stream(self) -> None:
        if self.cuda:
            torch.cuda.current_stream(self.net.state.model32.device).synchronize()

    def _install(self, L: _Local) -> None:
        st = L.net.state
        st.refresh_bf16()
        st.set_anchor()
        self._order(L)

    def _order(self, L: _Local) -> None:
        """Learner L's stream waits for the work issued so far on the current
        stream: the community model copy, its bf16 / packed mirrors and FedProx
        anchor (``_install``), and the device-to-device staging of a learner
        checkpoint -- all issued outside ``_ctx(L)``.  Without it the
        learner's next graph replay (evaluation of the received model, its
        next task) could read a stale mirror or anchor, or overwrite m / v
        before the checkpoint copy read them."""
        s = self.streams[L.j]
        if s is not None and self.cuda:
            s.wait_stream(torch.cuda.current_stream(L.net.state.model32.device))

    def _start_task(self, L: _Local) -> None:
        # (ordered after the install / checkpoint staging by _order: those run
        # on the high-priority stream; ordering after the default stream here
        # would queue this learner behind whatever shares that stream's
        # in-order hardware queue)
        with self._ctx(L):
            L.net.reset_train_stats()
            L.gen = L.net.train_steps_iter(L.train_ds, L.num_local_updates, step_offset=L.steps_done)
        L.started = time.time()
        L.done_ev = None

    def _step(self, L: _Local) -> bool:
        """Issue the running task's next launch (one graph replay / eager
        step).  False once the task has issued everything."""
        with self._ctx(L):
            try:
                next(L.gen)
                return True
            except StopIteration:
                pass
            if self.cuda:
                L.done_ev = torch.cuda.Event()
                L.done_ev.record()
        L.gen = None
        return False

    def _task_meta(self, L: _Local, debug_delay_s: float) -> dict:
        """The finished task's metadata (host-side once its launches completed)."""
        if debug_delay_s:
            time.sleep(debug_delay_s)  # test hook: uneven learner speeds
        ms_b = (time.time() - L.started) * 1e3 / max(1, L.num_local_updates)
        L.steps_done += L.num_local_updates
        spe = L.train_ds.steps_per_epoch
        with self._hp_after(L.done_ev):
            tr = L.net.train_stats()
        return {"task": L.task_index, "weight": self._weight(L, L.num_local_updates),
                "loss": tr["loss"], "accuracy": tr["accuracy"], "batches": L.num_local_updates,
                "base_version": L.base_version, "eval": self._eval_result(L), "started_at": L.started,
                "n_train": int(L.train_ds.n), "ms_per_batch": ms_b, "ms_per_epoch": ms_b * spe,
                "epochs": L.num_local_updates / spe}

    def _submit(self, L: _Local, meta: dict) -> None:
        """FedRec of the finished task; the learner leaves holding the new
        community model.  Runs on the high-priority stream after the task's
        end marker; the learner's stream is ordered after it (``_install``)."""
        with self._hp_after(L.done_ev):
            self._submit_body(L, meta)

    def _submit_body(self, L: _Local, meta: dict) -> None:
        model = L.net.state.model32
        # secure aggregation: the learner encrypts its model where it lives and
        # decrypts the community ciphertext it gets back
        # (one ciphertext buffer per rank: this rank's submissions are sequential
        # and the aggregator copies what it keeps)
        sub = self.he.encrypt(model, out=self._ct_buf) if self.secure else model
        if self.secure:
            self._ct_buf = sub
        if self.rank == 0:
            with self._lock:
                self._record_eval(L.gid, meta.get("eval"))
                self._fedrec(L.gid, sub, meta)
                back = self._community()
                if not self.secure:
                    model.copy_(back)
                self._sync_stream()
                L.base_version = self.version
                self._after_update()
        else:
            self.store.set(_KEY.format(self.tag, L.gid, L.sub), json.dumps(meta))
            self.comm.send(sub, 0, group=self.p2p)
            back = sub if self.secure else model
            self.comm.recv(back, 0, group=self.p2p)
            L.base_version = int(self.store.get(_VER.format(self.tag, L.gid, L.sub)))
        if self.secure:
            self.he.decrypt_into(back, model)
        self._sync_stream()  # the learner's stream reads the model next
        self._install(L)
        L.sub += 1
        L.task_index += 1
        L.tasks_run += 1

    def _evaluate_received(self, L: _Local) -> None:
        """Issue learner L's evaluation of the community model it received
        on its own stream (ahead of its next task there) without waiting:
        the host goes on serving the other learners; the result is read when
        it is needed -- in L's next submission, or when L leaves
        (``_eval_result``)."""
        L.last_eval = None
        L.extra.pop("eval_owner", None)
        if L.test_ds is None or not self.cfg.evaluate_community:
            return
        ev = None
        with self._ctx(L):
            owner = L.net.begin_evaluate(L.test_ds, self.cfg.eval_max_steps)
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record()
        L.extra["eval_owner"] = (owner, L.base_version, ev)
        if owner is L.net:  # evaluated in the training statistics' buffer (no twin): read it before the next task
            self._eval_result(L)

    def _eval_result(self, L: _Local) -> dict | None:
        pend = L.extra.pop("eval_owner", None)
        if pend is not None:
            owner, ver, done = pend
            with self._hp_after(done):  # the read waits for this evaluation only
                ev = L.net.finish_evaluate(owner)
            L.last_eval = {"version": ver, "loss": ev["loss"], "accuracy": ev["accuracy"], "n": L.test_ds.n}
        return L.last_eval

    # ---- the event loop over this rank's learners ---------------------------------
    def _drive(self, more_tasks, debug_delay_s: float = 0.0, fault_task: int | None = None, on_fault=None,
               after_task=None) -> None:
        """Run this rank's learners concurrently (co-located: one stream each)
        until each has finished its last task.  ``more_tasks(L)``: whether
        learner L starts another task; ``after_task(L)``: called after each
        completed submission."""
        for L in self.learners:  # capture before the streams run concurrently
            L.net.prepare_graphs(L.train_ds, L.num_local_updates)
        if self.cuda:
            cur = torch.cuda.current_stream(self.net.state.model32.device)
            for s in self.streams:
                if s is not None:
                    s.wait_stream(cur)

        def start_or_finish(L: _Local) -> None:
            if more_tasks(L):
                if fault_task is not None and L.task_index + 1 == int(fault_task) and on_fault is not None:
                    self.flush()
                    on_fault(L.task_index + 1)
                self._start_task(L)
            else:
                L.finished = True
                self._leave(L)

        for L in self.learners:
            L.finished = False
            start_or_finish(L)
        chunked_server = self.rank == 0 and self.world > 1 and not self.threaded
        while not all(L.finished for L in self.learners):
            progressed = False
            for L in self.learners:
                if L.finished or L.gen is None:
                    continue
                if self._step(L):
                    progressed = True
                    if chunked_server:
                        self.serve(block=False)
            for L in self.learners:
                if L.finished or L.gen is not None:
                    continue
                if L.done_ev is not None and not L.done_ev.query():
                    continue
                progressed = True
                meta = self._task_meta(L, debug_delay_s)
                self._submit(L, meta)
                self._evaluate_received(L)
                if after_task is not None:
                    after_task(L)
                start_or_finish(L)
            if chunked_server:
                progressed = bool(self.serve(block=False)) or progressed
            if not progressed:
                time.sleep(0.0002)
        if self.cuda:
            cur = torch.cuda.current_stream(self.net.state.model32.device)
            for s in self.streams:
                if s is not None:
                    cur.wait_stream(s)

    def _leave(self, L: _Local) -> None:
        """A learner that starts no more tasks: its last evaluation reaches rank
        0 (remote learners: through their done message)."""
        if not self._until:
            return
        if self.rank == 0:
            with self._lock:
                self._record_eval(L.gid, self._eval_result(L))
        else:
            self.store.set(_DONE.format(self.tag, L.gid), json.dumps({"eval": self._eval_result(L)}))

    # ---- the two entry points -----------------------------------------------------
    _until = False

    def _pending(self) -> bool:
        if self._until:
            return len(self._done) < len(self.remote)
        return any(self.next_task[g] < self._goal[g] for g in self.remote)

    _goal: dict = {}  # rank 0, run(): the submission count each remote learner reaches

    def _serve_loop(self) -> None:
        """Rank 0 service thread: serve the remote learners' submissions as
        they arrive."""
        try:
            st = self.net.state
            if st.model32.is_cuda:
                torch.cuda.set_device(st.model32.device)
                # a hardware queue of its own (see self._hp)
                stream = torch.cuda.Stream(device=st.model32.device, priority=torch.cuda.Stream.priority_range()[1])
                ctx = torch.cuda.stream(stream)
            else:
                ctx = contextlib.nullcontext()
            with ctx:
                while self._pending():
                    if not self.serve(block=False):
                        time.sleep(0.0005)
        except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
            self._svc_error = e

    def _start_service(self):
        if self.rank == 0 and self.world > 1 and self.remote and self.threaded:
            svc = threading.Thread(target=self._serve_loop, name="metisfl-async-aggregator", daemon=True)
            svc.start()
            return svc
        return None

    def _end_service(self, svc) -> None:
        if self.rank != 0:
            return
        if svc is not None:
            svc.join()
            if self._svc_error is not None:
                raise RuntimeError("async aggregator thread failed") from self._svc_error
        else:
            while self._pending():
                if not self.serve(block=False):
                    time.sleep(0.001)

    def run(self, debug_delay_s: float = 0.0) -> list[AsyncUpdate]:
        """Run ``tasks_per_learner`` asynchronous tasks on every hosted learner;
        rank 0 also serves every remote learner's submissions until all are
        done.  ``debug_delay_s``: sleep after each task (uneven speeds)."""
        self._until = False
        if self.rank == 0:
            self._goal = {g: self.next_task[g] + self.tasks for g in self.remote}
        svc = self._start_service()
        start = {L.j: L.tasks_run for L in self.learners}
        self._drive(lambda L: L.tasks_run - start[L.j] < self.tasks, debug_delay_s)
        self._end_service(svc)
        self._close_bookkeeping()
        return self.updates

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
        and leaves; rank 0 serves until all remote learners have left.
        ``checkpoint_dir`` / ``checkpoint_every``: see the module docstring;
        ``fault_task``: the rank calls ``on_fault`` when one of its learners
        is about to start that task (1 = its first; fault injection)."""
        self._until = True
        self.ckpt_dir, self.ckpt_every = checkpoint_dir, int(checkpoint_every or 0)
        self._max_updates = max_updates
        self._deadline = time.time() + cutoff_s if cutoff_s else None
        self._metric, self._metric_cutoff = metric, metric_cutoff
        self.stop_reason = None
        svc = self._start_service()

        def after(L: _Local) -> None:
            if self.ckpt_dir and self.ckpt_every and L.task_index % self.ckpt_every == 0:
                with self._hp_after(L.done_ev):  # staged after the task, before the next one
                    self._checkpoint_learner(L)
                    self._order(L)

        self._drive(lambda L: not self._stopped(), debug_delay_s, fault_task, on_fault, after)
        self._end_service(svc)
        if self.rank == 0 and self.ckpt_dir:
            self._checkpoint_aggregator(block=True)
        if self.ckpt_dir:
            for L in self.learners:
                self._checkpoint_learner(L, block=True)
        self.flush()
        self._close_bookkeeping()
        self.tasks_run = sum(L.tasks_run for L in self.learners)
        return self.updates

    # ---- aggregator side (rank 0) ---------------------------------------------------
    def serve(self, block: bool = False) -> int:
        """Apply every pending remote submission (FedRec) and answer it with
        the community model.  Returns the number served."""
        served = 0
        for g in self.remote:
            t = self.next_task[g]
            if (not self._until and t >= self._goal[g]) or g in self._done:
                continue
            key = _KEY.format(self.tag, g, t)
            if not block and not self.store.check([key]):
                if self._until:
                    dkey = _DONE.format(self.tag, g)
                    if self.store.check([dkey]):  # its last submission was served
                        with self._lock:
                            self._record_eval(g, json.loads(self.store.get(dkey)).get("eval"))
                        self._done.add(g)
                continue
            meta = json.loads(self.store.get(key))
            src = self.owners[g]
            self.comm.recv(self.rbuf, src, group=self.p2p)
            with self._lock:
                self._record_eval(g, meta.get("eval"))
                self._fedrec(g, self.rbuf, meta)
                comm_model = self._community()
                ver = self.version
                self._sync_stream()
                self._after_update()
            self.store.set(_VER.format(self.tag, g, t), str(ver))
            self.comm.send(comm_model, src, group=self.p2p)
            self.next_task[g] = t + 1
            served += 1
        return served

    def _fedrec(self, g: int, theta: torch.Tensor, meta: dict) -> None:
        t0 = time.perf_counter()
        stale = self.version - int(meta.get("base_version", self.version))
        w0 = float(meta["weight"])
        w = w0 * staleness_discount(self.cfg.staleness, stale, self.cfg.staleness_a, self.cfg.staleness_b)
        # plaintext: the FedRec running sum; secure: only the latest ciphertext
        # and weight are kept, the PWA runs over all of them (_community)
        if self.last[g] is not None:
            if not self.secure:
                agg.rolling_op(self.S, self.last[g], agg.MERGE_SUB, self.last_w[g])
            self.Z -= self.last_w[g]
        else:
            self.last[g] = torch.empty_like(theta)
        if not self.secure:
            agg.rolling_op(self.S, theta, agg.MERGE_ADD, w)
        self.Z += w
        self.last[g].copy_(theta)
        self.last_w[g] = w
        self.version += 1
        k = int(getattr(self.cfg, "fedrec_resum_every", 0) or 0)
        if k and self.version % k == 0:
            self._resum()
        if theta.is_cuda:  # this thread's stream only: the learners keep running on theirs
            torch.cuda.current_stream(theta.device).synchronize()
        up = AsyncUpdate(g, int(meta["task"]), w, time.time(), (time.perf_counter() - t0) * 1e3,
                         float(meta["loss"]), int(meta["batches"]), stale, w0)
        self.updates.append(up)
        if self.engine is not None:
            # one FederatedTaskRuntimeMetadata per community version + the
            # finisher's local task lineage (the reference's async controller
            # records both per completion, controller.cc:201-259, 428-518);
            # sent by the bookkeeping thread, not under the aggregator lock
            self._bookkeep("update", self.version, g, meta, up)
        self._after_fedrec()

    def _resum(self) -> None:
        """S <- sum_g w_g theta_g and Z <- sum_g w_g, recomputed from every
        learner's last contribution (one K1 launch over the resident models;
        Z with exact fp64 summation): the rounding the incremental FedRec
        updates accumulated (S -= w_old theta_old; S += w_new theta_new, in
        fp32, every version) is dropped.  Secure aggregation keeps no running
        sum (the PWA runs over the latest ciphertexts)."""
        import math
        idx = [g for g in range(self.G) if self.last[g] is not None]
        if not idx:
            return
        self.Z = math.fsum(self.last_w[g] for g in idx)
        if not self.secure:
            agg.weighted_sum(self.S, [self.last[g] for g in idx], [self.last_w[g] for g in idx])

    def _community(self) -> torch.Tensor:
        """The community model as rank 0 hands it out: S / Z, or (secure
        aggregation) the PWA ciphertext over every learner's latest one."""
        if self.secure:
            idx = [g for g in range(self.G) if self.last[g] is not None]
            return self.he.pwa([self.last[g] for g in idx], [self.last_w[g] for g in idx])
        c = self.S.clone()
        agg.rolling_op(c, None, agg.SCALE_DIV, self.Z)
        return c

    def community(self) -> torch.Tensor:
        """Rank 0: the plaintext community model (secure aggregation: rank 0
        decrypts it as the host of its own learners -- the key pair is shared
        by all learners, as in the reference)."""
        c = self._community()
        if not self.secure:
            return c
        out = torch.empty_like(self.net.state.model32)
        self.he.decrypt_into(c, out)
        return out

    def community_reference(self) -> np.ndarray:
        """Host recomputation of sum_g w_g theta_g / sum_g w_g over the latest
        contributions (tests; secure aggregation: each learner's latest
        ciphertext decrypted on its own)."""
        if self.secure:
            xs = [self.he.decrypt_fresh(x) for x in self.last if x is not None]
        else:
            xs = [x.double().cpu().numpy() for x in self.last if x is not None]
        ws = [w for x, w in zip(self.last, self.last_w) if x is not None]
        return sum(w * x for w, x in zip(ws, xs)) / sum(ws)

    def _after_update(self) -> None:
        """Rank 0, under the lock, after every FedRec update: the termination
        signals."""
        if not self._until or self._stop_flag:
            return
        why = None
        if self._max_updates and self.version >= self._max_updates:
            why = "rounds"
        elif self._deadline is not None and time.time() > self._deadline:
            why = "time"
        elif self._metric_cutoff is not None and self.evaluations:
            last = [e for e in self.evaluations if e["num_examples"]][-self.G:]
            vals = [e.get(self._metric) for e in last if e.get(self._metric) is not None]
            if vals and float(np.mean(vals)) >= self._metric_cutoff:
                why = "metric"
        if why is None and self._driver_stop:
            why = "driver"
        if why is not None:
            self._stop_flag = True
            self.stop_reason = why
            if self.store is not None:
                self.store.set(_STOP.format(self.tag), why)

    def _stopped(self) -> bool:
        if self.rank == 0:
            return self._stop_flag
        return bool(self.store.check([_STOP.format(self.tag)]))

    # ---- termination-driven mode: evaluations ---------------------------------------
    def _record_eval(self, g: int, ev) -> None:
        """A learner's evaluation of the community model version it received
        (it rides in its next submission / its done message)."""
        if not ev:
            return
        rec = {"version": int(ev["version"]), "learner": g, "loss": float(ev["loss"]),
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
        # (secure aggregation: the aggregator holds no plaintext model to hand
        # to the controller's lineage)
        if self.snapshot_every and v % self.snapshot_every == 0:
            self._snapshot_community(block=False)

    _snap_sent = -1  # rank 0: last community version handed to the controller's lineage

    def _snapshot_community(self, block: bool) -> None:
        """Rank 0 (under the lock): hand community version ``self.version``
        to the controller's lineage, staged device-to-device and sent from a
        background thread.  Latest wins while a send is in flight
        (``block=False`` skips the version); ``flush`` re-sends the final
        version when it was skipped, as the synchronous path's
        ``flush_checkpoints`` does."""
        if self.engine is None or self.secure or not hasattr(self.engine, "snapshot_community"):
            return
        from metisfl_amd.parallel import checkpoint as ck
        if self._lineage is None:
            self._lineage = ck.AsyncSnapshot(self.S.device, "metisfl-async-lineage")
        st, engine, z, v = self.net.state, self.engine, float(self.Z), self.version
        if v == self._snap_sent or z == 0.0:
            return

        def write(h):
            flat = (h["S"].double() / z).float().numpy()
            engine.snapshot_community([sp.name for sp in st.specs],
                                      [flat[sp.offset: sp.offset + sp.numel].reshape(sp.shape) for sp in st.specs],
                                      [sp.trainable for sp in st.specs], v)
        if block:
            self._lineage.submit({"S": self.S}, write)
        elif self._lineage.try_submit({"S": self.S}, write) is None:
            return
        self._snap_sent = v

    def _checkpoint_aggregator(self, block: bool = False) -> None:
        from metisfl_amd.parallel import checkpoint as ck
        if self._ckpt is None:
            self._ckpt = ck.AsyncSnapshot(self.S.device, "metisfl-async-checkpoint")
        if self._ckpt.busy() and not block:
            return
        v, root, secure = self.version, self.ckpt_dir, self.secure
        # secure aggregation: the latest ciphertext of every learner (the
        # aggregator's whole state; no plaintext community model is written)
        tensors = {} if secure else {"S": self.S}
        for g, x in enumerate(self.last):
            if x is not None:
                tensors[f"last:{self.learner_ids[g]}"] = x
        meta = {"Z": float(self.Z), "version": v, "world": self.world, "learners": self.G,
                "learner_ids": list(self.learner_ids), "secure_aggregation": secure,
                "last_w": {self.learner_ids[g]: w for g, w in enumerate(self.last_w) if self.last[g] is not None},
                "protocol": "asynchronous", "global_iteration": v,
                "updates": [{"learner": self.learner_ids[u.learner], "task": u.task, "weight": u.weight,
                             "staleness": u.staleness} for u in self.updates[-1000:]]}
        st = self.net.state
        n_contrib = sum(1 for x in self.last if x is not None)

        def write(h):
            d = os.path.join(root, f"round_{v}")
            os.makedirs(d, exist_ok=True)
            state = {k: t.clone() for k, t in h.items()}
            ck.atomic_torch_save(state, os.path.join(d, "async_state.pt"))
            if not secure:
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

    @staticmethod
    def learner_file(root: str, lid: str) -> str:
        return os.path.join(root, f"async_learner_{lid}.pt")

    def _checkpoint_learner(self, L: _Local, block: bool = False) -> None:
        """Learner L's local state after a task, keyed by its stable id."""
        from metisfl_amd.parallel import checkpoint as ck
        if L.lckpt is None:
            L.lckpt = ck.AsyncSnapshot(L.net.state.model32.device, f"metisfl-async-learner-{L.lid}")
        st = L.net.state
        tensors = {"step": st.step, "perm": L.train_ds.perm}
        for k in ("m", "v", "anchor"):
            t = getattr(st, k)
            if t is not None:
                tensors[k] = t
        host = {"steps_done": L.steps_done, "base_version": L.base_version, "task": L.task_index}
        path = self.learner_file(self.ckpt_dir, L.lid)

        def write(h):
            d = {k: t.clone() for k, t in h.items()}
            d.update({k: torch.tensor(v) for k, v in host.items()})
            ck.atomic_torch_save(d, path)

        os.makedirs(self.ckpt_dir, exist_ok=True)
        if block:
            L.lckpt.submit(tensors, write)
            L.lckpt.wait()
        else:
            L.lckpt.try_submit(tensors, write)

    def flush(self) -> None:
        if self.rank == 0 and self._lineage is not None and self.snapshot_every:
            with self._lock:  # the final community version, if its snapshot was skipped
                self._snapshot_community(block=True)
        for w in [self._ckpt, self._lineage] + [L.lckpt for L in self.learners]:
            if w is not None:
                w.wait()

    def resume(self, path: str, prev_rank: int | None = None) -> None:
        """Collective.  Continue an asynchronous federation from its last
        checkpoint on (possibly) fewer learners, on any placement: every
        learner restores its local state from its own file (stable learner
        id), rank 0 restores the FedRec state of the learner ids present now
        and drops the contributions of the ones that are gone; everyone starts
        from the restored community model and the version count continues.
        (``prev_rank``: accepted for the driver's legacy relaunch arguments;
        state is matched by learner id.)"""
        from metisfl_amd.parallel import checkpoint as ck
        dev = self.net.state.model32.device
        for L in self.learners:
            st = L.net.state
            lpath = self.learner_file(path, L.lid)
            if not os.path.exists(lpath):
                continue
            d = torch.load(lpath, weights_only=True)
            st.step.copy_(d["step"].to(dev))
            for k in ("m", "v"):
                if k in d and getattr(st, k) is not None and d[k].numel() == getattr(st, k).numel():
                    getattr(st, k).copy_(d[k].to(dev))
            if d["perm"].numel() == L.train_ds.perm.numel():
                L.train_ds.perm.copy_(d["perm"].to(dev))
                L.steps_done = int(d["steps_done"])
            L.task_index = int(d["task"])
        found = ck.resolve(path)
        ver = torch.zeros(1, dtype=torch.float64, device=dev)
        st = self.net.state
        if self.rank == 0 and found is not None:
            with open(os.path.join(found, "federation.json")) as f:
                meta = json.load(f)
            state = torch.load(os.path.join(found, "async_state.pt"), weights_only=True)
            if bool(meta.get("secure_aggregation", False)) != self.secure:
                raise RuntimeError(f"checkpoint {found}: secure aggregation "
                                   f"{meta.get('secure_aggregation', False)}, this federation {self.secure}")
            S = self.S.clone() if self.secure else state["S"].to(dev)
            Z = float(meta["Z"])
            old_w = dict(meta["last_w"])
            present = {lid: g for g, lid in enumerate(self.learner_ids)}
            self.last = [None] * self.G
            self.last_w = [0.0] * self.G
            dropped = []
            for lid, w in old_w.items():
                x = state.get(f"last:{lid}")
                if x is None:
                    continue
                if lid in present:
                    g = present[lid]
                    self.last[g] = x.to(dev)
                    self.last_w[g] = float(w)
                else:  # the lost learners leave the running sum (secure: the PWA set)
                    if not self.secure:
                        agg.rolling_op(S, x.to(dev), agg.MERGE_SUB, float(w))
                    Z -= float(w)
                    dropped.append(lid)
            self.S.copy_(S)
            self.Z = Z
            self.version = int(meta["version"])
            self.resumed = {"version": self.version, "dropped": sorted(dropped)}
            # secure: rank 0 decrypts as the host of its own learners
            if any(x is not None for x in self.last):
                st.model32.copy_(self.community())
            ver[0] = self.version
        self.comm.broadcast_(ver, src=0)
        self.comm.broadcast_(st.model32, src=0)
        for L in self.learners:
            if L.net is not self.net:
                L.net.state.model32.copy_(st.model32)
            L.base_version = int(ver.item())
            self._install(L)
