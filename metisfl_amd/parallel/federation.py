"""Collective (single-node, one process per GPU) federation engine.

Each process hosts L >= 1 persistent learners (co-located on its GPU,
models/colocated.py) whose models, optimizer states and data shards stay
resident in HBM across rounds.  A synchronous FedAvg round is

  1. local training: ``num_local_updates`` graph-replayed steps,
  2. all-gather of a few scalars per learner (dataset size, completed
     batches, per-batch / per-epoch time, train metrics) -- the payload of the
     reference's MarkTaskCompleted metadata (learner.py:197-206),
  3. scaling factors from the configured scaler (identical on every rank, so
     no broadcast is needed; rank 0's native controller computes the same),
  4. in-place pre-scale ``theta_i *= w_i`` (K1) and ONE RCCL all-reduce of the
     flat model buffer: every learner now holds the community model, which is
     the reference's gather -> FedAvg -> RunTask broadcast
     (controller.cc:428-518, 795-950) collapsed into one collective.  With L
     co-located learners the rank first sums its own learners' scaled models
     (one K1 launch), so xGMI carries one model per GPU whatever L is.

Semi-synchronous rounds use the same barrier with per-learner step budgets
recomputed from the measured per-batch times (controller.cc:520-569).
Asynchronous federations (per-learner dispatch, FedRec) are
``async_federation.AsyncCollectiveFederation`` (point-to-point send / recv to
the aggregator rank) on this data plane, or the controller path (gRPC
control plane + native engine's asynchronous scheduler).

Rank 0 additionally drives the native controller engine (engine_bridge.py)
so the collective federation has the reference's runtime metadata, task
lineages and model quantifiers.  ``save_checkpoint`` / ``resume`` implement
SURVEY §5.4 (the reference has no checkpointing): the community model,
per-rank optimizer state, step counters and round history.
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict, dataclass, field

import numpy as np
import torch

from metisfl_amd.ops import optim as opt_ops
from metisfl_amd.parallel import scaling
from metisfl_amd.parallel.comm import Comm
from metisfl_amd.utils import tracing

META_FIELDS = ("num_training_examples", "completed_batches", "ms_per_batch", "ms_per_epoch",
               "train_loss", "train_accuracy", "completed_epochs", "global_iteration",
               "test_loss", "test_accuracy", "participated")


@dataclass
class FederationConfig:
    protocol: str = "synchronous"          # synchronous | semi_synchronous
    # fed_avg | fed_stride.  FedStride (federated_stride.cc:6-64) exists to bound
    # the AGGREGATOR's memory: the reference controller folds `stride_length`
    # learner models at a time into a rolling scaled sum instead of holding
    # all N.  On the collective data plane no process ever holds more than its
    # own model plus ring chunks (reduce-scatter + all-gather), so the bound
    # holds for any N and the rolling sum sum_i(w_i x_i) / sum_i(w_i) is ONE
    # scale + all-reduce; the result equals the engine's FedStride up to fp32
    # summation order (tests/test_collective_federation.py::test_fed_stride_*).
    aggregation: str = "fed_avg"
    scaling_factor: str = "NUM_TRAINING_EXAMPLES"
    stride_length: int = 0
    batch_size: int = 32
    local_epochs: int = 4
    semi_sync_lambda: float = 2.0
    semi_sync_recompute: bool = False
    evaluate_test: bool = True             # learner test-set eval at task end
    # every learner evaluates the NEW community model on its test shard after
    # the all-reduce (the reference's SendEvaluationTasks, controller.cc:469-485,
    # 571-587); rank 0 records the CommunityModelEvaluation with the round
    evaluate_community: bool = True
    # the community evaluation runs in the background, on a frozen copy of
    # the community model, while the learners train the next round (the
    # reference's evaluation is asynchronous too: SendEvaluationTasks is
    # dispatched after the round and digested by its own completion-queue
    # thread, controller.cc:469-485, 589-694); its results are recorded with
    # their round once complete (next round's end, or finish_evaluations)
    defer_community_eval: bool = False
    eval_max_steps: int | None = None
    # rank 0 hands the community model to the controller's lineage every
    # ``snapshot_every`` rounds (0: never; background thread, see
    # snapshot_community)
    snapshot_every: int = 1
    quantify: bool = True                  # per-variable zero counts of each community model
    jsonl_log: str | None = None           # rank 0: one JSON line per round (utils/tracing.py)
    # CKKS secure aggregation (reference: PWA over Palisade CKKS, HESchemeConfig
    # metis.proto:281-299, batch 4096 / 52 scaling bits in template_with_fhe.yaml)
    # asynchronous protocol: staleness-aware FedRec weights (FedAsync-style
    # discount s(t) of the staleness t = community version at submission -
    # version the learner trained from): "none" | "polynomial" (1+t)^-a |
    # "hinge" 1 if t <= b else 1 / (a (t - b) + 1)
    staleness: str = "none"
    staleness_a: float = 0.5
    staleness_b: int = 4
    # asynchronous protocol: every ``fedrec_resum_every`` community versions
    # the aggregator re-sums S = sum_g w_g theta_g from every learner's last
    # contribution (resident in HBM; one K1 launch) instead of carrying the
    # fp32 subtract / add running sum forever (0: never, the reference's
    # behaviour, federated_recency.cc:8-100)
    fedrec_resum_every: int = 32
    secure_aggregation: bool = False
    he_batch_size: int = 4096
    he_scaling_bits: int = 52
    # directory of the driver's CKKS key files (cryptocontext / public /
    # private key, driver_session.py): every rank loads them; None: rank 0
    # generates a key pair and broadcasts it
    he_key_dir: str | None = None
    # Straggler handling (the reference carries
    # GlobalModelSpecs.learners_participation_ratio, metis.proto:307, but
    # never acts on it).  A synchronous round closes once
    # ceil(participation_ratio * N) learners finished their budget, or at
    # round_deadline_s: learners still training then stop, contribute weight
    # 0 (their partial work is discarded) and receive the community model.
    # Progress is polled every poll_steps local updates (host-side, over the
    # process group's key-value store -- no collective, no GPU sync beyond
    # the chunk boundary).
    participation_ratio: float = 1.0
    round_deadline_s: float | None = None
    poll_steps: int = 64
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
    allreduce_ms: float = 0.0              # the model all-reduce alone
    allreduce_gbps: float = 0.0            # algorithm bandwidth: model bytes / all-reduce time
    hbm_used_bytes: int = 0
    he_stats: dict | None = None           # secure aggregation: encrypt / all-reduce / decrypt ms
    # per-learner test metrics of the community model (rank order), and the
    # time the evaluation took: after the barrier (outside completed_at -
    # started_at, as in the reference) but inside round_ms
    community_eval: list | None = None
    community_eval_ms: float = 0.0
    snapshot_ms: float = 0.0               # rank 0: staging the community model for the controller's lineage
    checkpoint_ms: float = 0.0             # this rank: time the round's checkpoint held it (staging)
    # host wall time of the round's phases (local_train: training + the
    # learners' test evaluations; gather: metadata all-gather; aggregate;
    # community_eval; bookkeeping: controller records, quantifiers, lineage
    # snapshot -- after round_ms)
    phase_ms: dict | None = None

    def to_json(self) -> dict:
        d = asdict(self)
        d["learner_meta"] = self.learner_meta.tolist()
        return d


def install_community_model(net, fm, he_scheme=None) -> None:
    """Install a ``FederatedModel`` (proto or serialized bytes) into ``net``
    as the community model, matching variables by name (``he_scheme``:
    decrypts ciphertext variables, e.g. the driver's initial model under
    CKKS)."""
    from metisfl_amd.proto import model_pb2
    from metisfl_amd.utils.tensor_codec import model_to_arrays
    if isinstance(fm, (bytes, bytearray)):
        m = model_pb2.FederatedModel()
        m.ParseFromString(bytes(fm))
        fm = m
    names, arrays, _ = model_to_arrays(fm.model, he_scheme)
    st = net.state
    st.load_numpy(dict(zip(names, arrays)))
    st.set_anchor()


def learner_file(learner_id: str) -> str:
    """Checkpoint file of one learner's local state (optimizer slots, step
    counter, epoch permutation)."""
    safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in str(learner_id))
    return f"learner_{safe}.safetensors"


def setup_ckks(comm: Comm, cfg: FederationConfig):
    """Collective.  One CKKS key pair shared by all learners (the reference's
    driver generates it once, driver_session.py:122-135): rank 0 generates,
    the key files travel as bytes over the process group -> (scheme, key
    directory of this rank)."""
    import tempfile

    from metisfl_amd.encryption import CKKS
    names = ("cryptocontext.txt", "key-public.txt", "key-private.txt")
    scheme = CKKS(cfg.he_batch_size, cfg.he_scaling_bits)
    if cfg.he_key_dir:
        scheme.load_context_and_keys_from_files(*(os.path.join(cfg.he_key_dir, nm) for nm in names))
        return scheme, cfg.he_key_dir
    d = tempfile.mkdtemp(prefix=f"metisfl_amd_ckks_r{comm.rank}_")
    blobs = []
    if comm.rank == 0:
        scheme.gen_crypto_context_and_keys(d)
        for nm in names:
            with open(os.path.join(d, nm), "rb") as f:
                blobs.append(f.read())
    for i, nm in enumerate(names):
        b = comm.broadcast_bytes(blobs[i] if comm.rank == 0 else None)
        if comm.rank != 0:
            with open(os.path.join(d, nm), "wb") as f:
                f.write(b)
    if comm.rank != 0:
        scheme.load_context_and_keys_from_files(*(os.path.join(d, nm) for nm in names))
    return scheme, d


class DeferredCommunityEval:
    """The community model's evaluation on every local learner's test shard,
    run on its own stream over a FROZEN copy of the model (``FlatState.
    detached_copy``), so the learners train the next round meanwhile.  One
    snapshot serves all co-located learners (they hold the same community
    model); each learner's shard is evaluated by a model of its architecture
    bound to the snapshot (its evaluation twin)."""

    def __init__(self, nets: list, test_dss: list):
        self.src = nets[0].state
        self.state = self.src.detached_copy()
        self.evals = [n.detached_evaluator(d, self.state) if d is not None else None
                      for n, d in zip(nets, test_dss)]
        self.stream = self._make_stream(self.src.model32.device)
        self.event = torch.cuda.Event()
        self.pending = None  # (global_iteration, owners)

    # The evaluation stream must not share a hardware queue with a learner:
    # HIP deals streams round-robin onto GPU_MAX_HW_QUEUES (4) in-order queues,
    # so on a shared queue the whole evaluation runs in FIFO order ahead of
    # that queue's learners' next round (measured: two of 8 learners started
    # ~70 ms late).  A high-priority stream gets a queue of its own (HIP keeps
    # queues per priority); MFL_CE_STREAM=plain|cumask|prio (default prio) for
    # A/B runs -- cumask: a full-chip CU-masked stream, also a queue of its own.
    stream_kind = os.environ.get("MFL_CE_STREAM", "prio")

    @classmethod
    def _make_stream(cls, dev):
        if cls.stream_kind == "plain":
            return torch.cuda.Stream(device=dev)
        if cls.stream_kind == "cumask":
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            words = (ncu + 31) // 32
            arr = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
            h = ctypes.c_void_p()
            with torch.cuda.device(dev):
                if hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), arr) != 0:
                    raise RuntimeError("hipExtStreamCreateWithCUMask failed")
            return torch.cuda.ExternalStream(h.value, device=dev)
        lo, hi = torch.cuda.Stream.priority_range()
        return torch.cuda.Stream(device=dev, priority=hi)

    @classmethod
    def build(cls, nets: list, test_dss: list):
        """None when a learner's model has no detached evaluator (models
        without evaluation twins, CPU runs): evaluation stays synchronous."""
        if not nets or nets[0].state.model32.device.type != "cuda" or not hasattr(nets[0], "detached_evaluator"):
            return None
        if all(d is None for d in test_dss):
            return None
        ev = cls(nets, test_dss)
        if any(e is None for e, d in zip(ev.evals, test_dss) if d is not None):
            return None
        return ev

    def submit(self, global_iteration: int, max_steps: int | None = None) -> None:
        """Snapshot the community model (current stream order) and issue the
        evaluations on the side stream; no host wait."""
        assert self.pending is None, "collect the previous evaluation first"
        cur = torch.cuda.current_stream(self.src.model32.device)
        self.stream.wait_stream(cur)
        owners = []
        with torch.cuda.stream(self.stream):
            self.state.copy_model_from(self.src)
            for e in self.evals:
                owners.append(None if e is None else e[0].begin_evaluate(e[1], max_steps))
            self.event.record()
        self.pending = (global_iteration, owners)

    def collect(self):
        """-> (global_iteration, [metrics or None per local learner]) of the
        submitted evaluation (waits for it), or None."""
        if self.pending is None:
            return None
        gi, owners = self.pending
        self.pending = None
        self.event.synchronize()
        out = []
        for e, o in zip(self.evals, owners):
            out.append(None if o is None else e[0].finish_evaluate(o))
        return gi, out


class CollectiveFederation:
    """Drives rounds for the learner(s) hosted by this rank.

    ``net`` / ``train_ds`` / ``test_ds``: one learner, or lists of the L
    learners co-located on this rank's GPU (the same L on every rank).
    Learner ``j`` of rank ``r`` is global learner ``r * L + j``: metadata
    rows, aggregation weights, step budgets and learner ids are per global
    learner, in that order."""

    def __init__(self, comm: Comm, net, train_ds, cfg: FederationConfig, test_ds=None,
                 learner_ids: list[str] | None = None, engine=None, broadcast_initial: bool = True):
        self.comm = comm
        nets = list(net) if isinstance(net, (list, tuple)) else [net]
        tds = list(train_ds) if isinstance(train_ds, (list, tuple)) else [train_ds]
        vds = list(test_ds) if isinstance(test_ds, (list, tuple)) else [test_ds] * len(nets)
        if not (len(nets) == len(tds) == len(vds)):
            raise ValueError(f"{len(nets)} learners, {len(tds)} train / {len(vds)} test datasets")
        self.L = len(nets)
        self.nets, self.train_dss, self.test_dss = nets, tds, vds
        self.net, self.train_ds, self.test_ds = nets[0], tds[0], vds[0]
        self.group = None
        if self.L > 1:
            from metisfl_amd.models.colocated import CoLocatedLearners
            self.group = CoLocatedLearners(nets, tds, vds)
        self.cfg = cfg
        self.engine = engine if comm.rank == 0 else None
        self.world = comm.world
        self.rank = comm.rank
        # co-located learners per rank (may differ: learners grouped by device)
        Ls = comm.all_gather_rows(torch.tensor([float(self.L)], dtype=torch.float64, device=comm.device))
        self.Ls = [int(x) for x in Ls.cpu().numpy()[:, 0]]
        self.Lmax = max(self.Ls)
        self.offsets = [sum(self.Ls[:r]) for r in range(self.world)]
        self.n_learners = sum(self.Ls)
        self._local_done = 0  # quorum counter of a one-process federation (no store)
        self.learner_ids = learner_ids or [f"learner_{r}" for r in range(self.n_learners)]
        # reference: num_local_updates = epochs * ceil(N_train / batch) per
        # learner (controller.cc:148-153); the join-time dataset sizes are
        # exchanged once
        sizes = self._gather_learner_rows([[float(d.n)] for d in tds])[:, 0]
        self.dataset_sizes = [int(x) for x in sizes]
        self.num_local_updates = [cfg.local_epochs * max(1, math.ceil(n / cfg.batch_size))
                                  for n in self.dataset_sizes]
        self.steps_done_l = [0] * self.L
        self._ckpt = self._lineage = None   # background writers (parallel/checkpoint.py)
        self._ckpt_tag = f"{os.getpid()}_{id(self)}" if comm.rank == 0 else ""
        if comm.distributed:  # every rank uses rank 0's tag for its store keys
            self._ckpt_tag = comm.broadcast_bytes(self._ckpt_tag.encode() if comm.rank == 0 else None).decode()
        self.global_iteration = 0
        self.history: list[RoundRecord] = []
        self._spes = [d.steps_per_epoch for d in tds]
        self._spe = self._spes[0]
        dev = comm.device
        self._ev0 = torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else None
        self._ev1 = torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else None
        self._log = tracing.JsonlLog(cfg.jsonl_log if comm.rank == 0 else None)
        self.he = self.he_dev = None
        self._he_ct = None
        self.last_he_stats: dict = {}
        if cfg.secure_aggregation:
            self._setup_he()
        self._ce = None  # DeferredCommunityEval, built at the first deferred evaluation
        if broadcast_initial:
            self.broadcast_initial_model()

    @property
    def steps_done(self) -> int:
        """Local updates run so far by this rank's first learner."""
        return self.steps_done_l[0]

    @steps_done.setter
    def steps_done(self, v: int) -> None:
        self.steps_done_l[0] = int(v)

    def local_learners(self) -> list[int]:
        """Global indices of this rank's learners."""
        return [self.offsets[self.rank] + j for j in range(self.L)]

    def _gather_learner_rows(self, rows: list[list[float]]) -> np.ndarray:
        """Every rank's per-learner rows (equal width), in global learner
        order -> [n_learners, width] (host).  Ranks may host different
        numbers of learners: rows are padded to the largest count for the
        all-gather."""
        width = len(rows[0])
        buf = torch.full((self.Lmax, width), float("nan"), dtype=torch.float64)
        buf[: len(rows)] = torch.tensor(rows, dtype=torch.float64)
        got = self.comm.all_gather_rows(buf.reshape(-1).to(self.comm.device)).cpu().numpy()
        got = got.reshape(self.world, self.Lmax, width)
        return np.concatenate([got[r, : self.Ls[r]] for r in range(self.world)], axis=0)

    # ------------------------------------------------------------------------
    def broadcast_initial_model(self) -> None:
        """ReplaceCommunityModel equivalent: rank 0's model becomes everyone's."""
        st = self.net.state
        self.comm.broadcast_(st.model32, src=0)
        self._install_local(st.model32)

    def _install_local(self, src: torch.Tensor) -> None:
        if self.group is not None:
            self.group.install(src)
        else:
            self.net.state.refresh_bf16()
            self.net.state.set_anchor()

    def _sync(self):
        """Wait for the current stream (every learner stream the round joined
        into it; not a dropped learner's chunks still in flight on its own
        stream, models/colocated.py ``pending``)."""
        if self.comm.device.type == "cuda":
            torch.cuda.current_stream(self.comm.device).synchronize()

    @property
    def elastic(self) -> bool:
        """Straggler drop active (participation ratio < 1 or a round deadline)
        in a federation of more than one learner (co-located or not)."""
        return self.n_learners > 1 and (self.cfg.participation_ratio < 1.0 or self.cfg.round_deadline_s is not None)

    def quorum(self) -> int:
        """Learners (global, co-located ones counted one by one) whose
        completion ends the round."""
        n = self.n_learners
        return max(1, min(n, math.ceil(self.cfg.participation_ratio * n - 1e-9)))

    def _store(self):
        import torch.distributed as dist
        return dist.distributed_c10d._get_default_store()

    def _slow_s(self, g: int) -> float:
        """Test hook ``extra.debug_slow_s``: {global learner index: seconds of
        host delay after each chunk} (with one learner per rank: the rank)."""
        return float(self.cfg.extra.get("debug_slow_s", {}).get(str(g), 0.0))

    def _train_elastic_group(self, nsteps: list[int], t0: float) -> tuple[list, list, list]:
        """Straggler drop for this rank's co-located learners: each learner's
        completion counts toward the round's quorum (the process group's
        store key, shared with one-learner ranks; a local counter in a
        one-process federation); once the quorum has finished or the deadline
        passed, learners still training stop issuing updates and sit the
        round out -> (ms, updates run, participated) per local learner."""
        q, deadline = self.quorum(), self.cfg.round_deadline_s
        if self.comm.distributed:
            store, key = self._store(), f"metisfl/round{self.global_iteration}/done"

            def on_finish(j):
                store.add(key, 1)

            def count():
                return int(store.add(key, 0))
        else:
            self._local_done = 0

            def on_finish(j):
                self._local_done += 1

            def count():
                return self._local_done

        def stop():
            return count() >= q or (deadline is not None and time.perf_counter() - t0 > deadline)

        slow = [self._slow_s(g) for g in self.local_learners()]
        return self.group.train_elastic(list(nsteps), list(self.steps_done_l), stop, on_finish,
                                        poll_steps=max(1, self.cfg.poll_steps), slow_s=slow)

    def _train_elastic(self, nsteps: int, t0: float) -> tuple[int, bool]:
        """Chunked local training that stops early once the round's quorum
        has finished or the deadline passed -> (steps run, participated)."""
        store, key = self._store(), f"metisfl/round{self.global_iteration}/done"
        q = self.quorum()
        deadline = self.cfg.round_deadline_s
        slow = self._slow_s(self.offsets[self.rank])
        done = 0
        while done < nsteps:
            k = min(self.cfg.poll_steps, nsteps - done)
            self.net.train_steps(self.train_ds, k, step_offset=self.steps_done + done)
            self._sync()
            if slow:
                time.sleep(slow)  # test hook: a deliberately slow learner
            done += k
            if done >= nsteps:
                break
            if int(store.add(key, 0)) >= q or (deadline is not None and time.perf_counter() - t0 > deadline):
                return done, False  # dropped from this round
        store.add(key, 1)
        return done, True

    def local_train_all(self, nsteps: list[int]) -> list[dict]:
        """Local training of every learner of this rank (concurrently on
        their own streams when co-located) -> one result dict per learner."""
        if self.L == 1:
            return [self.local_train(nsteps[0])]
        self.group.reset_train_stats()
        part = [True] * self.L
        tests = None
        with tracing.range("metisfl.local_train"):
            if self.elastic:
                ms, nsteps, part = self._train_elastic_group(nsteps, time.perf_counter())
            elif self.cfg.evaluate_test:
                # each learner's test evaluation right behind its own last update
                ms, tests = self.group.train(list(nsteps), list(self.steps_done_l), eval_dss=self.test_dss,
                                             eval_max_steps=self.cfg.eval_max_steps)
            else:
                ms = self.group.train(list(nsteps), list(self.steps_done_l))
        out = []
        for j, (net, ran) in enumerate(zip(self.nets, nsteps)):
            self.steps_done_l[j] += ran
            # a dropped learner's statistics are still being accumulated on
            # its stream: it completed no task this round (no train metrics)
            tr = net.train_stats() if j not in self.group.pending else {"loss": float("nan"),
                                                                        "accuracy": float("nan")}
            spe = self._spes[j]
            out.append({"ms": ms[j], "ms_per_batch": ms[j] / max(1, ran), "ms_per_epoch": ms[j] / max(1, ran) * spe,
                        "completed_batches": ran, "completed_epochs": ran / spe,
                        "train_loss": tr["loss"], "train_accuracy": tr["accuracy"], "participated": bool(part[j])})
        if self.cfg.evaluate_test:
            if tests is None:
                with tracing.range("metisfl.evaluate"):
                    tests = self.group.evaluate(max_steps=self.cfg.eval_max_steps)
            for o, t in zip(out, tests):
                if t is not None:
                    o["test"] = t
        return out

    def local_train(self, nsteps: int) -> dict:
        net = self.net
        net.reset_train_stats()
        t0 = time.perf_counter()
        participated = True
        ran = nsteps
        with tracing.range("metisfl.local_train"):
            if self._ev0 is not None:
                self._ev0.record()
            if self.elastic:
                ran, participated = self._train_elastic(nsteps, t0)
            else:
                net.train_steps(self.train_ds, nsteps, step_offset=self.steps_done)
            if self._ev1 is not None:
                self._ev1.record()
                self._ev1.synchronize()
                ms = self._ev0.elapsed_time(self._ev1)
            else:
                ms = (time.perf_counter() - t0) * 1e3
        self.steps_done += ran
        tr = net.train_stats()
        out = {"ms": ms, "ms_per_batch": ms / max(1, ran),
               "ms_per_epoch": ms / max(1, ran) * self._spe,
               "completed_batches": ran, "completed_epochs": ran / self._spe,
               "train_loss": tr["loss"], "train_accuracy": tr["accuracy"],
               "participated": participated}
        if self.cfg.evaluate_test and self.test_ds is not None:
            with tracing.range("metisfl.evaluate"):
                out["test"] = net.evaluate(self.test_ds, self.cfg.eval_max_steps)
        return out

    def aggregation_weights(self, meta: np.ndarray) -> list[float]:
        part = meta[:, 10] > 0.5
        if not part.any():
            # every learner hit the deadline before finishing its budget: the
            # ones that ran the most local updates stand in as participants
            # (an all-zero weight vector would zero the community model)
            part = meta[:, 1] >= meta[:, 1].max()
        if not part.all():  # stragglers dropped: scale over the participants only
            idx = np.flatnonzero(part)
            ws = scaling.compute(self.cfg.scaling_factor, meta[idx, 0], meta[idx, 1], len(idx))
            w = [0.0] * self.n_learners
            for i, x in zip(idx, ws):
                w[int(i)] = float(x)
            return w
        w = scaling.compute(self.cfg.scaling_factor, meta[:, 0], meta[:, 1], self.n_learners)
        if self.engine is not None:
            we = self.engine.weights(meta[:, 0], meta[:, 1])
            if not np.allclose(we, w, rtol=1e-12, atol=0):
                raise RuntimeError(f"scaler mismatch: engine {we} vs collective {w}")
        return w

    def _rank_weights(self, weights: list[float]) -> list[float]:
        """Per-rank PWA weights: a one-learner rank's learner weight; ranks
        hosting several learners sum them (scaled) before encrypting: 1."""
        return [float(weights[self.offsets[r]]) if self.Ls[r] == 1 else 1.0 for r in range(self.world)]

    def _setup_he(self) -> None:
        self.he, self._he_dir = setup_ckks(self.comm, self.cfg)
        if self.comm.device.type == "cuda":
            from metisfl_amd.encryption.device import DeviceCKKS
            self.he_dev = DeviceCKKS(self.he, self.comm.device)

    def _secure_aggregate(self, weights: list[float]) -> None:
        """model32 <- Dec(PWA(Enc(model32_r), w_r)): ciphertexts are what
        crosses the process boundary; plaintext weights stay on their GPU.
        ``weights``: one per rank (co-located learners were pre-summed in
        plaintext inside their own process: weight 1)."""
        st = self.net.state
        if self.he_dev is not None:
            with tracing.range("metisfl.secure_allreduce"):
                if self._he_ct is None:
                    self._he_ct = torch.empty(self.he_dev.ct_numel(st.model32.numel()),
                                              dtype=torch.int64, device=self.comm.device)
                self.last_he_stats = self.he_dev.secure_weighted_allreduce(
                    self.comm, st.model32, weights[self.rank], ct=self._he_ct)  # per-rank weights
            self.last_allreduce_ms = self.last_he_stats["allreduce_ms"]
            return
        # host path (CPU / gloo): host encrypt, all-gather ciphertexts, host PWA
        t0 = time.perf_counter()
        n = st.model32.numel()
        ct = self.he.encrypt(st.model32.double().numpy())
        t1 = time.perf_counter()
        buf = torch.frombuffer(bytearray(ct), dtype=torch.uint8)
        rows = self.comm.all_gather_rows(buf)
        t2 = time.perf_counter()
        cts = [bytes(rows[r].numpy().tobytes()) for r in range(self.world)]
        agg = self.he.compute_weighted_average(cts, [float(w) for w in weights])
        st.model32.copy_(torch.from_numpy(self.he.decrypt(agg, n)).to(st.model32.dtype))
        t3 = time.perf_counter()
        self.last_he_stats = {"encrypt_ms": (t1 - t0) * 1e3, "allreduce_ms": (t2 - t1) * 1e3,
                              "decrypt_ms": (t3 - t2) * 1e3, "ciphertext_bytes": len(ct)}
        self.last_allreduce_ms = (t2 - t1) * 1e3

    def aggregate(self, meta: np.ndarray) -> tuple[list[float], float]:
        """Scale + all-reduce; returns (weights, ms)."""
        t0 = time.perf_counter()
        weights = self.aggregation_weights(meta)
        st = self.net.state
        self.last_allreduce_ms = 0.0
        if self.L > 1:
            wl = [weights[i] for i in self.local_learners()]
            if self.cfg.secure_aggregation and self.he_dev is not None:
                self.group.settle([0])  # the output buffer is learner 0's model
                parts = [j for j, w in enumerate(wl) if w != 0.0] or list(range(self.L))
                # every co-located learner encrypts its own model; the weighted
                # ciphertexts are summed on the device, then all-reduced
                with tracing.range("metisfl.secure_allreduce"):
                    if self._he_ct is None:
                        self._he_ct = torch.empty(self.he_dev.ct_numel(st.model32.numel()),
                                                  dtype=torch.int64, device=self.comm.device)
                        self._he_tmp = torch.empty_like(self._he_ct)
                    # participants only (a dropped learner's model is never read)
                    self.last_he_stats = self.he_dev.secure_weighted_allreduce_many(
                        self.comm, [self.nets[j].state.model32 for j in parts], [wl[j] for j in parts],
                        st.model32, ct=self._he_ct, tmp=self._he_tmp)
                self.last_allreduce_ms = self.last_he_stats["allreduce_ms"]
                self._install_local(st.model32)
                self._sync()
                return weights, (time.perf_counter() - t0) * 1e3
            # hierarchical: this GPU's learners summed locally (K1), then the
            # cross-GPU reduction carries one model per GPU
            with tracing.range("metisfl.local_reduce"):
                self.group.weighted_sum_into(st.model32, wl)
            if self.cfg.secure_aggregation:
                self._secure_aggregate(self._rank_weights(weights))  # host CKKS path (CPU runs)
            elif self.world > 1:
                self._sync()
                t1 = time.perf_counter()
                with tracing.range("metisfl.all_reduce"):
                    self.comm.all_reduce_(st.model32)
                    self._sync()
                self.last_allreduce_ms = (time.perf_counter() - t1) * 1e3
            self._install_local(st.model32)
            self._sync()
            return weights, (time.perf_counter() - t0) * 1e3
        if self.cfg.secure_aggregation:
            self._secure_aggregate(self._rank_weights(weights))
        elif self.world > 1:
            with tracing.range("metisfl.scale"):
                opt_ops.scale_(st.model32, weights[self.local_learners()[0]])
            self._sync()
            t1 = time.perf_counter()
            with tracing.range("metisfl.all_reduce"):
                self.comm.all_reduce_(st.model32)
                self._sync()
            self.last_allreduce_ms = (time.perf_counter() - t1) * 1e3
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
        # called at the end of round ``global_iteration``: the end of round 1
        # sets the budgets round 2 runs with (controller.cc:527-532)
        if not (self.global_iteration == 1 or self.cfg.semi_sync_recompute):
            return
        t_max = self.cfg.semi_sync_lambda * float(meta[:, 3].max())
        self.num_local_updates = [max(1, int(math.ceil(t_max / max(1e-6, float(mpb)))))
                                  for mpb in meta[:, 2]]

    def _quantifiers(self):
        from metisfl_amd.ops.aggregate import count_zeros
        st = self.net.state
        segs = st.segments()
        zeros = count_zeros(st.model32, segs)
        lengths = [e - b for b, e in segs]
        return zeros, [n * 4 for n in lengths], lengths

    def _deferred_eval(self) -> "DeferredCommunityEval | None":
        if not self.cfg.defer_community_eval:
            return None
        if self._ce is None:  # collective decision: every rank defers, or none does
            ce = DeferredCommunityEval.build(self.nets, self.test_dss)
            ok = torch.tensor([1.0 if ce is not None else 0.0], dtype=torch.float64, device=self.comm.device)
            if self.comm.distributed:
                ok = self.comm.all_gather_rows(ok).min(0).values
            self._ce = ce if float(ok[0]) > 0.5 else False
        return self._ce or None

    def _collect_community_eval(self) -> None:
        """Collective.  Record the deferred evaluation of an earlier round
        (all-gathered over the ranks) with that round."""
        ce = self._ce or None
        got = ce.collect() if ce is not None else None  # every rank submits and collects in lockstep
        if got is None:
            return
        gi, evs = got
        out = self._community_rows(evs)
        rec = next((r for r in reversed(self.history) if r.global_iteration == gi), None)
        if rec is not None:
            rec.community_eval = out
        if self.engine is not None and out and hasattr(self.engine, "record_evaluations"):
            self.engine.record_evaluations(gi, out)

    def finish_evaluations(self) -> None:
        """Collective.  Wait for and record the pending deferred community
        evaluation (the bench calls it inside its timed region)."""
        if self._ce:
            self._collect_community_eval()

    def _community_rows(self, evs: list) -> list | None:
        nan = {"loss": float("nan"), "accuracy": float("nan")}
        vals = []
        for ev, ds in zip(evs, self.test_dss):
            ev = ev or nan
            vals.append([ev["loss"], ev["accuracy"], float(ds.n) if ds is not None and ev is not nan else 0.0])
        rows = self._gather_learner_rows(vals)
        out = [{"loss": float(r[0]), "accuracy": float(r[1]), "num_examples": int(r[2])} for r in rows]
        if all(o["num_examples"] == 0 for o in out):
            return None
        return out

    def evaluate_community(self) -> tuple[list | None, float]:
        """Every learner evaluates the community model (resident after the
        all-reduce) on its test shard; the metrics are all-gathered (a few
        scalars per learner).  -> ([{"loss", "accuracy", "num_examples"}] per
        rank, ms).  With ``defer_community_eval`` the evaluation is only
        issued here (-> (None, ms)); its results are recorded with this
        round at the next round's end or by ``finish_evaluations``."""
        if not self.cfg.evaluate_community:
            return None, 0.0
        t0 = time.perf_counter()
        ce = self._deferred_eval()
        if ce is not None:
            self._collect_community_eval()  # the previous round's (long finished)
            # (the snapshot reads learner 0's model, where the community model
            # was reduced: never a pending learner's buffer, weighted_sum_into)
            ce.submit(self.global_iteration, self.cfg.eval_max_steps)
            return None, (time.perf_counter() - t0) * 1e3
        nan = {"loss": float("nan"), "accuracy": float("nan")}
        if self.group is not None:
            with tracing.range("metisfl.community_eval"):
                evs = self.group.evaluate(max_steps=self.cfg.eval_max_steps)
        else:
            evs = [None]
            if self.test_ds is not None:
                with tracing.range("metisfl.community_eval"):
                    evs = [self.net.evaluate(self.test_ds, self.cfg.eval_max_steps)]
        vals = []
        for ev, ds in zip(evs, self.test_dss):
            ev = ev or nan
            vals.append([ev["loss"], ev["accuracy"], float(ds.n) if ds is not None and ev is not nan else 0.0])
        rows = self._gather_learner_rows(vals)
        out = [{"loss": float(r[0]), "accuracy": float(r[1]), "num_examples": int(r[2])} for r in rows]
        if all(o["num_examples"] == 0 for o in out):
            return None, (time.perf_counter() - t0) * 1e3
        return out, (time.perf_counter() - t0) * 1e3

    def run_round(self) -> RoundRecord:
        self.global_iteration += 1
        started = time.time()
        results = self.local_train_all([self.num_local_updates[i] for i in self.local_learners()])
        t_trained = time.time()
        rows = []
        for ds, res in zip(self.train_dss, results):
            test = res.get("test") or {}
            rows.append([ds.n, res["completed_batches"], res["ms_per_batch"],
                         res["ms_per_epoch"], res["train_loss"], res["train_accuracy"],
                         res["completed_epochs"], self.global_iteration,
                         test.get("loss", float("nan")), test.get("accuracy", float("nan")),
                         1.0 if res["participated"] else 0.0])
        meta = self._gather_learner_rows(rows)
        res = dict(results[0])
        res["ms"] = max(r["ms"] for r in results)
        completed = time.time()
        weights, agg_ms = self.aggregate(meta)
        agg_done = time.time()
        ar_ms = getattr(self, "last_allreduce_ms", 0.0)
        community_eval, ce_ms = self.evaluate_community()
        round_done = time.time()
        nbytes = self.net.state.model32.numel() * 4
        rec = RoundRecord(self.global_iteration, started, completed, completed, agg_done,
                          (round_done - started) * 1e3, res["ms"], agg_ms, meta, weights,
                          list(self.num_local_updates), res.get("test"), ar_ms,
                          nbytes / (ar_ms * 1e6) if ar_ms > 0 else 0.0,
                          tracing.hbm_usage(self.comm.device).get("used_bytes", 0)
                          if self.comm.device.type == "cuda" else 0)
        rec.community_eval, rec.community_eval_ms = community_eval, ce_ms
        if self.cfg.secure_aggregation:
            rec.he_stats = dict(self.last_he_stats)
        if self.rank == 0:
            self._log.write({"kind": "round", **rec.to_json(),
                             "rounds_per_s": 1e3 / rec.round_ms if rec.round_ms > 0 else 0.0})
        self.stop_requested = False
        self.regroup_requested = False
        if self.engine is not None:
            r = self.engine.record_round(rec, self.cfg.batch_size,
                                         self._quantifiers() if self.cfg.quantify else None)
            self.stop_requested = bool(r)  # the driver asked the federation to stop
            # the driver asked for a relaunch on a new membership (a learner joins)
            self.regroup_requested = bool(getattr(self.engine, "regroup_requested", False))
            if self.cfg.snapshot_every and self.global_iteration % self.cfg.snapshot_every == 0:
                rec.snapshot_ms = self.snapshot_community()
        self.update_templates(meta)
        rec.phase_ms = {"local_train": (t_trained - started) * 1e3, "gather": (completed - t_trained) * 1e3,
                        "aggregate": (agg_done - completed) * 1e3, "community_eval": (round_done - agg_done) * 1e3,
                        "bookkeeping": (time.time() - round_done) * 1e3}
        self.history.append(rec)
        return rec

    def community_metric(self, rec: RoundRecord, metric: str) -> float | None:
        """Mean over learners of a community-model test metric (the driver's
        MetricCutoffScore statistic, driver_session.py:423-467)."""
        vals = [e[metric] for e in (rec.community_eval or []) if e.get("num_examples") and metric in e]
        return float(np.mean(vals)) if vals else None

    # -- checkpoint / resume ------------------------------------------
    COMMUNITY_FILE = "community_model.pb"

    def community_model_proto(self):
        """The community model as the reference's wire message
        ``metisfl.FederatedModel`` (model.proto:48-52): one Variable per
        tensor, in FlatState order, plaintext fp32."""
        from metisfl_amd.proto import model_pb2
        from metisfl_amd.utils.tensor_codec import model_from_arrays
        st = self.net.state
        vals = st.to_numpy()
        names = [s.name for s in st.specs]
        fm = model_pb2.FederatedModel()
        fm.num_contributors = self.n_learners
        fm.global_iteration = self.global_iteration
        fm.model.CopyFrom(model_from_arrays(names, [vals[n] for n in names], [s.trainable for s in st.specs]))
        return fm

    def _community_proto_from(self, flat: np.ndarray, gi: int):
        """``FederatedModel`` of a host copy of the flat community model of
        round ``gi``."""
        from metisfl_amd.proto import model_pb2
        from metisfl_amd.utils.tensor_codec import model_from_arrays
        st = self.net.state
        fm = model_pb2.FederatedModel()
        fm.num_contributors = self.n_learners
        fm.global_iteration = gi
        fm.model.CopyFrom(model_from_arrays([s.name for s in st.specs],
                                            [flat[s.offset: s.offset + s.numel].reshape(s.shape) for s in st.specs],
                                            [s.trainable for s in st.specs]))
        return fm

    def _federation_json(self) -> dict:
        st = self.net.state
        return {"global_iteration": self.global_iteration, "protocol": self.cfg.protocol,
                "num_local_updates": list(self.num_local_updates),
                "world": self.world, "learners_per_rank": list(self.Ls), "learner_ids": self.learner_ids,
                "dataset_sizes": self.dataset_sizes,
                "config": {k: v for k, v in asdict(self.cfg).items() if k != "extra"},
                "variables": [[s.name, list(s.shape), s.trainable] for s in st.specs],
                "history": [r.to_json() for r in self.history]}

    def save_checkpoint(self, path: str, block: bool = True, keep: int = 2) -> float:
        """Collective.  Checkpoint ``path/round_<gi>/``: rank 0 writes the
        community model as a serialized ``FederatedModel`` proto (the layout
        the gRPC controller exchanges: ``ReplaceCommunityModel`` /
        ``GetCommunityModelLineage`` carry the same message) plus
        federation.json; every rank writes its learners' local optimizer
        state (safetensors layout).  Both writers are native and run with
        the GIL released (checkpoint.save_tensors / write_federated_model);
        ``path/LATEST`` moves to it once every rank's files are written
        (parallel/checkpoint.py).  ``block=False``: the tensors are snapshot
        device-to-device now and written by a background thread while the
        next round runs.  -> milliseconds the call held this rank."""
        from metisfl_amd.parallel import checkpoint as ck
        t_prep = time.perf_counter()
        if self.group is not None:
            self.group.settle()  # dropped learners' optimizer state is final once their chunks land
        if self._ckpt is None:
            self._ckpt = ck.AsyncSnapshot(self.comm.device, "metisfl-checkpoint")
        gi = self.global_iteration
        name = f"round_{gi}"
        d = os.path.join(path, name)
        # one file per learner, keyed by its (stable) learner id, so a relaunch
        # may pack the learners onto processes differently (a lost GPU, a
        # joining learner, learners sharing a device)
        tensors, host = {}, {}
        for j, (net, ds) in enumerate(zip(self.nets, self.train_dss)):
            pre = f"{j}/"
            lst = net.state
            tensors[pre + "step"] = lst.step
            tensors[pre + "perm"] = ds.perm
            host[pre + "steps_done"] = torch.tensor(self.steps_done_l[j])
            for k in ("m", "v", "anchor"):
                t = getattr(lst, k)
                if t is not None:
                    tensors[pre + k] = t
        my_ids = [self.learner_ids[i] for i in self.local_learners()]
        if self.rank == 0:
            tensors["@community"] = self.net.state.model32
            fed_json = self._federation_json()
        store = self._store() if self.comm.distributed else None
        key = f"metisfl_ckpt/{self._ckpt_tag}/{gi}"
        rank, world = self.rank, self.world
        specs, n_learners = self.net.state.specs, self.n_learners

        def write(h):
            os.makedirs(d, exist_ok=True)
            for j, lid in enumerate(my_ids):
                pre = f"{j}/"
                per = {k[len(pre):]: v for k, v in host.items() if k.startswith(pre)}
                per.update({k[len(pre):]: v for k, v in h.items() if k.startswith(pre)})
                ck.save_tensors(per, os.path.join(d, learner_file(lid)))
            if store is not None:
                store.set(f"{key}/{rank}", "1")
            if rank == 0:
                ck.write_federated_model(os.path.join(d, self.COMMUNITY_FILE), h["@community"].numpy(), specs,
                                         n_learners, gi)
                ck.atomic_write(os.path.join(d, "federation.json"), json.dumps(fed_json).encode())
                ck.publish(path, name, store, world, key, keep)

        os.makedirs(path, exist_ok=True)
        self.last_checkpoint_prep_ms = (time.perf_counter() - t_prep) * 1e3
        ms = self._ckpt.submit(tensors, write) + self.last_checkpoint_prep_ms
        if block:
            self._ckpt.wait()
            self.comm.barrier()
        return ms

    def flush_checkpoints(self) -> None:
        """Wait for background checkpoint / lineage writes of this rank (and
        send the last community model if the lineage skipped its round).
        Not collective: a deferred community evaluation still pending is
        collected by ``finish_evaluations``."""
        if self._lineage is not None and getattr(self, "_lineage_skipped", False):
            self._lineage.wait()
            self.snapshot_community()
        for w in (self._ckpt, self._lineage):
            if w is not None:
                w.wait()

    def snapshot_community(self) -> float:
        """Rank 0 with a controller bridge: hand the community model to the
        controller's lineage (``ReplaceCommunityModel``; the reference
        replaces its community model every global iteration,
        controller.cc:466), staged now and sent from a background thread.
        Latest wins: while the controller is still receiving an earlier
        round's model the round is not staged (the caller never waits on the
        controller); ``flush_checkpoints`` sends the final model if its round
        was skipped.  -> milliseconds on the caller's path."""
        if self.engine is None or not hasattr(self.engine, "snapshot_community"):
            return 0.0
        from metisfl_amd.parallel import checkpoint as ck
        if self._lineage is None:
            self._lineage = ck.AsyncSnapshot(self.comm.device, "metisfl-lineage")
        st = self.net.state
        gi, engine = self.global_iteration, self.engine

        def write(h):
            flat = h["model"].numpy()
            engine.snapshot_community([s.name for s in st.specs],
                                      [flat[s.offset: s.offset + s.numel].reshape(s.shape) for s in st.specs],
                                      [s.trainable for s in st.specs], gi)

        ms = self._lineage.try_submit({"model": st.model32}, write)
        self._lineage_skipped = ms is None
        if ms is None:
            self.lineage_skipped_rounds = getattr(self, "lineage_skipped_rounds", 0) + 1
            return 0.0
        return ms

    def load_community_model(self, fm) -> None:
        """Install a ``FederatedModel`` (proto or serialized bytes) as the
        community model, matching variables by name."""
        install_community_model(self.net, fm, self.he)
        if self.group is not None:
            self._install_local(self.net.state.model32)

    def resume(self, path: str, prev_rank: int | None = None) -> None:
        """Reload a checkpoint written by ``save_checkpoint``.  The world size
        may differ (learners joined or left, SURVEY §5.3 / the reference's
        join-leave semantics, controller.cc:99-199): the community model is
        restored on every rank, learner-local state (optimizer slots, step
        counter, epoch permutation) for every learner the checkpoint has a
        file for (by learner id, whatever rank or co-located slot it has
        now; learners that joined since start fresh), and the step budgets /
        aggregation weights follow the CURRENT shards (computed at
        construction from the new dataset sizes).  ``prev_rank``: for
        checkpoints of the rounds-1..3 layout (one file per rank), this
        learner's rank in the checkpointed federation."""
        from metisfl_amd.parallel import checkpoint as ck
        found = ck.resolve(path)
        if found is None:
            raise FileNotFoundError(f"no complete checkpoint under {path}")
        path = found
        with open(os.path.join(path, "federation.json")) as f:
            meta = json.load(f)
        pb = os.path.join(path, self.COMMUNITY_FILE)
        legacy = os.path.join(path, "community.pt")
        if os.path.exists(pb):
            with open(pb, "rb") as f:
                self.load_community_model(f.read())
        elif os.path.exists(legacy):
            # round-1 checkpoint layout: the flat fp32 community model as a
            # plain tensor (loaded without unpickling code)
            flat = torch.load(legacy, weights_only=True)
            st = self.net.state
            if flat.numel() != st.model32.numel():
                raise RuntimeError(f"old-format checkpoint {legacy}: {flat.numel()} values, model has "
                                   f"{st.model32.numel()}")
            st.model32.copy_(flat.to(st.model32.device, st.model32.dtype).view_as(st.model32))
            self._install_local(st.model32)
        else:
            raise FileNotFoundError(f"no community model in checkpoint {path} ({self.COMMUNITY_FILE})")
        lpr = meta.get("learners_per_rank", 1)  # a list per rank; one int in round-4 checkpoints
        old_ls = [int(x) for x in lpr] if isinstance(lpr, list) else [int(lpr)] * int(meta["world"])
        same_world = meta["world"] == self.world and old_ls == list(self.Ls)
        old_ids = list(meta.get("learner_ids", []))
        for j, (net, ds) in enumerate(zip(self.nets, self.train_dss)):
            lid = self.learner_ids[self.local_learners()[j]]
            f = os.path.join(path, learner_file(lid))
            f_pt = f[: -len(".safetensors")] + ".pt"  # round-4 interim layout (torch.save)
            if os.path.exists(f):
                per = ck.load_tensors(f)
            elif os.path.exists(f_pt):
                per = torch.load(f_pt, weights_only=True)
            else:
                continue  # a learner that joined after the checkpoint: fresh optimizer state
            st = net.state
            dev = st.model32.device
            st.step.copy_(per["step"].to(dev))
            for k in ("m", "v"):
                t = per.get(k)
                if t is not None and getattr(st, k) is not None and t.numel() == getattr(st, k).numel():
                    getattr(st, k).copy_(t.to(dev))
            # the epoch order continues only on an unchanged shard (same
            # learner, same dataset size -> same steps per epoch)
            if lid in old_ids and per["perm"].numel() == ds.perm.numel():
                ds.perm.copy_(per["perm"].to(ds.perm.device))
                self.steps_done_l[j] = int(per["steps_done"])
        old_rank = self.rank if prev_rank is None else int(prev_rank)
        rank_file = os.path.join(path, f"rank{old_rank}.pt")  # round-1..3 layout: one file per rank
        if os.path.exists(rank_file) and 0 <= old_rank < meta["world"]:
            per_rank = torch.load(rank_file, weights_only=True)
            for j, (net, ds) in enumerate(zip(self.nets, self.train_dss)):
                pre = "" if j == 0 else f"l{j}/"
                if pre + "step" not in per_rank:
                    continue  # more co-located learners now than in the checkpoint
                st = net.state
                dev = st.model32.device
                st.step.copy_(per_rank[pre + "step"].to(dev))
                for k in ("m", "v"):
                    t = per_rank.get(pre + k)
                    if t is not None and getattr(st, k) is not None and t.numel() == getattr(st, k).numel():
                        getattr(st, k).copy_(t.to(dev))
                if same_world and old_rank == self.rank and per_rank[pre + "perm"].numel() == ds.perm.numel():
                    ds.perm.copy_(per_rank[pre + "perm"].to(ds.perm.device))
                    self.steps_done_l[j] = int(per_rank[pre + "steps_done"])
        for net in self.nets:
            net.state.set_anchor()  # FedProx anchors at the restored community model
        self.global_iteration = int(meta["global_iteration"])
        if same_world:
            self.num_local_updates = list(meta["num_local_updates"])
        self.resumed_from_world = int(meta["world"])
        self.resumed_from_learners = len(meta.get("learner_ids") or []) or self.resumed_from_world
