"""Co-located learners: several federation learners resident on ONE GPU.

The reference places learners on GPUs round-robin and lets several share a
device (its CIFAR-10 experiment runs 10 learners on 5 GPUs,
examples/config/cifar10/test_localhost_synchronous_momentumsgd.yaml:4-27;
driver_session.py:558-562 pins each learner process with
CUDA_VISIBLE_DEVICES).  There every learner is its own process with its own
framework runtime, and learners on one GPU time-share it.

Here the learners of one GPU live in ONE process, each with its own model,
optimizer state, workspace, data shard and captured step graphs, and each
replays its graphs on its own HIP stream.  A ResNet-18 update at batch 32 is
latency-bound on MI355X (~64 launches of 256-576 workgroups on 256 CUs, one
workgroup per CU for the halo convs: profiles/ANALYSIS.md), so one learner
leaves most of the chip idle between and inside launches; streams let the
hardware queues run up to four learners' kernels side by side
(GPU_MAX_HW_QUEUES=4, the HIP default: measured 0.70 ms per update with 4-8
learners against 1.04 ms for one, profiles/r4/colocated/).

The round's FedAvg over co-located learners is a local weighted sum (K1,
one launch over all of them) followed by the cross-GPU all-reduce
(parallel/federation.py), i.e. a hierarchical reduce: xGMI only ever carries
one model per GPU.
"""
from __future__ import annotations

import os

import torch


def configure_regime(learners_per_gpu: int) -> None:
    """Kernel choices for ``learners_per_gpu`` learners sharing each GPU, made
    BEFORE their models are built (the layer plans and workspaces are fixed
    at build): with 2+ co-located learners the 4x4x512 layers run the im2col
    convolution instead of the halo conv (8-slice split-K at one workgroup
    per CU: 0.6684 -> 0.6634 and 0.6823 -> 0.6737 ms per update with 8
    learners on two boxes, profiles/r6/bench/hconv_skip*.log; the one-learner
    latency regime keeps it), plus the paired-launch ring and plans that
    ``CoLocatedLearners`` also sets.  MFL_HCONV_SKIP in the environment wins."""
    from metisfl_amd.models import layers
    if learners_per_gpu >= CoLocatedLearners.pair_ring_min_learners and "MFL_HCONV_SKIP" not in os.environ:
        layers.HCONV_SKIP = {int(v) for v in CoLocatedLearners.hconv_skip.split(",") if v.strip()}
    CoLocatedLearners.apply_kernel_regime(learners_per_gpu)


class CoLocatedLearners:
    """L learners on one device; ``nets[j]`` trains ``train_dss[j]``."""

    def __init__(self, nets: list, train_dss: list, test_dss: list | None = None):
        assert len(nets) == len(train_dss) and nets
        self.nets = list(nets)
        self.train_dss = list(train_dss)
        self.test_dss = list(test_dss) if test_dss is not None else [None] * len(nets)
        dev = self.nets[0].device
        self.device = dev
        self.cuda = dev.type == "cuda"
        self.streams = (self._make_streams(dev, len(self.nets)) if self.cuda else [None] * len(nets))
        if self.cuda:
            self.apply_kernel_regime(len(self.nets))
        self._ev = ([(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                     for _ in self.nets] if self.cuda else None)
        self._ev2 = [torch.cuda.Event(enable_timing=True) for _ in self.nets] if self.cuda else None
        self.last_eval_ms: list[float] = []   # device ms of each learner's test evaluation (train(eval_dss=...))
        self.last_span_ms = 0.0               # first start -> last evaluation end
        self.last_host_ms: dict = {}          # host-side phases of the last train() call
        self.last_ms: list[float] = []        # per learner: start -> last update (train())
        # learners dropped from the last elastic round whose already-issued
        # chunks may still be running on their streams: the round closed
        # without waiting for them, so the current stream is NOT ordered after
        # their streams (``settle`` orders it)
        self.pending: set[int] = set()

    # MFL_COLOC_CUMASK=contig|interleave: confine learner j's stream to its
    # share of the CUs (hipExtStreamCreateWithCUMask) instead of letting every
    # learner's kernels spread over the whole chip (A/B knob, off by default)
    cu_mask = os.environ.get("MFL_COLOC_CUMASK", "")

    # In the throughput regime the fp32 paired conv launches run a 2-stage LDS
    # ring (32 KiB: 4 workgroups per CU instead of 3; conv32.hip
    # set_conv32_pair_ring).  Process-wide, set before the learners capture
    # their graphs.  MFL_COLOC_PAIR_RING=0 keeps the build default.
    pair_ring = os.environ.get("MFL_COLOC_PAIR_RING", "2")
    # from 2 learners on (the bench's N = 4 point: 0.8006 -> 0.7965 ms per
    # update, 3 alternating repeats, profiles/r6/bench/two_learner_regime_ab.log)
    pair_ring_min_learners = int(os.environ.get("MFL_COLOC_PAIR_RING_MIN", "2"))
    # ... and the input gradients split their reduction into fewer slices
    # than the one-learner table (fewer, fuller workgroups when other
    # learners' launches fill the CUs): the 16x16x128 / 8x8x256 3x3 ones 1 / 2
    # instead of 2 / 4, the stride-2 16x16x128->256 / 8x8x256->512 3x3 ones
    # 1 / 2 instead of 3 / 4, the 8x8x256->512 1x1 shortcut's 1 instead of 2.
    # 8 co-located learners 0.6678 -> 0.6607 -> 0.6534 ms per update in two
    # sweeps (one learner 1.074 -> 1.086: so only here), same box, 3
    # alternating repeats (profiles/r6/bench/plan_sweep*, plan_confirm*.log).
    # Plans only shrink: the workspaces sized at model build still fit.
    # MFL_COLOC_PLANS="" keeps the table; MFL_C32_PLANS overrides both.
    plans = os.environ.get("MFL_COLOC_PLANS", "1,16,128,128,3,1,1;1,8,256,256,3,1,2;1,16,128,256,3,2,1;"
                                              "1,8,256,512,3,2,2;1,8,256,512,1,2,1")

    hconv_skip = os.environ.get("MFL_COLOC_HCONV_SKIP", "4")  # see configure_regime
    # bf16 option: the forward / dgrad and weight-gradient plans aim at 128
    # split-K workgroups instead of 256 / 512 with 4+ co-located learners
    # (4 / 8 learners 0.469 / 0.466 -> 0.431 / 0.428 ms per update, 2 learners
    # neutral, same box, 2 alternating repeats, profiles/r6/s2/bf16_*.log;
    # one learner keeps the defaults).  "" keeps the defaults.
    bf16_targets = os.environ.get("MFL_COLOC_BF16_TARGETS", "128,128")
    # BERT: the grouped weight gradients split 2 ways instead of 3 / 7 with 4+
    # co-located learners (8 learners 1.330 -> 1.341M tokens/s, 3 alternating
    # repeats, profiles/r6/s2/bert8_splits*.log).  "" / 0 keeps the plan.
    wgrad2_splits = int(os.environ.get("MFL_COLOC_WGRAD2_SPLITS", "2") or 0)
    # ... and every large-tile GEMM runs 256-wide tiles (the one-learner plan
    # picks 192 for N = 768 / 2304 to save a round of workgroups; co-located
    # launches fill the CUs anyway): 8 learners 1.336 -> 1.383M tokens/s,
    # profiles/r6/s2/bert8_width.log.  "" / 0 keeps the per-shape plan.
    gemm_width = int(os.environ.get("MFL_COLOC_GB_WIDTH", "256") or 0)
    # fp32 BatchNorm applies: 256-workgroup grid cap instead of 512 with 4+
    # learners (8 learners 5.391 -> 5.343 ms per 8-learner step; one learner
    # keeps 512), profiles/r6/s2/bn32_grid_*.log.  "" / 0 keeps the default.
    bn32_grid = int(os.environ.get("MFL_COLOC_BN32_GRID", "256") or 0)

    @classmethod
    def apply_kernel_regime(cls, n: int) -> None:
        """Process-wide launch choices for n co-located learners (before their
        graphs are captured): the 2-stage pair ring and the plan overrides."""
        import torch as _t
        if n < cls.pair_ring_min_learners or not _t.cuda.is_available():
            return
        if cls.pair_ring:
            cls._set_pair_ring(int(cls.pair_ring))
        if cls.plans:
            from metisfl_amd.ops._native import ops
            ops().set_conv32_plan_overrides(cls.plans)
        if cls.bf16_targets and n >= 4:  # 2 learners: neutral (0.5765 / 0.5770 ms)
            from metisfl_amd.ops._native import ops
            ct, wt = (int(v) for v in cls.bf16_targets.split(","))
            ops().set_conv_plan_targets(ct, wt)
        if cls.wgrad2_splits and n >= 4:
            from metisfl_amd.ops._native import ops
            ops().set_gemm_wgrad2_splits(cls.wgrad2_splits)
        if cls.gemm_width and n >= 4:
            from metisfl_amd.ops._native import ops
            ops().set_gemm_width(cls.gemm_width)
        if cls.bn32_grid and n >= 4:
            from metisfl_amd.ops._native import ops
            ops().set_bn32_grid_cap(cls.bn32_grid)

    @staticmethod
    def _set_pair_ring(ns: int) -> None:
        from metisfl_amd.ops._native import ops
        ops().set_conv32_pair_ring(ns)

    @classmethod
    def _make_streams(cls, dev, n: int) -> list:
        if not cls.cu_mask or n < 2:
            return [torch.cuda.Stream(device=dev) for _ in range(n)]
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        per = max(1, ncu // n)
        out = []
        with torch.cuda.device(dev):
            for g in range(n):
                bits = [0] * ((ncu + 31) // 32)
                for cu in range(ncu):
                    if (cu // per == g) if cls.cu_mask == "contig" else (cu % n == g):
                        bits[cu // 32] |= 1 << (cu % 32)
                arr = (ctypes.c_uint32 * len(bits))(*bits)
                h = ctypes.c_void_p()
                if hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(bits)), arr) != 0:
                    raise RuntimeError("hipExtStreamCreateWithCUMask failed")
                out.append(torch.cuda.ExternalStream(h.value, device=dev))
        return out

    def __len__(self) -> int:
        return len(self.nets)

    def _ctx(self, j: int):
        import contextlib
        return torch.cuda.stream(self.streams[j]) if self.cuda else contextlib.nullcontext()

    def _fork(self) -> None:
        """Every learner stream waits for the work already issued on the
        current stream (e.g. the aggregation that wrote the models)."""
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            for s in self.streams:
                s.wait_stream(cur)

    def _join(self, only=None) -> None:
        """The current stream waits for the learners' streams (``only``: those
        learners)."""
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            for j, s in enumerate(self.streams):
                if only is None or j in only:
                    cur.wait_stream(s)

    def settle(self, only=None) -> None:
        """Order the current stream after the pending (dropped) learners'
        streams -- before anything on it reads or writes their buffers (their
        optimizer state for a checkpoint, their models for a test)."""
        js = set(self.pending) if only is None else set(only) & self.pending
        if js:
            self._join(js)
            self.pending -= js

    def active(self) -> list[int]:
        return [j for j in range(len(self)) if j not in self.pending]

    def train(self, nsteps: list[int], step_offsets: list[int], eval_dss: list | None = None,
              eval_max_steps: int | None = None):
        """Run ``nsteps[j]`` local updates of every learner concurrently ->
        per-learner milliseconds from the common start to that learner's last
        update (its wall-clock share of the co-located run).

        ``eval_dss``: each learner then evaluates its model on ``eval_dss[j]``
        (the reference learner's test evaluation at task end,
        keras_model_ops.py:174-176), issued on its stream right behind its
        last update -- an early finisher's evaluation overlaps the others'
        training -> (ms, [metrics or None per learner])."""
        import time
        th = [time.perf_counter()]
        lead = None
        if self.cuda:  # how long the device is still busy with earlier work when this call starts
            lead = torch.cuda.Event(enable_timing=True)
            lead.record()
        # capture before the streams run concurrently (a capture synchronises
        # the device)
        for net, ds, n in zip(self.nets, self.train_dss, nsteps):
            net.prepare_graphs(ds, n)
        self._fork()
        t0 = time.perf_counter()
        th.append(t0)
        if self.cuda:
            for j in range(len(self)):
                with self._ctx(j):
                    self._ev[j][0].record()
        gens = [net.train_steps_iter(ds, n, off)
                for net, ds, n, off in zip(self.nets, self.train_dss, nsteps, step_offsets)]
        live = list(range(len(gens)))
        host_ms = [0.0] * len(gens)
        owners = [None] * len(gens)
        while live:
            nxt = []
            for j in live:
                with self._ctx(j):
                    try:
                        next(gens[j])
                        nxt.append(j)
                    except StopIteration:
                        if self.cuda:
                            self._ev[j][1].record()
                        host_ms[j] = (time.perf_counter() - t0) * 1e3
                        if eval_dss is not None and eval_dss[j] is not None:
                            owners[j] = self.nets[j].begin_evaluate(eval_dss[j], eval_max_steps)
                            if self.cuda:
                                self._ev2[j].record()
            live = nxt
        th.append(time.perf_counter())
        self._join()
        self.pending = set()
        if self.cuda:
            for _, e1 in self._ev:
                e1.synchronize()
            th.append(time.perf_counter())
            ms = [e0.elapsed_time(e1) for e0, e1 in self._ev]
            if eval_dss is not None:
                # device time of each learner's test evaluation, and from the
                # first learner's start to the last evaluation's end
                ev = [j for j in range(len(self)) if owners[j] is not None]
                for j in ev:
                    self._ev2[j].synchronize()
                self.last_eval_ms = [self._ev[j][1].elapsed_time(self._ev2[j]) for j in ev]
                self.last_span_ms = max((self._ev[0][0].elapsed_time(self._ev2[j]) for j in ev), default=0.0)
        else:
            ms = host_ms
            th.append(time.perf_counter())
        res = None if eval_dss is None else \
            [n.finish_evaluate(o) if o is not None else None for n, o in zip(self.nets, owners)]
        th.append(time.perf_counter())
        self.last_ms = [round(float(x), 2) for x in ms]
        self.last_host_ms = {k: round((b - a) * 1e3, 3) for k, a, b in
                             zip(("prepare", "issue", "wait", "finish_eval"), th, th[1:])}
        if lead is not None:
            self.last_host_ms["device_lead"] = round(lead.elapsed_time(self._ev[0][0]), 3)
        return ms if eval_dss is None else (ms, res)

    def train_elastic(self, nsteps: list[int], step_offsets: list[int], stop, on_finish, poll_steps: int = 64,
                      slow_s: list[float] | None = None, poll_s: float = 0.005):
        """``train`` with straggler drop: every learner runs its budget in
        chunks of ``poll_steps`` updates, at most two chunks in flight on its
        stream.  A learner whose last chunk has completed on the device calls
        ``on_finish(j)`` (the round's quorum counter).  Once ``stop()`` is
        true (quorum reached / deadline passed; polled at most every
        ``poll_s`` seconds) no further chunk is issued: learners with updates
        still unissued are dropped from the round, those whose whole budget
        is already on the device complete and participate.  ``slow_s[j]``:
        test hook, learner j waits that long after each of its chunks
        completes (a deliberately slow learner, without stalling the others).
        -> (ms per learner, updates run per learner, participated per learner)."""
        import time
        n = len(self)
        for net, ds, k in zip(self.nets, self.train_dss, nsteps):
            net.prepare_graphs(ds, k)
        self._fork()
        t0 = time.perf_counter()
        if self.cuda:
            for j in range(n):
                with self._ctx(j):
                    self._ev[j][0].record()
        gens = [net.train_steps_iter(ds, k, off)
                for net, ds, k, off in zip(self.nets, self.train_dss, nsteps, step_offsets)]
        slow = list(slow_s) if slow_s is not None else [0.0] * n
        issued = [0] * n
        inflight = [[] for _ in range(n)]      # (event or None, updates issued through it)
        ready_at = [0.0] * n                   # slow hook: no chunk before this host time
        finished = [False] * n
        ms = [0.0] * n
        stopped = False
        last_poll = 0.0

        def issue(j: int) -> None:
            got = 0
            with self._ctx(j):
                while got < poll_steps and issued[j] + got < nsteps[j]:
                    got += next(gens[j])  # one replay: K updates (may overshoot the chunk)
                issued[j] += got
                ev = None
                if self.cuda:
                    ev = torch.cuda.Event()
                    ev.record()
                    if issued[j] >= nsteps[j]:
                        # the end marker goes in right behind the last chunk:
                        # recorded later (at finish), it would queue behind
                        # whatever a co-located straggler issued meanwhile on
                        # a shared hardware queue (4 per process), and the
                        # round would wait for the straggler through it
                        self._ev[j][1].record()
                inflight[j].append((ev, issued[j]))

        def finish(j: int) -> None:
            finished[j] = True
            if self.cuda and issued[j] == 0:  # an empty budget: no chunk carried the end marker
                with self._ctx(j):
                    self._ev[j][1].record()
            ms[j] = (time.perf_counter() - t0) * 1e3
            on_finish(j)

        while True:
            now = time.perf_counter()
            busy = progressed = False
            for j in range(n):
                if finished[j]:
                    continue
                # retire completed chunks
                while inflight[j] and (inflight[j][0][0] is None or inflight[j][0][0].query()):
                    inflight[j].pop(0)
                    progressed = True
                    if slow[j]:
                        ready_at[j] = time.perf_counter() + slow[j]
                if issued[j] >= nsteps[j] and not inflight[j]:
                    finish(j)
                    continue
                busy = True
                if not stopped and issued[j] < nsteps[j] and len(inflight[j]) < 2 and now >= ready_at[j]:
                    issue(j)
                    progressed = True
            if not busy:
                break
            if not stopped and now - last_poll >= poll_s:
                last_poll = now
                stopped = bool(stop())
            if stopped and all(finished[j] or issued[j] < nsteps[j] for j in range(n)):
                break  # only dropped learners left
            if not progressed:
                time.sleep(2e-4)
        # the round closes on its participants: the current stream joins
        # only their streams; a dropped learner's chunks already on the
        # device keep running on its own stream (``pending``), and nothing
        # of this round waits for them -- the aggregation reads participants
        # only, ``install`` orders the dropped learner's copy of the
        # community model after its own chunks, the evaluations skip it
        # (the deadline is a deadline)
        done = [j for j in range(n) if finished[j]]
        if self.cuda:  # on the end markers (not a fresh marker behind a straggler's chunks)
            cur = torch.cuda.current_stream(self.device)
            for j in done:
                cur.wait_event(self._ev[j][1])
        self.pending = set(range(n)) - set(done)
        ran = list(issued)
        if not self.cuda:
            self.pending = set()
            return ms, ran, finished
        for j in done:
            self._ev[j][1].synchronize()
        out = []
        for j, (e0, e1) in enumerate(self._ev):
            out.append(e0.elapsed_time(e1) if finished[j] else (time.perf_counter() - t0) * 1e3)
        return out, ran, finished

    def evaluate(self, dss: list | None = None, max_steps: int | None = None) -> list[dict | None]:
        """Every learner evaluates its current model on its dataset (default:
        its test shard), concurrently; None where a learner has no dataset."""
        dss = self.test_dss if dss is None else dss
        self._fork()
        owners = []
        for j, (net, ds) in enumerate(zip(self.nets, dss)):
            if ds is None or j in self.pending:  # a dropped learner still busy: not evaluated
                owners.append(None)
                continue
            with self._ctx(j):
                owners.append(net.begin_evaluate(ds, max_steps))
        self._join(set(self.active()))
        return [net.finish_evaluate(o) if o is not None else None for net, o in zip(self.nets, owners)]

    def weighted_sum_into(self, out: torch.Tensor, weights: list[float]) -> None:
        """out = sum_j (fp32)(w_j * model_j) in learner order (the reference's
        FedAvg term rounding, federated_average.cc:14-37; K1, one launch).
        ``out`` may alias learner 0's model buffer.
        Participants only: a learner of weight 0 (dropped from the round) is
        not read at all -- the reference's selector never hands a
        non-participant's model to the aggregation
        (scheduled_cardinality.h:21-29), and 0 * NaN would poison the sum.
        """
        from metisfl_amd.ops.aggregate import weighted_sum
        idx = [j for j, w in enumerate(weights) if float(w) != 0.0] or list(range(len(self)))
        for j, n in enumerate(self.nets):  # ``out`` is a still-busy learner's buffer
            if j in self.pending and n.state.model32.data_ptr() == out.data_ptr():
                self.settle([j])
        weighted_sum(out, [self.nets[j].state.model32 for j in idx], [float(weights[j]) for j in idx])

    def install(self, src: torch.Tensor) -> None:
        """Every learner's model <- ``src`` (the community model); mirrors and
        FedProx anchors follow.  A pending (dropped, still busy) learner's
        copy is issued on its own stream after the current stream's work, so
        it lands after its in-flight chunks without the caller waiting."""
        cur = torch.cuda.current_stream(self.device) if self.cuda else None
        for j, net in enumerate(self.nets):
            st = net.state
            ctx = _null()
            if j in self.pending and self.cuda:
                self.streams[j].wait_stream(cur)
                ctx = self._ctx(j)
            with ctx:
                if st.model32.data_ptr() != src.data_ptr():
                    st.model32.copy_(src)
                st.refresh_bf16()
                st.set_anchor()

    def reset_train_stats(self) -> None:
        """Zero every learner's loss / accuracy accumulators (a pending
        learner's on its own stream, after its in-flight chunks)."""
        for j, net in enumerate(self.nets):
            with self._ctx(j) if j in self.pending else _null():
                net.reset_train_stats()


def _null():
    import contextlib
    return contextlib.nullcontext()
