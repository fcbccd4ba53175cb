"""StaticNet: a learner model whose whole training step is one hipGraph.

The reference delegates the local SGD loop to ``keras.Model.fit`` with a
step-counter callback (metisfl/models/keras/keras_model_ops.py:117-197,
callbacks/step_counter.py:39-45).  Here a step is: device-side batch gather
-> forward -> fused loss/head -> backward -> ONE fused optimizer launch ->
step-counter tick, all recorded once into a HIP graph and replayed, so the
host issues one graph launch per local update and never synchronises inside
a task.  Loss / accuracy are accumulated on device and read once per task.
"""
from __future__ import annotations

import gc
import os
import time

import numpy as np
import torch

from metisfl_amd.models.flat import FlatState, VarSpec
from metisfl_amd.models.layers import Layer, OptTailScheduler, Workspace
from metisfl_amd.ops import nn as K
from metisfl_amd.ops import optim as opt_ops
from metisfl_amd.ops.optim import OptimizerSpec


class DeviceDataset:
    """A learner's shard resident in device memory (NHWC rows in the model's
    compute dtype, int32 labels) plus a per-epoch permutation buffer.  Rows
    are padded so each is a multiple of 8 elements (16-B vector gathers).

    An epoch is ceil(n / batch) steps, as in Keras ``fit`` -- the count the
    controller budgets with (epochs * ceil(n / batch), controller.cc:148-153).
    The graph has a static batch shape, so the last batch of an epoch is
    completed with the first samples of the same epoch's permutation instead
    of running short (``drop_last=True``: floor(n / batch) full batches)."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor, batch_size: int, seed: int = 0,
                 shuffle: bool = True, drop_last: bool = False, pad_tail: bool = False):
        assert x.shape[0] == y.shape[0]
        self.n = int(x.shape[0])
        # pad_tail (evaluation): ceil(n / B) batches, the last one completed
        # with a padding row (zeros, label -1) that the loss / accuracy
        # kernels skip -- every sample is evaluated exactly once, as Keras
        # ``evaluate`` does
        self.pad_tail = bool(pad_tail) and not shuffle
        if self.pad_tail:
            x = torch.cat([x, torch.zeros((1,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)])
            y = torch.cat([y.to(torch.int32), torch.full((1,), -1, dtype=torch.int32, device=y.device)])
        self.x = x.contiguous()
        self.y = y.to(torch.int32).contiguous()
        self.batch_size = batch_size
        self.steps_per_epoch = max(1, self.n // batch_size) if drop_last else max(1, -(-self.n // batch_size))
        self.shuffle = shuffle
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(seed)
        self.perm = torch.zeros(self.steps_per_epoch * batch_size, dtype=torch.int32, device=x.device)
        self.reshuffle()

    def reshuffle(self) -> None:
        need = self.steps_per_epoch * self.batch_size
        if self.shuffle:
            p = torch.randperm(self.n, generator=self.gen)
        else:
            p = torch.arange(self.n)
        if p.numel() < need and self.pad_tail:  # the padding row
            p = torch.cat([p, torch.full((need - p.numel(),), self.n, dtype=p.dtype)])
        if p.numel() < need:  # last partial batch wraps around
            p = torch.cat([p, p[: need - p.numel()]])
        p = p[:need].to(torch.int32)
        if self.perm.is_cuda:
            # from pinned memory: a pageable host-to-device copy returns only
            # once the stream has drained up to it, which stalled the host
            # (and every co-located learner it feeds) at each epoch boundary
            # until this learner's queued updates had run
            p = p.pin_memory()
        self.perm.copy_(p, non_blocking=True)

    @property
    def row_shape(self):
        return tuple(self.x.shape[1:])


class StaticNet:
    """Base class: subclasses build ``self.layers`` / ``self.head`` via
    ``build()`` and implement ``forward``/``backward``."""

    input_channels_padded: int = 8
    num_classes: int = 10
    # activation / compute dtype: bf16 (mixed precision, the default of the
    # example models) or fp32 (reference precision -- ResNet18's default)
    compute_dtype: torch.dtype = torch.bfloat16

    def __init__(self, batch_size: int, device="cpu", optimizer: OptimizerSpec | None = None,
                 seed: int = 0, shared_state: FlatState | None = None):
        self.B = batch_size
        self.device = torch.device(device)
        self.build()
        specs: list[VarSpec] = []
        for l in self.all_layers():
            specs.extend(l.specs())
        if shared_state is not None:
            # a twin of an existing model (same architecture, another batch
            # size): its layers bind to the SAME parameters / statistics
            assert sorted(v.name for v in shared_state.specs) == sorted(v.name for v in specs), "twin of another model"
            self.state = shared_state
        else:
            self.state = FlatState(specs, self.device, optimizer or OptimizerSpec(), seed=seed,
                                   compute_dtype=self.compute_dtype)
        self.ws = Workspace(self.compute_dtype)
        for l in self.all_layers():
            l.bind(self.state, self.ws, self.device)
        self.ws.allocate(self.device)
        self.post_bind()
        dev = self.device
        self.xb = torch.zeros((self.B,) + self.input_shape, dtype=self.compute_dtype, device=dev)
        self.yb = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(4, dtype=torch.float32, device=dev)
        self.eval_step_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self._train_graph = None
        self._train_graph_k = None
        self._train_graph_ds = None
        self._eval_graph = None
        self._eval_graph_ds = None
        self._eval_twins = {}      # evaluation batch -> twin model (False: the model has none)
        self._eval_views = {}      # id(source dataset) -> (source dataset, the twin's view of it)

    # -- to override ----------------------------------------------------------
    input_shape: tuple = (32, 32, 8)

    def build(self) -> None:
        raise NotImplementedError

    def post_bind(self) -> None:
        """Allocate model-level buffers once layers are bound."""

    def packed_input(self) -> torch.Tensor | None:
        """A buffer the batch gather also fills with the packed bf16x3 split of
        ``xb`` (models whose first conv reads packed operands), else None."""
        return None

    def all_layers(self) -> list[Layer]:
        raise NotImplementedError

    def forward(self, x, train: bool):
        raise NotImplementedError

    def backward(self, dlast) -> None:
        raise NotImplementedError

    def forward_to_head(self, x, train: bool):
        """The head's input (models whose last BatchNorm the head applies
        return a layers.Pending instead of a tensor)."""
        return self.forward(x, train)

    # -- step bodies ---------------------------------------------------------
    # When False (tests that inspect gradients after a step) the gradient
    # buffer is zeroed at the start of the step instead of by the optimizer.
    zero_grad_in_optimizer: bool = True

    # Models whose backward reports finished variable ranges
    # (``grads_final_from``) let later paired fp32 backward launches carry the
    # optimizer step of those ranges (layers.OptTailScheduler, MFL_OPT_TAIL).
    opt_tails_supported: bool = False

    def grads_final_from(self, prefix: str) -> None:
        """The backward of every trainable variable from the one named
        ``prefix``... on has been issued (their gradients are final)."""
        sched = self.ws.opt_tails
        if sched is not None:
            lo = self.state.offset_of_prefix(prefix)
            if lo is not None:
                sched.mark_ready(lo)

    def _train_body(self, ds: DeviceDataset) -> None:
        st = self.state
        if not self.zero_grad_in_optimizer:
            st.grad32.zero_()
        tails = (self.opt_tails_supported and OptTailScheduler.chunk > 0 and st.optimizer is not None
                 and st.n_params > 0)
        self.ws.opt_tails = OptTailScheduler(st, self.zero_grad_in_optimizer) if tails else None
        K.gather_batch(ds.x, ds.y, ds.perm, st.step, ds.steps_per_epoch, self.B, self.xb, self.yb,
                       xp=self.packed_input())
        out = self.forward_to_head(self.xb, train=True)
        dlast = self.head.forward_backward(out, self.yb, self.stats, train=True)
        for l in self.all_layers():
            l.prepare_backward()
        self.backward(dlast)
        self.ws.join()  # weight-gradient branch (side stream) must land first
        hi = self.ws.opt_tails.done if self.ws.opt_tails is not None else None
        self.ws.opt_tails = None
        # one launch: optimizer (of what no tail covered) + grad re-zero + BN
        # accumulator re-zero + step tick
        if not st.optimizer_step(zero_grad=self.zero_grad_in_optimizer, zero_region=self.ws.bn_acc,
                                 tick=True, hi=hi):
            opt_ops.tick(st.step, 1)

    def _eval_body(self, ds: DeviceDataset) -> None:
        K.gather_batch(ds.x, ds.y, ds.perm, self.eval_step_ctr, ds.steps_per_epoch, self.B,
                       self.xb, self.yb, xp=self.packed_input())
        out = self.forward_to_head(self.xb, train=False)
        self.head.forward_backward(out, self.yb, self.stats, train=False)
        opt_ops.tick(self.eval_step_ctr, 1)

    # -- graph capture ---------------------------------------------------------
    def _capture(self, body, ds):
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        # warm-up on a side stream (allocator/library init), state restored below
        snap = self.state.model32.clone()
        step0 = self.state.step.clone()
        slots = [t.clone() if t is not None else None for t in (self.state.m, self.state.v)]
        # the warm-up and captured bodies also accumulate loss / accuracy and
        # tick the evaluation counter: restored too, so a task's statistics
        # cover its own updates only
        stats0 = self.stats.clone()
        ectr0 = self.eval_step_ctr.clone()
        with torch.cuda.stream(s):
            body(ds)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # no garbage collection while capturing: a collected object whose
        # destructor frees device memory or destroys an event / stream (another
        # learner's CKKS buffers, a finished task's events) is an illegal call
        # under global-mode capture and aborts the process
        # thread-local capture mode: other threads of this process keep using
        # the GPU while a learner captures -- the asynchronous aggregator's
        # service thread (receives, FedRec kernels, host copies), the
        # background checkpoint writer -- and under the default global mode
        # any "unsafe" call of theirs (a synchronous copy, a stream sync, a
        # device allocation) invalidates this capture
        # (hipErrorStreamCaptureInvalidated; seen on rank 0 of a 2-rank async
        # run, tests/test_multirank_gpu.py).  Their work runs on their own
        # streams, so none of it enters the graph.
        gc.collect()
        was = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                body(ds)
        finally:
            if was:
                gc.enable()
        torch.cuda.synchronize(self.device)
        self.state.model32.copy_(snap)
        self.state.step.copy_(step0)
        for t, c in zip((self.state.m, self.state.v), slots):
            if t is not None:
                t.copy_(c)
        self.stats.copy_(stats0)
        self.eval_step_ctr.copy_(ectr0)
        self.state.refresh_bf16()
        return g

    def use_graphs(self) -> bool:
        return self.device.type == "cuda"

    # Updates per captured train graph: a K-update graph replays K steps per
    # host launch (the batch gather reads the device step counter, so the
    # steps need nothing from the host); chunks never cross an epoch boundary,
    # where the host reshuffles.  MFL_GRAPH_STEPS=1: one graph per update.
    graph_steps: int = int(os.environ.get("MFL_GRAPH_STEPS", "8"))

    def prepare_graphs(self, ds: DeviceDataset, nsteps: int | None = None) -> None:
        """Capture the step graphs for ``ds`` now (1-update and, when a task of
        ``nsteps`` can use it, K-update), instead of lazily at the first
        replay: co-located learners capture before their streams run
        concurrently (models/colocated.py)."""
        if not self.use_graphs():
            return
        if self._train_graph is None or self._train_graph_ds is not ds:
            self._train_graph = self._capture(self._train_body, ds)
            self._train_graph_k = None
            self._train_graph_ds = ds
        K = max(1, self.graph_steps)
        if K > 1 and self._train_graph_k is None and (nsteps is None or nsteps >= K) and ds.steps_per_epoch >= K:
            body = self._train_body
            self._train_graph_k = self._capture(lambda d: [body(d) for _ in range(K)], ds)

    def train_steps_iter(self, ds: DeviceDataset, nsteps: int, step_offset: int = 0):
        """``train_steps`` as a generator that yields after every host launch
        (one graph replay, or one eager step): the co-located learner runner
        interleaves several learners' launches on their own streams."""
        graphs = self.use_graphs()
        if graphs and (self._train_graph is None or self._train_graph_ds is not ds):
            self._train_graph = self._capture(self._train_body, ds)
            self._train_graph_k = None
            self._train_graph_ds = ds
        spe = ds.steps_per_epoch
        K = max(1, self.graph_steps)
        i = 0
        while i < nsteps:
            gstep = step_offset + i
            if gstep > 0 and gstep % spe == 0:
                ds.reshuffle()
            if graphs and K > 1 and nsteps - i >= K and spe - gstep % spe >= K:
                if self._train_graph_k is None:
                    body = self._train_body
                    self._train_graph_k = self._capture(lambda d: [body(d) for _ in range(K)], ds)
                self._train_graph_k.replay()
                i += K
                yield K
                continue
            if graphs:
                self._train_graph.replay()
            else:
                self._train_body(ds)
            i += 1
            yield 1

    def train_steps(self, ds: DeviceDataset, nsteps: int, step_offset: int = 0) -> None:
        """Run ``nsteps`` local updates; reshuffles at epoch boundaries."""
        for _ in self.train_steps_iter(ds, nsteps, step_offset):
            pass

    # Evaluation micro-batch.  BatchNorm runs on its running statistics in
    # inference mode, so a sample's loss / prediction does not depend on the
    # batch it is evaluated in: a full test-set pass (the reference's Keras
    # ``evaluate`` at the training batch size, controller.cc:611) runs through
    # a twin of the model bound to the same parameters at this wider batch --
    # the same samples, each exactly once (padded tail skipped), at 1.35-1.6x
    # the throughput of batch-32 passes on MI355X (scripts/eval_probe.py:
    # 10,000 CIFAR samples 108 -> 80 ms at 128, 68 ms at 512).  ``eval_batch``
    # is the widest twin; a smaller one is used when the widest would pad the
    # dataset's last batch by more than 1/16 of the samples (a 1,250-sample
    # shard at 8 learners: 256).  Twins are kept per batch size (an evaluation
    # task may cover train / validation / test sets of different sizes).
    # MFL_EVAL_BATCH=0 disables it.
    eval_batch: int = int(os.environ.get("MFL_EVAL_BATCH", "512"))

    def _pick_eval_batch(self, n: int) -> int:
        eb = self.eval_batch
        while eb > 128 and (-(-n // eb) * eb - n) * 16 > n:
            eb //= 2
        return eb

    def _make_eval_twin(self, batch: int, state: FlatState | None = None) -> "StaticNet | None":
        """A model of the same architecture at ``batch`` bound to
        ``self.state`` (or ``state``: a detached copy of it) -- models opt in;
        None: evaluate at the training batch."""
        return None

    def _eval_view(self, ds: DeviceDataset):
        """(twin, the twin's dataset over ds's samples), or None."""
        EB = self._pick_eval_batch(ds.n)
        if not (self.use_graphs() and ds.pad_tail and not ds.shuffle and EB > self.B and ds.n > self.B):
            return None
        if EB not in self._eval_twins:
            self._eval_twins[EB] = self._make_eval_twin(EB) or False
        twin = self._eval_twins[EB]
        if twin is False:
            return None
        hit = self._eval_views.get(id(ds))
        if hit is None or hit[0] is not ds or hit[1].batch_size != EB:
            hit = (ds, DeviceDataset(ds.x[:ds.n], ds.y[:ds.n], EB, shuffle=False, pad_tail=True))
            self._eval_views[id(ds)] = hit
        return twin, hit[1]

    def detached_evaluator(self, ds: DeviceDataset, state: FlatState):
        """(model, dataset view) evaluating ``ds`` on ``state`` -- a
        ``FlatState.detached_copy`` of this model's state -- with the
        evaluation twin this model would use, or None when the model has no
        twin (then evaluation stays on the live model)."""
        if not (self.use_graphs() and ds.pad_tail and not ds.shuffle):
            return None
        eb = self._pick_eval_batch(ds.n) if ds.n > self.B else self.B
        twin = self._make_eval_twin(eb, state=state)
        if twin is None:
            return None
        return twin, DeviceDataset(ds.x[:ds.n], ds.y[:ds.n], eb, shuffle=False, pad_tail=True)

    def begin_evaluate(self, ds: DeviceDataset, max_steps: int | None = None):
        """Issue a loss / accuracy pass over ``ds`` (BN in inference mode) on
        the current stream without waiting for it; ``finish_evaluate`` reads
        the result.  -> the model whose statistics hold it (self or the
        evaluation twin)."""
        view = self._eval_view(ds) if max_steps is None else None
        if view is not None:
            return view[0].begin_evaluate(view[1])
        nsteps = ds.steps_per_epoch if max_steps is None else min(max_steps, ds.steps_per_epoch)
        self.stats.zero_()
        self.eval_step_ctr.zero_()
        if self.use_graphs() and (self._eval_graph is None or self._eval_graph_ds is not ds):
            self._eval_graph = self._capture(self._eval_body, ds)
            self._eval_graph_ds = ds
            self.stats.zero_()
            self.eval_step_ctr.zero_()
        for _ in range(nsteps):
            if self.use_graphs():
                self._eval_graph.replay()
            else:
                self._eval_body(ds)
        return self

    @staticmethod
    def finish_evaluate(owner: "StaticNet") -> dict:
        s = owner.stats.cpu().numpy()
        n = max(1.0, float(s[2]))
        return {"loss": float(s[0] / n), "accuracy": float(s[1] / n)}

    def evaluate(self, ds: DeviceDataset, max_steps: int | None = None) -> dict:
        """Loss / accuracy of the current model on ``ds`` (BN in inference mode)."""
        return self.finish_evaluate(self.begin_evaluate(ds, max_steps))

    def reset_train_stats(self) -> None:
        self.stats.zero_()

    def train_stats(self) -> dict:
        s = self.stats.cpu().numpy()
        n = max(1.0, float(s[2]))
        return {"loss": float(s[0] / n), "accuracy": float(s[1] / n)}

    # -- data helpers ----------------------------------------------------------
    def make_dataset(self, x_nhwc: np.ndarray | torch.Tensor, y: np.ndarray | torch.Tensor,
                     seed: int = 0, shuffle: bool = True, batch_size: int | None = None,
                     drop_last: bool | None = None) -> DeviceDataset:
        """Upload a shard: pads channels to the model's input width, casts to
        the compute dtype."""
        x = torch.as_tensor(x_nhwc)
        if x.dim() > 2 and len(self.input_shape) == 1:
            x = x.reshape(x.shape[0], -1)  # (N, H, W[, 1]) images into a flat MLP input
        if x.shape[-1] < self.input_shape[-1]:
            pad = self.input_shape[-1] - x.shape[-1]
            x = torch.nn.functional.pad(x, (0, pad))  # zero channels / features up to the 8-wide rows
        x = x.to(self.compute_dtype).to(self.device)
        y = torch.as_tensor(y)
        if y.is_floating_point():  # regression targets: fp32 bits in the int32 label slots
            y = y.to(torch.float32).contiguous().view(torch.int32)
        y = y.to(torch.int32).to(self.device)
        # training shards: ceil(n / B) steps per epoch (wrapped last batch);
        # evaluation shards (unshuffled): ceil(n / B) steps, the last batch's
        # tail is padding the statistics skip (every sample exactly once)
        return DeviceDataset(x, y, batch_size or self.B, seed=seed, shuffle=shuffle,
                             drop_last=bool(drop_last), pad_tail=not shuffle and not drop_last)

    @staticmethod
    def timer():
        return time.perf_counter()
