"""User PyTorch models on the collective data plane (``DataPlane: rccl``).

The reference runs every model through one protocol and one aggregation
path whatever its backend: a Keras model's ``fit`` (metisfl/models/keras/
keras_model_ops.py:117-197) or a user PyTorch model's own ``fit``
(metisfl/models/pytorch/pytorch_model_ops.py:83-131, examples/pytorch/
dummy.py:18-103), the weights then serialized through the controller.

``TorchNet`` gives a user ``nn.Module`` (a :class:`TorchModelDef`) the
interface the collective federation drives (the one ``StaticNet`` exposes:
``state`` / ``make_dataset`` / ``train_steps_iter`` / ``begin_evaluate`` ...),
so synchronous / semi-synchronous FedAvg (K1 over co-located learners + one
RCCL all-reduce), asynchronous FedRec over point-to-point transfers,
straggler drop, checkpoints and recovery run on user models unchanged:

* every floating-point ``state_dict`` entry of the module is re-pointed into
  ONE flat fp32 buffer (:class:`ModuleState`, a ``FlatState``): trainable
  parameters first -- the fused HIP optimizer's domain, one launch per
  update (ops/optim.py) -- then frozen parameters and buffers (BatchNorm
  running statistics, which FedAvg averages like the reference's Keras
  weights, federated_average.cc:97-99).  Gradients land in one flat
  gradient buffer the same way.  The module computes straight from those
  views: no copy in or out around a task;
* the shard is device-resident (:class:`TorchDataset`): per-epoch
  permutation on the device, batches gathered by index, targets kept in
  their own dtype (regression ages, class ids);
* the step is the module's own forward (PyTorch-ROCm ops: these are user
  layers, not framework hot paths) + ``model_def.loss`` + backward + the
  fused optimizer; a ``TorchModelDef`` that overrides ``fit(model, dataset,
  epochs)`` keeps full control of its loop, as with the reference's
  PyTorchDef, and is handed a host ``ModelDataset`` of its shard;
* loss / accuracy accumulate on the device and are read once per task.

Integer buffers (``num_batches_tracked``) stay local to each replica: they
are counters, not model state the reference federates (its PyTorch learner
exports ``named_parameters`` only, pytorch_model_ops.py:61-70)."""
from __future__ import annotations

import math

import numpy as np
import torch

from metisfl_amd.models.flat import ALIGN, FlatState, VarSpec
from metisfl_amd.ops import optim as opt_ops
from metisfl_amd.ops.optim import OptimizerSpec


class ModuleState(FlatState):
    """FlatState over an existing ``nn.Module``: the module's floating-point
    parameters and buffers BECOME views of ``model32`` (parameter gradients
    views of ``grad32``)."""

    def __init__(self, module: torch.nn.Module, device, optimizer: OptimizerSpec | None = None):
        sd = module.state_dict(keep_vars=True)
        seen, specs, self._entries = set(), [], []
        for name, t in sd.items():
            if not torch.is_floating_point(t) or id(t) in seen:  # int counters; tied weights once
                continue
            seen.add(id(t))
            trainable = isinstance(t, torch.nn.Parameter) and t.requires_grad
            specs.append(VarSpec(name, tuple(t.shape), trainable=trainable))
            self._entries.append((name, t))
        # fp32 master, no compute mirror: the module computes from model32
        super().__init__(specs, device, None, seed=0, compute_dtype=torch.float32)
        self.psplit = None
        with torch.no_grad():
            for name, t in self._entries:
                s = self.by_name[name]
                view = self.model32[s.offset: s.offset + s.numel].view(s.shape)
                view.copy_(t.detach().to(self.device, torch.float32))
                if isinstance(t, torch.nn.Parameter):
                    t.data = view
                    if s.trainable:
                        t.grad = self.grad32[s.offset: s.offset + s.numel].view(s.shape)
                else:  # a registered buffer: swap the owning module's entry
                    owner, _, leaf = name.rpartition(".")
                    mod = module.get_submodule(owner) if owner else module
                    mod._buffers[leaf] = view
        if optimizer is not None:
            self.set_optimizer(optimizer)

    def refresh_bf16(self) -> None:  # fp32 module: no mirror to re-derive
        return


class TorchDataset:
    """A learner's shard resident on the device for a user module: inputs as
    given (float32 or integer token ids), targets in their own dtype, and a
    per-epoch permutation buffer (the ``DeviceDataset`` contract: ``n``,
    ``steps_per_epoch``, ``perm``, ``reshuffle``).  An epoch is ceil(n / B)
    batches, the last one short (Keras / the reference's torch loop do the
    same)."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor, batch_size: int, seed: int = 0, shuffle: bool = True):
        assert x.shape[0] == y.shape[0]
        self.n = int(x.shape[0])
        self.x, self.y = x.contiguous(), y.contiguous()
        self.batch_size = int(batch_size)
        self.steps_per_epoch = max(1, -(-self.n // self.batch_size))
        self.shuffle = shuffle
        self.pad_tail = not shuffle
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(seed)
        self.perm = torch.zeros(self.n, dtype=torch.int64, device=x.device)
        self.reshuffle()

    def reshuffle(self) -> None:
        p = torch.randperm(self.n, generator=self.gen) if self.shuffle else torch.arange(self.n)
        if self.perm.is_cuda:
            p = p.pin_memory()  # an asynchronous copy (models/net.py DeviceDataset.reshuffle)
        self.perm.copy_(p, non_blocking=True)

    def batch(self, i: int):
        """Batch ``i`` of the current epoch."""
        idx = self.perm[i * self.batch_size: min(self.n, (i + 1) * self.batch_size)]
        return self.x.index_select(0, idx), self.y.index_select(0, idx)

    def host_dataset(self):
        from metisfl_amd.models.model_dataset import ModelDataset
        return ModelDataset(self.x.cpu().numpy(), self.y.cpu().numpy(), self.n)


class TorchNet:
    """A TorchModelDef's module driven like a StaticNet (see module doc)."""

    def __init__(self, model_def, batch_size: int, device="cpu", optimizer: OptimizerSpec | None = None,
                 seed: int = 0):
        torch.manual_seed(seed)
        self.model_def = model_def
        self.B = int(batch_size)
        self.device = torch.device(device)
        self.module = model_def.get_model().to(self.device)
        self.state = ModuleState(self.module, self.device, optimizer or OptimizerSpec())
        self.stats = torch.zeros(3, dtype=torch.float64, device=self.device)  # loss sum, correct, samples
        self._eval_stats = torch.zeros(3, dtype=torch.float64, device=self.device)
        self._user_fit = callable(getattr(model_def, "fit", None))
        self._user_eval = callable(getattr(model_def, "evaluate", None))

    # -- datasets --------------------------------------------------------------------
    def make_dataset(self, x, y, seed: int = 0, shuffle: bool = True, batch_size: int | None = None,
                     drop_last: bool | None = None) -> TorchDataset:
        x = torch.as_tensor(np.asarray(x))
        x = x.to(self.device, torch.float32 if x.is_floating_point() else x.dtype)
        y = torch.as_tensor(np.asarray(y)).to(self.device)
        return TorchDataset(x, y, batch_size or self.B, seed=seed, shuffle=shuffle)

    # -- training --------------------------------------------------------------------
    def prepare_graphs(self, ds, nsteps=None) -> None:
        """User modules run eagerly (arbitrary Python control flow is not a
        capturable static graph)."""

    def _accumulate(self, stats: torch.Tensor, out: torch.Tensor, yb: torch.Tensor, loss: torch.Tensor) -> None:
        n = yb.shape[0]
        stats[0] += loss.detach().double() * n
        if out.dim() == 2 and out.shape[1] > 1:
            stats[1] += (out.detach().argmax(1) == yb.long()).sum().double()
        stats[2] += n

    def _step(self, ds: TorchDataset, i: int) -> None:
        st = self.state
        xb, yb = ds.batch(i)
        out = self.module(xb)
        loss = self.model_def.loss(out, yb)
        loss.backward()
        if st.n_params:
            opt_ops.fused_step(st.optimizer, st.params32, st.grad32, st.m, st.v, st.anchor, None, st.lr_scale,
                               st.step, zero_grad=True)
        opt_ops.tick(st.step, 1)
        self._accumulate(self.stats, out, yb, loss)

    def train_steps_iter(self, ds: TorchDataset, nsteps: int, step_offset: int = 0):
        """``nsteps`` local updates (yields after each; the co-located runner
        interleaves learners).  A user ``fit`` runs once for the task's
        epochs and counts as the whole budget."""
        self.module.train()
        if self._user_fit:
            spe = ds.steps_per_epoch
            self.model_def.fit(self.module, ds.host_dataset(), max(1, math.ceil(nsteps / spe)))
            opt_ops.tick(self.state.step, nsteps)
            yield nsteps
            return
        spe = ds.steps_per_epoch
        for k in range(nsteps):
            g = step_offset + k
            if g > 0 and g % spe == 0:
                ds.reshuffle()
            self._step(ds, g % spe)
            yield 1

    def train_steps(self, ds: TorchDataset, nsteps: int, step_offset: int = 0) -> None:
        for _ in self.train_steps_iter(ds, nsteps, step_offset):
            pass

    def reset_train_stats(self) -> None:
        self.stats.zero_()

    @staticmethod
    def _read(stats: torch.Tensor) -> dict:
        s = stats.cpu().numpy()
        n = max(1.0, float(s[2]))
        return {"loss": float(s[0] / n), "accuracy": float(s[1] / n)}

    def train_stats(self) -> dict:
        return self._read(self.stats)

    # -- evaluation --------------------------------------------------------------------
    @torch.no_grad()
    def begin_evaluate(self, ds: TorchDataset, max_steps: int | None = None):
        """Loss / accuracy of the current model over ``ds`` (every sample
        once; BatchNorm in inference mode), issued on the current stream."""
        if self._user_eval:
            self.module.eval()
            self._eval_result = dict(self.model_def.evaluate(self.module, ds.host_dataset()))
            self.module.train()
            return self
        self._eval_result = None
        self._eval_stats.zero_()
        self.module.eval()
        nb = ds.steps_per_epoch if max_steps is None else min(max_steps, ds.steps_per_epoch)
        for i in range(nb):
            xb, yb = ds.batch(i)
            out = self.module(xb)
            self._accumulate(self._eval_stats, out, yb, self.model_def.loss(out, yb))
        self.module.train()
        return self

    @staticmethod
    def finish_evaluate(owner: "TorchNet") -> dict:
        if owner._eval_result is not None:
            r = owner._eval_result
            return {"loss": float(r.get("loss", float("nan"))), "accuracy": float(r.get("accuracy", 0.0)), **r}
        return owner._read(owner._eval_stats)

    def evaluate(self, ds: TorchDataset, max_steps: int | None = None) -> dict:
        return self.finish_evaluate(self.begin_evaluate(ds, max_steps))


def aligned(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN
