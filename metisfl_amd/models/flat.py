"""Flat, device-resident model state.

Every variable of a learner's model lives in ONE fp32 buffer (``model32``):
trainable variables first (the optimizer's domain), then non-trainable ones
(BatchNorm running statistics).  Around it sit the fp32 gradient buffer, the
optimizer slots, the proximal anchor and the bf16 compute mirror.  Because
the layout is flat:

* a whole optimizer step is one kernel launch (ops.optim.fused_step),
* FedAvg of the whole model is one scale kernel + ONE RCCL all-reduce,
* the community model is resident on every learner GPU after the collective,
* export to the reference's ``Model`` proto (one ``Variable`` per tensor,
  metisfl/proto/model.proto:79-99) is a per-segment view, no gather.

The reference aggregates all variables, trainable or not
(federated_average.cc:97-99); so does this layout.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from metisfl_amd.ops import optim as opt_ops
from metisfl_amd.ops.optim import OptimizerSpec

ALIGN = 64  # elements: every segment starts 256-B aligned (16-B vector loads)


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class VarSpec:
    name: str
    shape: tuple
    trainable: bool = True
    init: str = "zeros"        # zeros | ones | he_normal | glorot_uniform | normal
    fan_in: int = 0
    fan_out: int = 0
    offset: int = 0            # filled by FlatState
    # rows (dim 0) >= live_rows are zero-initialised: padding units that the
    # 8-wide kernels need stay exactly zero (inert) through training
    live_rows: int | None = None

    @property
    def numel(self) -> int:
        return int(np.prod(self.shape)) if self.shape else 1


class FlatState:
    def __init__(self, specs: list[VarSpec], device: torch.device | str = "cpu",
                 optimizer: OptimizerSpec | None = None, seed: int = 0,
                 compute_dtype: torch.dtype = torch.bfloat16):
        self.device = torch.device(device)
        # fp32 models compute straight from the master (no mirror); bf16
        # models keep a bf16 compute copy refreshed by the optimizer launch
        self.compute_dtype = compute_dtype
        train = [s for s in specs if s.trainable]
        frozen = [s for s in specs if not s.trainable]
        off = 0
        for s in train:
            s.offset = off
            off += _align(s.numel)
        self.n_params = off
        for s in frozen:
            s.offset = off
            off += _align(s.numel)
        self.n_total = max(off, ALIGN)
        self.specs = train + frozen
        self.by_name = {s.name: s for s in self.specs}
        dev = self.device
        self.model32 = torch.zeros(self.n_total, dtype=torch.float32, device=dev)
        self.params32 = self.model32[: self.n_params]
        self.grad32 = torch.zeros(max(self.n_params, ALIGN), dtype=torch.float32, device=dev)[: self.n_params]
        self.p16 = (torch.zeros(self.n_params, dtype=torch.bfloat16, device=dev)
                    if compute_dtype == torch.bfloat16 else None)
        # fp32 GPU models whose convolutions run bf16x3 products keep a packed
        # (hi << 16 | lo) bf16 split of the weights, written by the optimizer
        # launch like the bf16 mirror (conv32.hip decodes it with v_perm
        # instead of splitting every weight fragment in every k-loop)
        self.psplit = None
        if compute_dtype == torch.float32 and dev.type == "cuda" and self.n_params:
            from metisfl_amd.ops.nn import conv_products
            if conv_products() == "bf16x3":
                self.psplit = torch.zeros(self.n_params, dtype=torch.int32, device=dev)
        self.anchor: torch.Tensor | None = None
        self.m: torch.Tensor | None = None
        self.v: torch.Tensor | None = None
        self.lr_scale = torch.ones(1, dtype=torch.float32, device=dev)
        self.step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.optimizer: OptimizerSpec | None = None
        self.initialize(seed)
        if optimizer is not None:
            self.set_optimizer(optimizer)

    # ---- views --------------------------------------------------------------
    def view(self, name: str) -> torch.Tensor:
        s = self.by_name[name]
        return self.model32[s.offset: s.offset + s.numel].view(s.shape)

    def grad(self, name: str) -> torch.Tensor:
        s = self.by_name[name]
        assert s.trainable
        return self.grad32[s.offset: s.offset + s.numel].view(s.shape)

    def bf16(self, name: str) -> torch.Tensor:
        s = self.by_name[name]
        assert s.trainable and self.p16 is not None
        return self.p16[s.offset: s.offset + s.numel].view(s.shape)

    def packed(self, name: str) -> torch.Tensor | None:
        """The packed bf16x3 split of a weight (int32 view), or None."""
        if self.psplit is None:
            return None
        s = self.by_name[name]
        assert s.trainable
        return self.psplit[s.offset: s.offset + s.numel]

    def compute(self, name: str) -> torch.Tensor:
        """The weight view the kernels read: the bf16 mirror, or the fp32
        master itself for reference-precision models."""
        return self.bf16(name) if self.p16 is not None else self.view(name)

    # ---- init ---------------------------------------------------------------
    def initialize(self, seed: int = 0) -> None:
        rng = np.random.default_rng(seed)
        host = np.zeros(self.n_total, dtype=np.float32)
        for s in self.specs:
            n = s.numel
            if s.init == "ones":
                val = np.ones(n, np.float32)
            elif s.init == "he_normal":
                std = math.sqrt(2.0 / max(1, s.fan_in))
                val = rng.normal(0.0, std, n).astype(np.float32)
            elif s.init == "glorot_uniform":
                lim = math.sqrt(6.0 / max(1, s.fan_in + s.fan_out))
                val = rng.uniform(-lim, lim, n).astype(np.float32)
            elif s.init == "normal":
                val = rng.normal(0.0, 0.02, n).astype(np.float32)
            else:
                val = np.zeros(n, np.float32)
            if s.live_rows is not None and s.shape:
                val = val.reshape(s.shape[0], -1)
                val[s.live_rows:] = 0.0
                val = val.reshape(-1)
            host[s.offset: s.offset + n] = val
        self.model32.copy_(torch.from_numpy(host))
        self.refresh_bf16()

    def refresh_bf16(self) -> None:
        """Re-derive the weight mirror (bf16 copy or packed bf16x3 split) from
        the fp32 master after it was written outside the optimizer."""
        if self.n_params and self.p16 is not None:
            opt_ops.cast_bf16(self.params32, self.p16)
        if self.n_params and self.psplit is not None:
            opt_ops.split_pack(self.params32, self.psplit)

    # ---- optimizer ----------------------------------------------------------
    def set_optimizer(self, spec: OptimizerSpec, reset_state: bool = False) -> None:
        prev = self.optimizer
        self.optimizer = spec
        dev = self.device
        if spec.needs_m and (self.m is None or reset_state or (prev and prev.kind != spec.kind)):
            self.m = torch.zeros(self.n_params, dtype=torch.float32, device=dev)
        if spec.needs_v and (self.v is None or reset_state or (prev and prev.kind != spec.kind)):
            self.v = torch.zeros(self.n_params, dtype=torch.float32, device=dev)
        if spec.needs_anchor and self.anchor is None:
            self.anchor = self.params32.clone()

    def optimizer_step(self, zero_grad: bool = True, zero_region: torch.Tensor | None = None,
                       tick: bool = False, hi: int | None = None) -> bool:
        """One fused optimizer launch over the trainables [0, hi) (default:
        all; the rest was updated by optimizer tails); ``tick``: it also
        increments the step counter (returns False when no launch happened --
        the caller ticks)."""
        if self.n_params == 0 or self.optimizer is None:
            return False
        r = self.opt_range(0, self.n_params if hi is None else hi, zero_grad)
        opt_ops.fused_step(self.optimizer, r.p, r.g, r.m, r.v, r.anchor, r.mirror, self.lr_scale, self.step,
                           zero_grad, zero_region, tick)
        return True

    def opt_range(self, lo: int, hi: int, zero_grad: bool = True) -> "opt_ops.OptRange":
        """The optimizer step over trainables [lo, hi) (multiples of ALIGN)."""
        assert 0 <= lo <= hi <= self.n_params and lo % ALIGN == 0 and (hi % ALIGN == 0 or hi == self.n_params)

        def part(t):
            return None if t is None else t[lo:hi]
        mirror = self.p16 if self.p16 is not None else self.psplit
        return opt_ops.OptRange(self.optimizer, part(self.params32), part(self.grad32), part(self.m), part(self.v),
                                part(self.anchor), part(mirror), self.lr_scale, self.step, zero_grad)

    def offset_of_prefix(self, prefix: str) -> int | None:
        """Offset of the first trainable variable whose name starts with
        ``prefix`` (trainables are laid out in layer order), or None."""
        for s in self.specs:
            if s.trainable and s.name.startswith(prefix):
                return s.offset
        return None

    def set_anchor(self) -> None:
        """Snapshot the received community model as the FedProx anchor."""
        if self.anchor is not None:
            self.anchor.copy_(self.params32)

    def detached_copy(self) -> "FlatState":
        """A state of the same layout with its OWN model buffers (fp32 master
        and compute mirror) and no optimizer: a frozen snapshot a forward-only
        model binds to (the deferred community evaluation evaluates the
        round's community model on it while the learners already train the
        next round).  The gradient buffer is shared: a forward pass never
        writes it."""
        import copy
        c = copy.copy(self)
        c.model32 = self.model32.clone()
        c.params32 = c.model32[: self.n_params]
        c.p16 = self.p16.clone() if self.p16 is not None else None
        c.psplit = self.psplit.clone() if self.psplit is not None else None
        c.anchor = c.m = c.v = None
        c.optimizer = None
        c.step = self.step.clone()
        c.lr_scale = self.lr_scale.clone()
        return c

    def copy_model_from(self, src: "FlatState") -> None:
        """model32 and its compute mirror <- ``src``'s (same layout; on the
        current stream)."""
        self.model32.copy_(src.model32)
        if self.p16 is not None and src.p16 is not None:
            self.p16.copy_(src.p16)
        if self.psplit is not None and src.psplit is not None:
            self.psplit.copy_(src.psplit)
        elif self.psplit is not None or self.p16 is not None:
            self.refresh_bf16()

    # ---- variable export / import (Model proto boundary) ---------------------
    def named_variables(self):
        for s in self.specs:
            yield s.name, s.trainable, self.view(s.name)

    def to_numpy(self) -> dict[str, np.ndarray]:
        host = self.model32.detach().cpu().numpy()
        return {s.name: host[s.offset: s.offset + s.numel].reshape(s.shape).copy() for s in self.specs}

    def load_numpy(self, values: dict[str, np.ndarray], strict: bool = True) -> None:
        host = self.model32.detach().cpu().numpy().copy()
        for s in self.specs:
            if s.name not in values:
                if strict:
                    raise KeyError(f"missing variable {s.name}")
                continue
            v = np.asarray(values[s.name], dtype=np.float32).reshape(-1)
            if v.size != s.numel:
                raise ValueError(f"{s.name}: {v.size} values, expected {s.numel}")
            host[s.offset: s.offset + s.numel] = v
        self.model32.copy_(torch.from_numpy(host))
        self.refresh_bf16()

    def segments(self) -> list[tuple[int, int]]:
        return [(s.offset, s.offset + s.numel) for s in self.specs]
