"""Fused flat-buffer optimizers (K3/K4/K5).

One launch updates EVERY trainable variable of a learner: the fp32 master
weights, the optimizer slots and the bf16 compute copy.  The optimizer kinds
and their hyper-parameters mirror ``OptimizerConfig`` of the reference
(metisfl/proto/model.proto:116-151, applied in
metisfl/models/keras/keras_model_ops.py:245-283):

* ``vanilla_sgd``      p -= lr * (g + l2*p + l1*sign(p))
* ``momentum_sgd``     v = mu*v - lr*g ; p += v            (Keras form)
* ``fed_prox``         p -= lr * (g + mu*(p - p_community))
* ``adam``             bias-corrected Adam (Keras default eps 1e-7)
* ``adam_weight_decay`` Adam + decoupled weight decay

FedProx note: the reference's Keras FedProx keeps its ``vstar`` slot at zero
(fed_prox.py:44-60); here the anchor is the community
model received for the round, which is the algorithm's intended semantics.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from metisfl_amd.ops._native import ops

OPT_SGD, OPT_MOMENTUM, OPT_FEDPROX, OPT_ADAM, OPT_ADAMW = range(5)
_KIND = {
    "vanilla_sgd": OPT_SGD,
    "momentum_sgd": OPT_MOMENTUM,
    "fed_prox": OPT_FEDPROX,
    "adam": OPT_ADAM,
    "adam_weight_decay": OPT_ADAMW,
}


@dataclass
class OptimizerSpec:
    kind: str = "vanilla_sgd"
    learning_rate: float = 0.01
    l1: float = 0.0
    l2: float = 0.0
    momentum: float = 0.0
    proximal_term: float = 0.0
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-7
    weight_decay: float = 0.0
    extra: dict = field(default_factory=dict)

    @property
    def mode(self) -> int:
        return _KIND[self.kind]

    @property
    def needs_m(self) -> bool:
        return self.mode in (OPT_MOMENTUM, OPT_ADAM, OPT_ADAMW)

    @property
    def needs_v(self) -> bool:
        return self.mode in (OPT_ADAM, OPT_ADAMW)

    @property
    def needs_anchor(self) -> bool:
        return self.mode == OPT_FEDPROX

    @classmethod
    def from_proto(cls, pb) -> "OptimizerSpec":
        """Build from a ``metisfl.OptimizerConfig`` message."""
        which = pb.WhichOneof("config")
        if which is None:
            raise ValueError("OptimizerConfig has no optimizer set")
        c = getattr(pb, which)
        if which == "vanilla_sgd":
            return cls(which, c.learning_rate, l1=c.L1_reg, l2=c.L2_reg)
        if which == "momentum_sgd":
            return cls(which, c.learning_rate, momentum=c.momentum_factor)
        if which == "fed_prox":
            return cls(which, c.learning_rate, proximal_term=c.proximal_term)
        if which == "adam":
            return cls(which, c.learning_rate, beta1=c.beta_1 or 0.9, beta2=c.beta_2 or 0.999,
                       epsilon=c.epsilon or 1e-7)
        if which == "adam_weight_decay":
            return cls(which, c.learning_rate, weight_decay=c.weight_decay)
        raise ValueError(f"unsupported optimizer {which}")


def fused_step(spec: OptimizerSpec, p: torch.Tensor, g: torch.Tensor,
               m: torch.Tensor | None = None, v: torch.Tensor | None = None,
               anchor: torch.Tensor | None = None, p16: torch.Tensor | None = None,
               lr_scale: torch.Tensor | None = None, step: torch.Tensor | None = None,
               zero_grad: bool = False, zero_region: torch.Tensor | None = None,
               tick: bool = False) -> None:
    """Apply one optimizer step in place over flat buffers.  ``zero_grad``
    writes 0 back into ``g`` once consumed and ``zero_region`` (e.g. the
    BatchNorm accumulators) is cleared by the same launch, so the next step's
    atomic accumulations start from zero without a memset node.
    ``tick``: also increment ``step`` once, after the optimizer has read it
    (inside the same launch for the modes that never read it)."""
    if p.is_cuda:
        ops().fused_optimizer(spec.mode, p, g, m, v, anchor, p16, spec.learning_rate, spec.l1,
                              spec.l2, spec.momentum, spec.proximal_term, spec.beta1, spec.beta2,
                              spec.epsilon, spec.weight_decay, lr_scale, step, zero_grad,
                              zero_region, tick)
        return
    _reference_step(spec, p, g, m, v, anchor, p16, lr_scale, step)
    if zero_grad:
        g.zero_()
    if zero_region is not None:
        zero_region.zero_()
    if tick:
        step.add_(1)


class OptRange:
    """One fused optimizer step over a range of the flat model (views of the
    master, gradient, slots, anchor and weight mirror): the unit an
    optimizer tail carries (conv32.h OptTail -- the range's update rides in a
    later layer's paired backward launch).  ``run()`` is the stand-alone
    launch (fallback paths)."""

    def __init__(self, spec: OptimizerSpec, p, g, m=None, v=None, anchor=None, mirror=None,
                 lr_scale=None, step=None, zero_grad: bool = True):
        self.spec, self.p, self.g, self.m, self.v = spec, p, g, m, v
        self.anchor, self.mirror, self.lr_scale, self.step, self.zero_grad = anchor, mirror, lr_scale, step, zero_grad

    @property
    def numel(self) -> int:
        return int(self.p.numel())

    def hyper(self) -> list[float]:
        s = self.spec
        return [s.learning_rate, s.l1, s.l2, s.momentum, s.proximal_term, s.beta1, s.beta2, s.epsilon,
                s.weight_decay]

    def binding_args(self) -> tuple:
        """The trailing optimizer-tail arguments of conv32_backward_pair."""
        return (self.p, self.g, self.m, self.v, self.anchor, self.mirror, self.lr_scale, self.step,
                self.spec.mode, self.hyper(), self.zero_grad)

    def run(self) -> None:
        fused_step(self.spec, self.p, self.g, self.m, self.v, self.anchor, self.mirror, self.lr_scale, self.step,
                   zero_grad=self.zero_grad)


NO_OPT_TAIL = (None, None, None, None, None, None, None, None, 0, [0.0] * 9, False)


@torch.no_grad()
def _reference_step(spec, p, g, m, v, anchor, p16, lr_scale, step):
    lr = spec.learning_rate * (float(lr_scale[0]) if lr_scale is not None else 1.0)
    mode = spec.mode
    if mode == OPT_SGD:
        gr = g + spec.l2 * p
        if spec.l1:
            gr = gr + spec.l1 * torch.sign(p)
        p.sub_(lr * gr)
    elif mode == OPT_MOMENTUM:
        m.mul_(spec.momentum).sub_(lr * g)
        p.add_(m)
    elif mode == OPT_FEDPROX:
        p.sub_(lr * (g + spec.proximal_term * (p - anchor)))
    else:
        t = float(int(step[0]) + 1) if step is not None else 1.0
        m.mul_(spec.beta1).add_((1 - spec.beta1) * g)
        v.mul_(spec.beta2).add_((1 - spec.beta2) * g * g)
        mh = m / (1 - spec.beta1 ** t)
        vh = v / (1 - spec.beta2 ** t)
        upd = mh / (vh.sqrt() + spec.epsilon)
        if mode == OPT_ADAMW:
            upd = upd + spec.weight_decay * p
        p.sub_(lr * upd)
    if p16 is not None:
        p16.copy_(p.to(torch.bfloat16))


def split_pack(x: torch.Tensor, y: torch.Tensor) -> None:
    """y (int32) = packed (hi << 16 | lo) bf16 split of the fp32 x."""
    if x.is_cuda:
        ops().split_pack_f32(x, y)
        return
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    h = hi.view(torch.int16).to(torch.int32) & 0xFFFF
    lw = lo.view(torch.int16).to(torch.int32) & 0xFFFF
    y.copy_((h << 16) | lw)


def cast_bf16(x: torch.Tensor, y: torch.Tensor) -> None:
    if x.is_cuda:
        ops().cast_f32_bf16(x, y)
    else:
        y.copy_(x.to(torch.bfloat16))


def scale_(x: torch.Tensor, w: float, wdev: torch.Tensor | None = None) -> None:
    if x.is_cuda:
        ops().scale_f32(x, float(w), wdev)
    else:
        x.mul_(float(wdev[0]) if wdev is not None else float(w))


def tick(step: torch.Tensor, inc: int = 1) -> None:
    if step.is_cuda:
        ops().tick(step, inc)
    else:
        step.add_(inc)
