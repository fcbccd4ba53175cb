"""Neural-network ops of the learner's local-training step.

Device tensors dispatch to the hand-written HIP kernels in ``csrc/kernels``
(implicit-GEMM MFMA convolution, fused BatchNorm, fused classifier head, the
batch gather).  CPU tensors use plain-PyTorch references with identical
semantics; they power the host-only test suite and are what the GPU numerics
tests compare the kernels against.

Tensor conventions: activations NHWC ``[N, H, W, C]``; conv weights KRSC
``[Cout, R, S, Cin]``; all per-channel BatchNorm state is fp32.  Two compute
precisions share these ops and dispatch on the activation dtype:

* fp32 -- the reference precision (Keras trains fp32): conv32.hip on the exact
  fp32 MFMA (v_mfma_f32_32x32x2_f32), bn32.hip, the fp32 head; weights are the
  fp32 master itself.
* bf16 -- the explicit mixed-precision option: conv.hip on bf16 MFMA with a
  bf16 compute copy of the weights.

The fp32 convolutions have two product modes (:func:`set_conv_products`):
``"exact"`` (every product an fp32 FMA on the fp32 matrix pipe) and
``"bf16x3"`` (fp32 operands split in-register into bf16 hi + lo, products
hi*hi + hi*lo + lo*hi on the bf16 matrix pipe, fp32 accumulation: storage,
accumulation and every non-conv op stay fp32; the dropped lo*lo term and the
lo rounding bound each product's relative error by ~2^-17, measured 4e-6
relative on whole convolutions vs 3e-7 exact -- well inside the 1e-5 the
kernel tests pin, and ~100x tighter than the TF32 convolutions TensorFlow
runs "fp32" Keras models on by default on Ampere-class GPUs).
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from metisfl_amd.ops._native import ops


CONV_PRODUCTS = ("exact", "bf16x3")


def set_conv_products(mode: str) -> None:
    """Process-wide product mode of the fp32 convolutions (see module doc).
    Takes effect for launches issued afterwards: set it before a model
    captures its step graph."""
    if mode not in CONV_PRODUCTS:
        raise ValueError(f"conv products must be one of {CONV_PRODUCTS}, not {mode!r}")
    ops().set_conv32_mode(CONV_PRODUCTS.index(mode))


def conv_products() -> str:
    return CONV_PRODUCTS[ops().conv32_mode()]


def out_dim(n: int, k: int, stride: int, pad: int) -> int:
    return (n + 2 * pad - k) // stride + 1


@dataclass(frozen=True)
class ConvShape:
    N: int
    H: int
    W: int
    C: int
    Co: int
    R: int
    S: int
    stride: int
    pad: int

    @property
    def P(self) -> int:
        return out_dim(self.H, self.R, self.stride, self.pad)

    @property
    def Q(self) -> int:
        return out_dim(self.W, self.S, self.stride, self.pad)

    def args(self):
        return (self.N, self.H, self.W, self.C, self.Co, self.R, self.S, self.stride, self.pad)


@dataclass(frozen=True)
class ConvPlan:
    bm: int
    bn: int
    splits: int
    kchunk: int
    stats_rows: int
    workspace: int


def conv_plan(mode: int, shp: ConvShape, device: torch.device, dtype=torch.bfloat16) -> ConvPlan:
    """mode 0 fwd / 1 dgrad / 2 wgrad (tile sizes, split-K factor, fp32 split-K
    workspace floats).  CPU path: no workspace."""
    if device.type == "cuda":
        fn = ops().conv32_plan if dtype == torch.float32 else ops().conv_plan
        return ConvPlan(*fn(mode, *shp.args()))
    return ConvPlan(0, 0, 1, 0, 1, 0)


# ---------------------------------------------------------------------------
# CPU references
def _nchw(x: torch.Tensor) -> torch.Tensor:
    return x.float().permute(0, 3, 1, 2)


def _wt(w: torch.Tensor) -> torch.Tensor:
    return w.float().permute(0, 3, 1, 2)


def _acc_total(acc: torch.Tensor, C: int) -> torch.Tensor:
    """BN accumulators may hold R replicas [R][2][C] (the fp32 kernels spread
    their fp64 atomics over them); the statistics are their sum."""
    return acc[: acc.numel() // (2 * C) * 2 * C].reshape(-1, 2 * C).sum(0)


def _acc_stats_cpu(y: torch.Tensor, acc: torch.Tensor) -> None:
    yf = y.float().reshape(-1, y.shape[-1]).double()
    C = yf.shape[1]
    acc[:C] += yf.sum(0)
    acc[C:2 * C] += (yf * yf).sum(0)


def conv_forward(x, w, y, shp: ConvShape, ws=None, stats=None, wp=None, xp=None) -> None:
    """y = conv(x, w); ``stats`` (fp64 [2*Cout]) accumulates the per-channel
    sum / sum-of-squares of the bf16 output for the following BatchNorm.
    ``wp`` / ``xp``: the packed bf16x3 mirrors (int32) of ``w`` / ``x`` (fp32 /
    bf16x3 mode; packed on the fly when omitted)."""
    if x.is_cuda:
        if x.dtype == torch.float32:
            ops().conv32_forward(x if xp is None else xp, w, y, ws, stats, *shp.args(), wp)
        else:
            ops().conv_forward(x, w, y, ws, stats, *shp.args())
        return
    out = F.conv2d(_nchw(x), _wt(w), stride=shp.stride, padding=shp.pad)
    y.copy_(out.permute(0, 2, 3, 1).to(y.dtype))
    if stats is not None:
        _acc_stats_cpu(y, stats)


@dataclass
class BnBwdTarget:
    """The BatchNorm whose upstream gradient a dgrad produces: the dgrad
    epilogue adds that BN-backward's reductions (sum g, sum g*xhat;
    g = dx * [y > 0]) into ``acc`` while writing dx, so the BN backward runs
    with ``presummed=True`` (one launch fewer per layer)."""
    z: torch.Tensor
    y: torch.Tensor | None
    mean: torch.Tensor
    invstd: torch.Tensor
    acc: torch.Tensor


def _bnb_sums_cpu(dx: torch.Tensor, t: BnBwdTarget, store_masked: bool = True) -> None:
    C = dx.shape[-1]
    g = dx.float().reshape(-1, C)
    if t.y is not None:
        g = torch.where(t.y.float().reshape(-1, C) > 0, g, torch.zeros_like(g))
        if store_masked:  # as the GPU dgrad epilogues: dX is stored masked
            dx.copy_(g.view(dx.shape).to(dx.dtype))
    xh = (t.z.float().reshape(-1, C) - t.mean) * t.invstd
    t.acc[:C] += g.double().sum(0)
    t.acc[C:2 * C] += (g.double() * xh.double()).sum(0)


def _dy_arg(dy, dy_packed: bool):
    """``dy_packed``: the fp32 buffer holds packed bf16x3 splits (written by
    :func:`bn_backward` with ``dx_packed``); the binding takes it as int32."""
    return dy.view(torch.int32) if dy_packed else dy


def conv_dgrad(dy, w, dx, shp: ConvShape, ws=None, accumulate: bool = False,
               bnb: BnBwdTarget | None = None, wp=None, dy_packed: bool = False) -> None:
    """dx (+)= conv_transpose(dy, W); ``w`` is the KRSC weight [Cout][R][S][Cin]
    (the kernel forms W^T fragments with transposing LDS reads).  ``bnb``:
    fuse the consumer BatchNorm-backward reductions into the epilogue."""
    if dy.is_cuda:
        f32 = dy.dtype == torch.float32
        fn = ops().conv32_dgrad if f32 else ops().conv_dgrad
        extra = (wp,) if f32 else ()
        if f32:
            dy = _dy_arg(dy, dy_packed)
        if bnb is None:
            fn(dy, w, dx, ws, *shp.args(), accumulate, None, None, None, None, None, *extra)
        else:
            fn(dy, w, dx, ws, *shp.args(), accumulate, bnb.z, bnb.y, bnb.mean, bnb.invstd, bnb.acc, *extra)
        return
    _conv_dgrad_cpu(dy, w, dx, shp, accumulate)
    if bnb is not None:
        _bnb_sums_cpu(dx, bnb)


def _conv_dgrad_cpu(dy, w, dx, shp: ConvShape, accumulate: bool) -> None:
    w = w.float().permute(0, 3, 1, 2)  # -> [Cout][Cin][R][S]
    g = torch.nn.grad.conv2d_input((shp.N, shp.C, shp.H, shp.W), w, _nchw(dy),
                                   stride=shp.stride, padding=shp.pad)
    g = g.permute(0, 2, 3, 1)
    if accumulate:
        g = g + dx.float()
    dx.copy_(g.to(dx.dtype))


def conv_wgrad(x, dy, dw, shp: ConvShape, accumulate: bool = False, dy_packed: bool = False,
               xp=None) -> None:
    """dw (fp32 [Cout][R][S][Cin]) = sum over pixels of dy x im2col(x).
    accumulate=True promises dw is already zero (split-K slices add into it)."""
    if x.is_cuda:
        if x.dtype == torch.float32:
            ops().conv32_wgrad(x if xp is None else xp, _dy_arg(dy, dy_packed), dw, *shp.args(), accumulate)
        else:
            ops().conv_wgrad(x, dy, dw, *shp.args(), accumulate)
        return
    # contiguous NCHW: torch's CPU weight-gradient kernel corrupts the heap on
    # channels-last views for strided 1x1 convs with few channels (observed
    # with torch 2.10: N=4, C=8 -> 16, 1x1 stride 2)
    g = torch.nn.grad.conv2d_weight(_nchw(x).contiguous(), (shp.Co, shp.C, shp.R, shp.S),
                                    _nchw(dy).contiguous(), stride=shp.stride, padding=shp.pad)
    dw.copy_(g.permute(0, 2, 3, 1).reshape(dw.shape))


def conv_forward_pair(x, w1, y1, ws1, stats1, w2, y2, ws2, stats2, shp: ConvShape, wp1=None, wp2=None,
                      xp=None) -> None:
    """A downsampling block's conv1 (3x3, stride 2; ``shp``) and its 1x1 / stride-2
    projection shortcut of the same x -- one paired launch on the GPU."""
    assert shp.R == 3 and shp.stride == 2
    if x.is_cuda:
        if x.dtype == torch.float32:
            ops().conv32_forward_pair(x if xp is None else xp, w1, y1, ws1, stats1, w2, y2, ws2, stats2,
                                      shp.N, shp.H, shp.W, shp.C, shp.Co, wp1, wp2)
        else:
            ops().conv_forward_pair(x, w1, y1, ws1, stats1, w2, y2, ws2, stats2, shp.N, shp.H, shp.W, shp.C, shp.Co)
        return
    conv_forward(x, w1, y1, shp, ws1, stats1)
    conv_forward(x, w2, y2, ConvShape(shp.N, shp.H, shp.W, shp.C, shp.Co, 1, 1, 2, 0), ws2, stats2)


def conv_backward_pair(x, dy, dw, w, dx, shp: ConvShape, ws=None, accumulate: bool = False,
                       bnb: BnBwdTarget | None = None, wp=None, dy_packed: bool = False, xp=None,
                       opt=None) -> None:
    """A layer's weight gradient (dw += ..., dw zero on entry) and input
    gradient (as conv_dgrad) -- on the GPU in ONE paired launch, so the two
    independent, latency-bound GEMMs share the CUs (conv.hip
    conv_bwd_pair_kernel; MFL_CONV_PAIR=0 for two launches).  fp32: one
    launch too (conv32.hip conv32_bwd_pair_kernel, when both plans run 64x64
    tiles on the fast address paths; MFL_C32_PAIR=0 for two launches).
    ``opt`` (ops.optim.OptRange): an optimizer step over a range whose
    gradients are final, run by extra workgroups of the fp32 paired launch
    (elsewhere: its own launch after the pair)."""
    if dy.is_cuda and dy.dtype == torch.float32:
        dy = _dy_arg(dy, dy_packed)
        xa = x if xp is None else xp
        from metisfl_amd.ops.optim import NO_OPT_TAIL
        tail = opt.binding_args() if opt is not None else NO_OPT_TAIL
        if bnb is None:
            ops().conv32_backward_pair(xa, dy, dw, w, dx, ws, *shp.args(), accumulate, None, None, None, None, None,
                                       wp, *tail)
        else:
            ops().conv32_backward_pair(xa, dy, dw, w, dx, ws, *shp.args(), accumulate, bnb.z, bnb.y, bnb.mean,
                                       bnb.invstd, bnb.acc, wp, *tail)
        return
    if not _conv_backward_pair_unfused(x, dy, dw, w, dx, shp, ws, accumulate, bnb, wp, opt) and opt is not None:
        opt.run()


def _conv_backward_pair_unfused(x, dy, dw, w, dx, shp, ws, accumulate, bnb, wp, opt=None) -> bool:
    """-> whether ``opt`` (an optimizer tail) was taken by the launch."""
    if dy.is_cuda:
        from metisfl_amd.ops.optim import NO_OPT_TAIL
        tail = opt.binding_args() if opt is not None else NO_OPT_TAIL
        if bnb is None:
            ops().conv_backward_pair(x, dy, dw, w, dx, ws, *shp.args(), accumulate, None, None, None, None,
                                     None, *tail)
        else:
            ops().conv_backward_pair(x, dy, dw, w, dx, ws, *shp.args(), accumulate, bnb.z, bnb.y, bnb.mean,
                                     bnb.invstd, bnb.acc, *tail)
        return True
    conv_wgrad(x, dy, dw, shp, accumulate=True)
    conv_dgrad(dy, w, dx, shp, ws, accumulate, bnb=bnb, wp=wp)
    return False


def transpose_krsc(w, wt, Co: int, RS: int, Ci: int) -> None:
    if w.is_cuda:
        ops().transpose_krsc(w, wt, Co, RS, Ci)
        return
    wt.copy_(w.reshape(Co, RS, Ci).permute(2, 1, 0).reshape(wt.shape))


# ---------------------------------------------------------------------------
# Halo-tiled convolution with the producer's BatchNorm fused into the operand
# fill (hconv.hip; fp32 activations, bf16x3 products)
@dataclass
class BnParams:
    """One BatchNorm's parameters and statistics buffers: ``acc`` holds the
    fp64 sums of its input [reps][2][C] (train); ``mean`` / ``invstd`` are
    published and the running averages updated by the launch that applies it."""
    acc: torch.Tensor | None
    gamma: torch.Tensor
    beta: torch.Tensor
    mean: torch.Tensor
    invstd: torch.Tensor
    run_mean: torch.Tensor
    run_var: torch.Tensor
    momentum: float = 0.1
    eps: float = 1e-5


def hconv_workspace(shp: ConvShape, device: torch.device) -> int:
    """Split-K workspace floats of the halo conv for ``shp``, or -1 when the
    geometry is not covered (3x3 / stride 1 CIFAR-ResNet stages)."""
    if shp.R != 3 or shp.stride != 1 or shp.pad != 1 or shp.C != shp.Co:
        return -1
    if device.type == "cuda":
        return int(ops().hconv_fwd_workspace(shp.N, shp.H, shp.W, shp.C, shp.Co))
    ok = (shp.H == shp.W and (shp.H, shp.C) in ((32, 64), (16, 128), (8, 256), (4, 512))
          and shp.N % {32: 1, 16: 1, 8: 2, 4: 8}[shp.H] == 0)
    return 0 if ok else -1


def hconv_forward(z, wp, w, out, shp: ConvShape, bn: BnParams, train: bool, relu: bool, ws=None, stats=None,
                  res=None, zr=None, bnr: BnParams | None = None, y=None, yp=None, stamps=None) -> None:
    """out = conv3x3(T(z), w) with T(z) = relu?(BN(z) [+ res | + BN_r(zr)]) applied
    as the operand enters LDS (one launch: no separate BatchNorm apply).
    ``y`` / ``yp`` receive T(z) and its packed bf16x3 split (the activation
    the backward pass and later residual adds read); ``stats`` accumulates the
    output's BN sums (train).  Publishes ``bn`` (and ``bnr``) in train mode.
    ``wp``: the packed weight mirror (GPU), ``w``: the fp32 weights (CPU)."""
    C = shp.C
    if z.is_cuda:
        b2 = bnr if bnr is not None else None
        # bf16 option: the bf16 weights themselves (no packed mirror)
        ops().hconv_forward(z, wp if wp is not None else w, out, ws, stats, shp.N, shp.H, shp.W, C, shp.Co, train, relu,
                            bn.acc if train else None, bn.gamma, bn.beta, bn.mean, bn.invstd, bn.run_mean,
                            bn.run_var, bn.momentum, bn.eps, res, zr,
                            (b2.acc if train else None) if b2 else None, b2.gamma if b2 else None,
                            b2.beta if b2 else None, b2.mean if b2 else None, b2.invstd if b2 else None,
                            b2.run_mean if b2 else None, b2.run_var if b2 else None, y, yp, stamps)
        return
    # reference: the BatchNorm apply(s) the fill replaces, then the conv
    r = res
    if zr is not None:
        r = torch.empty_like(zr)
        bn_apply(zr, C, bnr.acc, bnr.gamma, bnr.beta, bnr.mean, bnr.invstd, bnr.run_mean, bnr.run_var, r,
                 relu=False, train=train, momentum=bnr.momentum, eps=bnr.eps)
    v = y if y is not None else torch.empty_like(z)
    bn_apply(z, C, bn.acc, bn.gamma, bn.beta, bn.mean, bn.invstd, bn.run_mean, bn.run_var, v, residual=r,
             relu=relu, train=train, momentum=bn.momentum, eps=bn.eps)
    conv_forward(v, w, out, shp, stats=stats)


def hconv_dgrad(dy, ymask, z, wp, w, out, shp: ConvShape, bn: BnParams, dgamma=None, dbeta=None, ws=None,
                dres=None, dzp=None, accumulate: bool = False, bnb: BnBwdTarget | None = None,
                stamps=None) -> None:
    """out (+)= conv3x3^T(dz, w) with dz = BN_backward(g), g = dy [* (ymask > 0)],
    applied as the operand enters LDS (one launch: no separate BatchNorm
    backward apply).  ``bn.acc`` holds the complete sums of g and g * xhat
    (the producer of dy accumulated them); dgamma / dbeta are published.
    ``dzp`` receives dz's packed bf16x3 split (the layer's wgrad operand),
    ``dres`` g (the residual branch's gradient).  ``bnb``: the consumer
    BatchNorm-backward reductions of ``out`` (as conv_dgrad)."""
    C = shp.Co  # dz channels (the layer's output): the reduction
    if dy.is_cuda:
        ops().hconv_dgrad(dy, ymask, z, wp, out, ws, shp.N, shp.H, shp.W, C, shp.C, bn.acc, bn.gamma, bn.mean,
                          bn.invstd, dgamma, dbeta, dres, dzp, accumulate,
                          bnb.z if bnb else None, bnb.y if bnb else None, bnb.mean if bnb else None,
                          bnb.invstd if bnb else None, bnb.acc if bnb else None, stamps)
        return
    # reference: the BatchNorm backward the fill replaces, then the dgrad
    dz = torch.empty_like(z)
    bn_backward(dy, z, ymask, C, bn.gamma, bn.mean, bn.invstd, bn.acc, dgamma, dbeta, dz, dy_masked=dres,
                presummed=True)
    if dzp is not None:
        dzp.copy_(dz)
    conv_dgrad(dz, w, out, shp, accumulate=accumulate, bnb=bnb)


def bn_stats(x, C: int, acc) -> None:
    """acc[0:C] += sum x, acc[C:2C] += sum x^2 (fp64) over the rows of NHWC x."""
    if x.is_cuda:
        (ops().bn32_stats if x.dtype == torch.float32 else ops().bn_stats)(x, C, acc)
        return
    _acc_stats_cpu(x, acc)


def bn_apply(x, C: int, acc, gamma, beta, mean, invstd, run_mean, run_var, y, residual=None,
             relu: bool = False, train: bool = True, momentum: float = 0.1,
             eps: float = 1e-5, yp=None) -> None:
    """y = relu?(BN(x) + residual).  train: batch statistics from ``acc`` (sums
    over the M rows), publishes mean/invstd, updates running stats; eval:
    running statistics.  ``yp`` (fp32 GPU path): also write y's packed bf16x3
    split (int32) -- the operand the next convolutions read."""
    if x.is_cuda:
        if x.dtype == torch.float32:
            ops().bn32_apply(x, C, acc, gamma, beta, mean, invstd, run_mean, run_var, residual, y, relu, train,
                             momentum, eps, yp)
        else:
            ops().bn_apply(x, C, acc, gamma, beta, mean, invstd, run_mean, run_var, residual, y, relu, train,
                           momentum, eps)
        return
    M = x.numel() // C
    if train:
        tot = _acc_total(acc, C)
        mu = tot[:C] / M
        var = (tot[C:2 * C] / M - mu * mu).clamp_min(0)
        mean.copy_(mu.float())
        invstd.copy_((1.0 / torch.sqrt(var + eps)).float())
        unb = var * M / (M - 1) if M > 1 else var
        run_mean.mul_(1 - momentum).add_(momentum * mu.float())
        run_var.mul_(1 - momentum).add_(momentum * unb.float())
        istd = (1.0 / torch.sqrt(var + eps)).float()
        mu = mu.float()
    else:
        mu = run_mean
        istd = 1.0 / torch.sqrt(run_var.double() + eps).float()
    scale = gamma * istd
    shift = beta - mu * scale
    v = x.float() * scale + shift
    if residual is not None:
        v = v + residual.float()
    if relu:
        v = v.clamp_min(0)
    y.copy_(v.to(y.dtype))


@dataclass
class BnSide:
    """A second BatchNorm whose upstream gradient is ``dy_masked`` (a
    downsampling block's projection shortcut): its backward sums are added
    into ``acc`` by the same launch (fp32 GPU path; C / 4 must divide 256)."""
    z: torch.Tensor
    mean: torch.Tensor
    invstd: torch.Tensor
    acc: torch.Tensor


def bn_backward(dy, x, y, C: int, gamma, mean, invstd, acc, dgamma, dbeta, dx,
                dy_masked=None, presummed: bool = False, side: BnSide | None = None,
                dx_packed: bool = False) -> None:
    """BN(+ReLU) backward.  ``y`` (the post-activation output) gives the ReLU
    mask; ``dy_masked`` optionally receives the masked upstream gradient (the
    residual-shortcut gradient of an add+ReLU).  ``acc`` (fp64 [2C]) must be
    zero on entry.  ``dx_packed`` (fp32 GPU path, bf16x3 conv products): dx
    receives the packed (hi << 16 | lo) bf16 split of the gradient instead of
    fp32 -- the dY operand encoding of the layer's dgrad / wgrad kernels, which
    then decode it with two v_perm per pair instead of splitting it per k-tile."""
    if dy.is_cuda:
        if dx_packed:
            assert dy.dtype == torch.float32, "packed dx is an fp32-path encoding"
            dx = dx.view(torch.int32)
        if side is not None:
            ops().bn32_backward_side(dy, x, y, C, gamma, mean, invstd, acc, dgamma, dbeta, dx, dy_masked, presummed,
                                     side.z, side.mean, side.invstd, side.acc)
            return
        fn = ops().bn32_backward if dy.dtype == torch.float32 else ops().bn_backward
        fn(dy, x, y, C, gamma, mean, invstd, acc, dgamma, dbeta, dx, dy_masked, presummed)
        return
    g = dy.float()
    if y is not None:
        g = torch.where(y.float() > 0, g, torch.zeros_like(g))
    if dy_masked is not None:  # (y None: dy arrives masked)
        dy_masked.copy_(g.to(dy_masked.dtype))
    if side is not None:
        gs = g.reshape(-1, C).double()
        xs = ((side.z.float() - side.mean) * side.invstd).reshape(-1, C).double()
        side.acc[:C] += gs.sum(0)
        side.acc[C:2 * C] += (gs * xs).sum(0)
    xf = x.float()
    xh = (xf - mean) * invstd
    gm = g.reshape(-1, C)
    M = gm.shape[0]
    if not presummed:  # else the producer of dy already added the sums
        acc[:C] += gm.double().sum(0)
        acc[C:2 * C] += (gm.double() * xh.reshape(-1, C).double()).sum(0)
    tot = _acc_total(acc, C)
    if dgamma is not None:
        dgamma.copy_(tot[C:2 * C].float())
    if dbeta is not None:
        dbeta.copy_(tot[:C].float())
    k1 = gamma * invstd
    out = k1 * (g - (tot[:C] / M).float() - xh * (tot[C:2 * C] / M).float())
    dx.copy_(out.to(dx.dtype))


def bn_backward_pair(a1: tuple, a2: tuple, dx_packed: bool = False) -> None:
    """Two presummed BN(+ReLU) backward applies in one launch on the GPU
    (bn32.hip bn32_bwd_apply_pair_kernel): ``a1`` / ``a2`` are
    (dy, z, relu mask y or None, C, gamma, mean, invstd, acc, dgamma, dbeta,
    dz) of a downsampling block's conv1 (with its ReLU mask) and projection
    shortcut (without); their sums must already be complete in ``acc``."""
    (dy1, x1, y1, C1, g1, m1, i1, acc1, dg1, db1, dx1) = a1
    (dy2, x2, y2, C2, g2, m2, i2, acc2, dg2, db2, dx2) = a2
    if dy1.is_cuda and dy1.dtype == torch.float32 and y2 is None:
        if dx_packed:
            dx1, dx2 = dx1.view(torch.int32), dx2.view(torch.int32)
        ops().bn32_backward_pair(dy1, x1, y1, C1, g1, m1, i1, acc1, dg1, db1, dx1,
                                 dy2, x2, C2, g2, m2, i2, acc2, dg2, db2, dx2)
        return
    bn_backward(dy1, x1, y1, C1, g1, m1, i1, acc1, dg1, db1, dx1, presummed=True, dx_packed=dx_packed)
    bn_backward(dy2, x2, y2, C2, g2, m2, i2, acc2, dg2, db2, dx2, presummed=True, dx_packed=dx_packed)


def stem_backward_ok(shp: ConvShape, device: torch.device) -> bool:
    """Whether the fused stem backward (:func:`stem_backward`) covers ``shp``
    (the CIFAR stem: 3x3 / stride 1 / pad 1, 8 padded input channels, 64
    outputs, 32x32 images)."""
    geo = shp.R == 3 and shp.S == 3 and shp.stride == 1 and shp.pad == 1
    if device.type == "cuda":
        return geo and bool(ops().stem_backward32_ok(shp.N, shp.H, shp.W, shp.C, shp.Co))
    return geo and shp.H == 32 and shp.W == 32 and shp.C == 8 and shp.Co == 64


def stem_backward(dy, z, y, x, shp: ConvShape, gamma, mean, invstd, acc, dgamma, dbeta, dw, opt=None) -> None:
    """A conv without dgrad (the stem): its BN(+ReLU) backward and its weight
    gradient in ONE launch on the GPU (bn32.hip stem_bwd32_kernel; dz never
    reaches memory, products are exact fp32).  ``acc`` holds the complete
    backward sums (presummed); ``dw`` (zero on entry) accumulates.  ``opt``
    (ops.optim.OptRange): an optimizer step riding in the same launch."""
    if dy.is_cuda:
        from metisfl_amd.ops.optim import NO_OPT_TAIL
        tail = opt.binding_args() if opt is not None else NO_OPT_TAIL
        ops().stem_backward32(dy, z, y, gamma, mean, invstd, acc, dgamma, dbeta, x, dw, *tail)
        return
    # reference: the BatchNorm backward apply, then the weight gradient
    dz = torch.empty_like(z)
    bn_backward(dy, z, y, shp.Co, gamma, mean, invstd, acc, dgamma, dbeta, dz, presummed=True)
    g = torch.empty_like(dw)
    conv_wgrad(x, dz, g, shp)
    dw.add_(g)
    if opt is not None:
        opt.run()


# ---------------------------------------------------------------------------
def head_forward_backward(x, B: int, HW: int, C: int, W, bias, labels, feat, dlogits, dx, stats,
                          backward: bool = True, dW=None, db=None) -> None:
    """avgpool -> linear -> softmax-CE (+ backward to the pooled input).
    stats[0:3] += (loss sum, #correct, #samples).  With ``dW`` (and ``db``)
    the weight / bias gradients are ADDED in the same launch (fused
    head_wgrad; the buffers must hold zeros or a running sum)."""
    if x.is_cuda:
        fn = ops().head32_forward_backward if x.dtype == torch.float32 else ops().head_forward_backward
        fn(x, B, HW, C, W, bias, labels, feat, dlogits, dx, stats, backward, dW, db)
        return
    xf = x.float().reshape(B, HW, C)
    f = xf.mean(1)
    K = W.numel() // C
    logits = f @ W.reshape(K, C).t() + (bias if bias is not None else 0)
    lab = labels[:B].long()
    lse = torch.logsumexp(logits, 1)
    if stats is not None:
        ok = lab >= 0  # label -1: an evaluation padding row (not counted)
        lv = lab.clamp_min(0)
        stats[0] += torch.where(ok, lse - logits.gather(1, lv[:, None])[:, 0], torch.zeros(())).sum()
        stats[1] += ((logits.argmax(1) == lab) & ok).float().sum()
        stats[2] += ok.float().sum()
    if not backward:
        return
    p = torch.softmax(logits, 1)
    d = p.clone()
    d[torch.arange(B), lab] -= 1
    d /= B
    feat.view(-1)[: B * C].copy_(f.reshape(-1))
    dlogits.view(-1)[: B * K].copy_(d.reshape(-1))
    dfeat = d @ W.reshape(K, C)
    dx.copy_((dfeat / HW)[:, None, :].expand(B, HW, C).reshape(dx.shape).to(dx.dtype))
    if dW is not None:
        dW.add_((d.t() @ f).reshape(dW.shape))
        if db is not None:
            db.add_(d.sum(0))


def head_forward_backward_bn(B: int, HW: int, C: int, W, bias, labels, feat, dlogits, dx, stats,
                             backward: bool, dW, db, z, res, bn: BnParams, train: bool, y, acc_b=None) -> None:
    """head_forward_backward of y = relu(BN(z) + res) with the BatchNorm apply
    folded into the head's pooling loop (y is written: the backward's ReLU
    mask) and, when ``acc_b`` is given (train, backward), the BN-backward sums
    of dx (sum g, sum g * xhat; g = dx * [y > 0]) added into it -- that BN's
    backward then runs presummed (no reduce launch)."""
    if z.is_cuda:
        ops().head32_forward_backward_bn(B, HW, C, W, bias, labels, feat, dlogits, dx, stats, backward, dW, db,
                                         z, res, bn.acc if train else None, bn.gamma, bn.beta, bn.mean, bn.invstd,
                                         bn.run_mean, bn.run_var, bn.momentum, bn.eps, train, y, acc_b)
        return
    # reference: the BatchNorm apply, the head, the BN-backward reduction
    bn_apply(z, C, bn.acc, bn.gamma, bn.beta, bn.mean, bn.invstd, bn.run_mean, bn.run_var, y, residual=res,
             relu=True, train=train, momentum=bn.momentum, eps=bn.eps)
    head_forward_backward(y, B, HW, C, W, bias, labels, feat, dlogits, dx, stats, backward, dW, db)
    if backward and acc_b is not None:
        _bnb_sums_cpu(dx, BnBwdTarget(z, y, bn.mean, bn.invstd, acc_b[:2 * C]), store_masked=False)


def head_wgrad(feat, dlogits, B: int, C: int, K: int, dW, db) -> None:
    if feat.is_cuda:
        ops().head_wgrad(feat, dlogits, B, C, K, dW, db)
        return
    f = feat.view(-1)[: B * C].view(B, C)
    d = dlogits.view(-1)[: B * K].view(B, K)
    dW.copy_((d.t() @ f).reshape(dW.shape))
    if db is not None:
        db.copy_(d.sum(0))


def gather_batch(shard, labels, perm, step, steps_per_epoch: int, B: int, xb, yb, xp=None) -> None:
    """xb / yb <- the step's mini-batch.  ``xp`` (fp32 shards on the GPU): also
    write the batch's packed bf16x3 split (int32), the stem conv's operand."""
    if shard.is_cuda:
        if shard.dtype == torch.float32:
            ops().gather_batch32(shard, labels, perm, step, steps_per_epoch, B, xb, yb, xp)
        else:
            ops().gather_batch(shard, labels, perm, step, steps_per_epoch, B, xb, yb)
        return
    if xp is not None:
        raise ValueError("packed input batches exist on the fp32 GPU path only")
    s = int(step[0]) % steps_per_epoch
    idx = perm[s * B:(s + 1) * B].long()
    xb.copy_(shard.view(labels.numel(), -1)[idx].reshape(xb.shape))
    yb[:B].copy_(labels[idx])


def gemm_nt(a, b, c, M: int, N: int, K: int, bias=None, epilogue: int = 0, aux=None) -> None:
    """c = a . b^T (+bias, +exact-erf gelu | +residual)."""
    if a.is_cuda:
        ops().gemm_nt(a, b, c, bias, M, N, K, epilogue, aux)
        return
    out = a.float().reshape(M, K) @ b.float().reshape(N, K).t()
    if epilogue >= 1 and bias is not None:
        out = out + bias
    if epilogue == 2:  # gelu of the bf16-rounded pre-activation, as on the GPU
        out = F.gelu(out.to(torch.bfloat16).float())
    if epilogue == 3:
        out = out + aux.float().reshape(M, N)
    c.copy_(out.reshape(c.shape).to(torch.bfloat16))


# ---------------------------------------------------------------------------
# example-model layers (layers.hip)
ACT_NONE, ACT_RELU = 0, 1


def bias_act(y, bias, N: int, act: int) -> None:
    """y = act(y + bias) in place (bf16 [M][N], fp32 bias)."""
    if y.is_cuda:
        ops().bias_act(y, bias, N, act)
        return
    v = y.float().reshape(-1, N) + bias[:N]
    if act == ACT_RELU:
        v = v.clamp_min(0)
    y.copy_(v.reshape(y.shape).to(torch.bfloat16))


def bias_act_backward(dy, y, dz, dbias, N: int, act: int) -> None:
    """dz = dy * act'(y); dbias += column sums of dz (dbias zero on entry)."""
    if dy.is_cuda:
        ops().bias_act_backward(dy, y, dz, dbias, N, act)
        return
    g = dy.float().reshape(-1, N)
    if act == ACT_RELU:
        g = torch.where(y.float().reshape(-1, N) > 0, g, torch.zeros_like(g))
    g16 = g.to(torch.bfloat16)
    dz.copy_(g16.reshape(dz.shape))
    dbias[:N] += g16.float().sum(0)


def maxpool2(x, y, N: int, H: int, W: int, C: int) -> None:
    if x.is_cuda:
        ops().maxpool2(x, y, N, H, W, C)
        return
    v = x.float().reshape(N, H // 2, 2, W // 2, 2, C).amax(dim=(2, 4))
    y.copy_(v.reshape(y.shape).to(torch.bfloat16))


def maxpool2_backward(dy, x, y, dx, N: int, H: int, W: int, C: int) -> None:
    if dy.is_cuda:
        ops().maxpool2_backward(dy, x, y, dx, N, H, W, C)
        return
    xv = x.float().reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, C, 4)
    m = y.float().reshape(N, H // 2, W // 2, C, 1)
    hit = xv == m
    first = hit & (hit.long().cumsum(-1) == 1)  # first maximal element of each window
    g = first.float() * dy.float().reshape(N, H // 2, W // 2, C, 1)
    g = g.reshape(N, H // 2, W // 2, C, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(N, H, W, C)
    dx.copy_(g.to(torch.bfloat16))


def _keep_mask_cpu(n: int, p: float, seed: int, step: int) -> torch.Tensor:
    """Same hash as the HIP dropout kernel (lowbias32), on the host."""
    M32 = 0xFFFFFFFF

    def mix(x):
        x = x ^ (x >> 16)
        x = (x * 0x7FEB352D) & M32
        x = x ^ (x >> 15)
        x = (x * 0x846CA68B) & M32
        return x ^ (x >> 16)

    idx = torch.arange(n, dtype=torch.int64)
    inner = ((step * 0x9E3779B9) & M32) ^ (idx & M32) ^ (((idx >> 32) * 0x85EBCA6B) & M32)
    h = mix(seed ^ mix(inner))
    thresh = min(int(p * 4294967296.0), M32)
    return h >= thresh


def dropout(inp, out, p: float, seed: int, step=None) -> None:
    """Inverted dropout; the mask is a hash of (seed, device step, index), so
    the backward pass (same call on dy) applies the identical mask."""
    if inp.is_cuda:
        ops().dropout(inp, out, p, seed, step)
        return
    st = int(step[0]) if step is not None else 0
    keep = _keep_mask_cpu(inp.numel(), p, seed & 0xFFFFFFFF, st).reshape(inp.shape)
    scale = 1.0 / (1.0 - p) if p < 1 else 0.0
    out.copy_(torch.where(keep, inp.float() * scale, torch.zeros(())).to(torch.bfloat16))


def xent(logits, labels, B: int, Kp: int, K: int, dlogits, stats) -> None:
    """Softmax cross-entropy over the first K of Kp logit columns; dlogits =
    (softmax - onehot)/B (None: forward only); stats += (loss, correct, n)."""
    if logits.is_cuda:
        ops().xent(logits, labels, B, Kp, K, dlogits, stats)
        return
    z = logits.float().reshape(B, Kp)[:, :K]
    y = labels[:B].long()
    lse = torch.logsumexp(z, 1)
    ok = y >= 0  # label -1: an evaluation padding row
    yv = y.clamp_min(0)
    stats[0] += float(torch.where(ok, lse - z.gather(1, yv[:, None])[:, 0], torch.zeros(())).sum())
    stats[1] += float(((z.argmax(1) == y) & ok).sum())
    stats[2] += float(ok.sum())
    if dlogits is not None:
        g = torch.zeros(B, Kp)
        g[:, :K] = (torch.softmax(z, 1) - F.one_hot(y, K).float()) / B
        dlogits.copy_(g.reshape(dlogits.shape).to(torch.bfloat16))


def mse(pred, target, B: int, Kp: int, dpred, stats) -> None:
    """Squared error on column 0 (fp32 targets); dpred = 2 (pred - t) / B."""
    if pred.is_cuda:
        ops().mse(pred, target, B, Kp, dpred, stats)
        return
    t = target[:B].view(torch.float32) if target.dtype == torch.int32 else target[:B].float()
    d = pred.float().reshape(B, Kp)[:, 0] - t
    ok = ~torch.isnan(t)  # the -1 label bits of an evaluation padding row
    stats[0] += float(torch.where(ok, d * d, torch.zeros(())).sum())
    stats[2] += float(ok.sum())
    if dpred is not None:
        g = torch.zeros(B, Kp)
        g[:, 0] = 2 * d / B
        dpred.copy_(g.reshape(dpred.shape).to(torch.bfloat16))
