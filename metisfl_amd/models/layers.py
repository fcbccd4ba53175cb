"""Static-graph layers for the learner's local training step.

A model is a fixed sequence of layers with a fixed batch size, so every
activation, gradient and workspace buffer is planned once (memory is sized
for 288 GB of HBM per learner -- nothing is allocated per step) and the whole
step -- batch gather, forward, loss, backward, optimizer -- is a pure
sequence of kernel launches on one HIP stream that is captured into a
hipGraph (see models/net.py).  There is no autograd tape: each layer owns its
backward and writes weight gradients straight into the flat fp32 gradient
buffer (models/flat.py), so there is no gradient accumulation pass and no
per-parameter launch.

These layers replace the Keras layers the reference trains with
(examples/keras/models/cifar_cnn.py, fashion_mnist_fc.py).
"""
from __future__ import annotations

import os

import torch

from metisfl_amd.models.flat import FlatState, VarSpec
from metisfl_amd.ops import nn as K
from metisfl_amd.ops.nn import ConvShape


class OptTailScheduler:
    """Optimizer tails for one training step (see ops.optim.OptRange,
    conv32.h OptTail).  The flat buffer holds the trainable variables in
    layer order and the backward finishes them from the end, so the
    gradients of [ready, n) are final once the layers from ``ready`` on have
    run their backward.  Every fp32 paired backward launch after that takes
    the next chunk (at most ``chunk`` parameters, from the top down) of the
    final-but-not-updated range [ready, done) as extra workgroups of its own
    launch; the step's last optimizer launch updates only [0, done).
    MFL_OPT_TAIL = parameters per launch (0: off; default 512K)."""

    # measured (profiles/r4/step/{c,d,e}_t*.log): 512K parameters per launch
    # -1.0..-1.3 % per update for one learner, -2 % for two co-located
    chunk = int(os.environ.get("MFL_OPT_TAIL", "524288"))
    ALIGN = 64  # flat segments start at multiples of 64 elements (models/flat.py)

    def __init__(self, st: FlatState, zero_grad: bool):
        self.st = st
        self.zero_grad = zero_grad
        self.ready = st.n_params
        self.done = st.n_params

    def mark_ready(self, lo: int) -> None:
        """Gradients of every trainable variable from offset ``lo`` on are final."""
        assert lo % self.ALIGN == 0
        self.ready = min(self.ready, lo)

    def take(self, everything: bool = False):
        """The next tail (an OptRange) or None; ``everything``: all of the
        final-but-not-updated range at once (the step's last backward launch)."""
        if self.chunk <= 0 or self.done <= self.ready:
            return None
        lo = self.ready if everything else max(self.ready, (self.done - self.chunk) // self.ALIGN * self.ALIGN)
        r = self.st.opt_range(lo, self.done, self.zero_grad)
        self.done = lo
        return r


class Workspace:
    """Shared scratch: the split-K fp32 slab (kernels on one stream run in
    order, so one buffer of the maximum size serves every layer) and the
    model-wide fp64 BatchNorm accumulator buffer, carved per layer.  The
    accumulators are re-zeroed by the optimizer launch at the end of a step."""

    def __init__(self, dtype: torch.dtype = torch.bfloat16):
        self.dtype = dtype  # activation / compute dtype of the model
        self.split_floats = 0
        self.split: torch.Tensor | None = None
        self.acc_len = 0
        self.bn_acc: torch.Tensor | None = None
        self.opt_tails: OptTailScheduler | None = None  # set for the duration of a training step

    def take_opt_tail(self, everything: bool = False):
        return self.opt_tails.take(everything) if self.opt_tails is not None else None

    def need_split(self, n: int) -> None:
        self.split_floats = max(self.split_floats, n)

    def take_acc(self, n: int) -> tuple[int, int]:
        off = self.acc_len
        self.acc_len += (n + 1) // 2 * 2  # keep 16-B alignment of every slice
        return (off, n)

    def acc(self, sl: tuple[int, int]) -> torch.Tensor:
        return self.bn_acc[sl[0]: sl[0] + sl[1]]

    def allocate(self, device) -> None:
        self.split = torch.zeros(max(4, self.split_floats), dtype=torch.float32, device=device)
        self.split2 = torch.zeros(max(4, self.split_floats), dtype=torch.float32, device=device)
        self.bn_acc = torch.zeros(max(2, self.acc_len), dtype=torch.float64, device=device)
        # Side stream for work that is off the critical path (weight gradients,
        # projection shortcuts).  Forked/joined with stream waits, so inside a
        # captured hipGraph these become parallel branches that fill CUs the
        # small CIFAR-sized kernels leave idle.
        dev = torch.device(device)
        self.side = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None

    # Measured on MI355X (round 1): forking wgrad / shortcuts onto a second
    # stream inside the graph made the ResNet-18 step ~12% SLOWER (the branches
    # contend for CUs and add cross-stream waits), so it is opt-in
    # (MFL_OVERLAP=1).
    overlap = os.environ.get("MFL_OVERLAP", "0") == "1"

    def fork(self):
        """Context: run the enclosed launches on the side stream, ordered after
        everything already issued on the current stream."""
        import contextlib
        if self.side is None or not self.overlap:
            return contextlib.nullcontext()
        self.side.wait_stream(torch.cuda.current_stream(self.side.device))
        return torch.cuda.stream(self.side)

    def join(self) -> None:
        if self.side is not None and self.overlap:
            torch.cuda.current_stream(self.side.device).wait_stream(self.side)


# Host-side tests run the fused-fill orchestration on the CPU references.
FUSED_FILL_CPU = os.environ.get("METISFL_AMD_FUSED_FILL_CPU", "0") == "1"
# halo-tiled forward convs with the producer's BatchNorm in the operand fill
# (MFL_HCONV=0: BN apply + im2col conv, for A/B runs)
HCONV = os.environ.get("MFL_HCONV", "1") == "1"
# ... for the bf16 option too (MFL_HCONV_BF16=0: BN apply + im2col conv)
HCONV_BF16 = os.environ.get("MFL_HCONV_BF16", "1") == "1"
# MFL_HCONV_SKIP="32,16": layers of these input sizes run the im2col path
# instead (A/B runs of the halo conv per stage; the co-located regime sets it,
# models/colocated.py configure_regime).  Read when a layer is built.
HCONV_SKIP: set[int] | None = None


def hconv_skip() -> set[int]:
    if HCONV_SKIP is not None:
        return HCONV_SKIP
    return {int(v) for v in os.environ.get("MFL_HCONV_SKIP", "").split(",") if v.strip()}
def premasked(t: torch.Tensor) -> bool:
    """Whether a dgrad that fuses a consumer BN's backward sums (``bnb``) into
    its epilogue stores dX already multiplied by that BN's ReLU mask (the
    conv32 / conv epilogues and their host mirror; not the opt-in halo
    dgrad), so the consumer's BN backward reads no mask."""
    return t.dtype in (torch.float32, torch.bfloat16) and not HALO_DGRAD and PREMASK


# MFL_BN_PREMASK=0: consumers re-apply the ReLU mask (A/B runs)
PREMASK = os.environ.get("MFL_BN_PREMASK", "1") == "1"


# a downsampling block's conv1 and shortcut BN-backward applies in one launch
# (MFL_BN_BWD_PAIR=0: two launches, for A/B runs)
BN_BWD_PAIR = os.environ.get("MFL_BN_BWD_PAIR", "1") == "1"
# halo dgrad with the BatchNorm backward in its fill (see ConvBN.backward)
HALO_DGRAD = os.environ.get("MFL_HALO_DGRAD", "0") == "1"
# the stem's BN backward + weight gradient in one launch (MFL_STEM_FUSED=0:
# BN backward apply + im2col wgrad, for A/B runs)
STEM_FUSED = os.environ.get("MFL_STEM_FUSED", "1") == "1"
# MFL_STEM_TAIL=1: the rest of the pending optimizer rides in the fused stem
# backward launch instead of the step's last optimizer launch -- measured
# neutral (1.0224 / 1.0225 vs 1.0162 / 1.0270 ms per update,
# profiles/r4/step/tail3/), so off
STEM_TAIL = os.environ.get("MFL_STEM_TAIL", "0") == "1"


class Pending:
    """An activation that has not been materialised yet:
    T = relu?(BN_src(z) [+ res | + BN_r(zr)]).  Its consumer applies T in the
    operand fill (halo conv) and writes it into ``y`` / ``yp`` (the owning
    layer's output buffers); ``materialize`` runs it as a BatchNorm apply
    instead, for consumers without a fused fill (stride-2 convs, the head)."""

    def __init__(self, layer: "ConvBN", res: torch.Tensor | None = None, res_layer: "ConvBN | None" = None):
        self.layer = layer
        self.z = layer.z
        self.bn = layer.bn_params()
        self.relu = layer.relu
        self.res = res
        self.res_layer = res_layer  # residual = BN of this (projection shortcut) layer's z
        self.zr = res_layer.z if res_layer is not None else None
        self.bnr = res_layer.bn_params() if res_layer is not None else None
        self.y = layer.y
        self.yp = layer.out_p()

    @staticmethod
    def of(layer: "ConvBN") -> "Pending":
        return Pending(layer)

    def materialize(self, train: bool) -> torch.Tensor:
        """BatchNorm apply(s) writing y (+ yp); returns y."""
        res = self.res
        if self.res_layer is not None:
            res = self.res_layer.bn_forward(train=train)
        self.layer.bn_forward(res, train)
        return self.y


class Layer:
    def specs(self) -> list[VarSpec]:
        return []

    def bind(self, st: FlatState, ws: Workspace, device) -> None:
        pass

    def prepare_backward(self) -> None:
        """Per-step weight re-layouts needed by backward (after optimizer)."""


class ConvBN(Layer):
    """conv(k x k, stride) -> BatchNorm -> [+ residual] -> [ReLU], NHWC in the
    model's compute dtype (fp32: reference precision, or bf16)."""

    def __init__(self, name: str, N: int, H: int, W: int, cin: int, cout: int, k: int,
                 stride: int, relu: bool = True, residual: bool = False, momentum: float = 0.1,
                 eps: float = 1e-5, need_dgrad: bool = True):
        self.name = name
        self.shp = ConvShape(N, H, W, cin, cout, k, k, stride, k // 2)
        self.relu = relu
        self.residual = residual
        self.momentum = momentum
        self.eps = eps
        self.need_dgrad = need_dgrad
        self.P, self.Q = self.shp.P, self.shp.Q
        self.M = N * self.P * self.Q

    # layers that run on the side stream use the second split-K slab
    alt_workspace = False

    @property
    def out_shape(self):
        return (self.shp.N, self.P, self.Q, self.shp.Co)

    def _split(self):
        return self.ws.split2 if self.alt_workspace else self.ws.split

    def specs(self):
        s, n = self.shp, self.name
        fan_in = s.R * s.S * s.C
        return [
            VarSpec(f"{n}.conv.weight", (s.Co, s.R, s.S, s.C), True, "he_normal", fan_in=fan_in),
            VarSpec(f"{n}.bn.gamma", (s.Co,), True, "ones"),
            VarSpec(f"{n}.bn.beta", (s.Co,), True, "zeros"),
            VarSpec(f"{n}.bn.moving_mean", (s.Co,), False, "zeros"),
            VarSpec(f"{n}.bn.moving_variance", (s.Co,), False, "ones"),
        ]

    def bind(self, st: FlatState, ws: Workspace, device):
        s, n = self.shp, self.name
        self.st = st
        self.ws = ws
        self.w16 = st.compute(f"{n}.conv.weight")
        self.wp = st.packed(f"{n}.conv.weight")  # bf16x3 weight mirror (fp32 GPU path), else None
        self.dw = st.grad(f"{n}.conv.weight")
        self.gamma = st.view(f"{n}.bn.gamma")
        self.beta = st.view(f"{n}.bn.beta")
        self.dgamma = st.grad(f"{n}.bn.gamma")
        self.dbeta = st.grad(f"{n}.bn.beta")
        self.rmean = st.view(f"{n}.bn.moving_mean")
        self.rvar = st.view(f"{n}.bn.moving_variance")
        bf = dict(dtype=ws.dtype, device=device)
        f32 = dict(dtype=torch.float32, device=device)
        self.z = torch.zeros(self.out_shape, **bf)      # conv output (pre-BN)
        self.y = torch.zeros(self.out_shape, **bf)      # layer output
        self.dz = torch.zeros(self.out_shape, **bf)
        # fp32 GPU path, bf16x3 conv products: the BN apply also writes y's
        # packed (hi << 16 | lo) split, the operand the consuming convolutions
        # (forward and wgrad) decode instead of splitting per k-tile
        self.yp = (torch.zeros(self.out_shape, dtype=torch.int32, device=device)
                   if ws.dtype == torch.float32 and torch.device(device).type == "cuda" else None)
        self.xp = None
        self.mean = torch.zeros(s.Co, **f32)
        self.invstd = torch.zeros(s.Co, **f32)
        # fp64 [2C] statistics accumulators (forward sums, backward sums),
        # carved from the model-wide buffer the optimizer launch re-zeroes
        # fp32 kernels spread their fp64 atomics over 8 replicas (one per
        # XCD under round-robin placement): 256+ workgroups adding into the
        # same 2*C addresses serialised at the memory side (~5 us per conv)
        reps = 8 if ws.dtype == torch.float32 and torch.device(device).type == "cuda" else 1
        self.acc_f = ws.take_acc(2 * s.Co * reps)
        self.acc_b = ws.take_acc(2 * s.Co * reps)
        dev = torch.device(device)
        self.pf = K.conv_plan(0, s, dev, ws.dtype)
        self.pd = K.conv_plan(1, s, dev, ws.dtype)
        self.pw = K.conv_plan(2, s, dev, ws.dtype)
        ws.need_split(self.pf.workspace)
        ws.need_split(self.pd.workspace)
        # halo conv with the fused BN fill: fp32 activations with bf16x3
        # products on the GPU (or FUSED_FILL_CPU for the host-side tests), or
        # the bf16 option's activations with plain bf16 products
        self._hconv_ws = -1
        if HCONV and s.H not in hconv_skip() and ((ws.dtype == torch.float32 and (
                (dev.type == "cuda" and K.conv_products() == "bf16x3") or (dev.type == "cpu" and FUSED_FILL_CPU)))
                or (ws.dtype == torch.bfloat16 and dev.type == "cuda" and HCONV_BF16)):
            self._hconv_ws = K.hconv_workspace(s, dev)
            if self._hconv_ws > 0:
                ws.need_split(self._hconv_ws)

    def out_p(self) -> torch.Tensor | None:
        """The packed mirror of this layer's output (None unless the fp32 GPU
        path runs bf16x3 conv products)."""
        return self.yp if self.yp is not None and K.conv_products() == "bf16x3" else None

    def bn_params(self) -> K.BnParams:
        return K.BnParams(self.ws.acc(self.acc_f), self.gamma, self.beta, self.mean, self.invstd,
                          self.rmean, self.rvar, self.momentum, self.eps)

    def hconv_ok(self) -> bool:
        """Whether this conv runs as a halo-tiled conv with its input's BN
        fused into the operand fill (fp32 activations, bf16x3 products)."""
        return self._hconv_ws >= 0

    def forward_fused(self, src: "Pending", train: bool = True) -> "Pending":
        """z = conv(T(src)) with the producer's BatchNorm (+ residual, + ReLU)
        applied in this conv's operand fill; the owner tiles materialise T(src)
        into src's y / yp.  Returns this layer's output as the next Pending."""
        s = self.shp
        self.x, self.xp = src.y, src.yp
        K.hconv_forward(src.z, self.wp, self.w16, self.z, s, src.bn, train, src.relu, ws=self._split(),
                        stats=self.ws.acc(self.acc_f) if train else None, res=src.res, zr=src.zr,
                        bnr=src.bnr, y=src.y, yp=src.yp)
        return Pending.of(self)

    def forward(self, x: torch.Tensor, residual: torch.Tensor | None = None, train: bool = True,
                xp: torch.Tensor | None = None, bn: bool = True):
        """``xp``: the packed mirror of ``x`` its producer wrote (or None).
        ``bn=False``: the convolution only (its BatchNorm is applied by the
        consumer, see forward_fused); returns None."""
        s = self.shp
        self.x = x
        self.xp = xp
        K.conv_forward(x, self.w16, self.z, s, self._split(), self.ws.acc(self.acc_f) if train else None,
                       wp=self.wp, xp=xp)
        if not bn:
            return None
        return self.bn_forward(residual, train)

    def bn_forward(self, residual: torch.Tensor | None = None, train: bool = True):
        """The BN (+residual, +ReLU) half of forward(), for a z already computed."""
        s = self.shp
        K.bn_apply(self.z, s.Co, self.ws.acc(self.acc_f), self.gamma, self.beta, self.mean,
                   self.invstd, self.rmean, self.rvar, self.y, residual, self.relu, train,
                   self.momentum, self.eps, yp=self.out_p())
        return self.y

    def bn_target(self) -> K.BnBwdTarget:
        """This layer's BN backward as the fused-reduction target of the dgrad
        that produces its upstream gradient."""
        return K.BnBwdTarget(self.z, self.y if self.relu else None, self.mean, self.invstd,
                             self.ws.acc(self.acc_b))

    def bn_side(self) -> K.BnSide | None:
        """This (shortcut) layer's BN backward sums as a side reduction of the
        launch that writes its upstream gradient (fp32 GPU path)."""
        if (self.ws.dtype == torch.float32 and self.z.is_cuda and 256 % (self.shp.Co // 4) == 0
                and self.shp.Co % 4 == 0):
            return K.BnSide(self.z, self.mean, self.invstd, self.ws.acc(self.acc_b))
        return None

    def bn_backward_args(self, dy: torch.Tensor, dy_masked: bool = False) -> tuple:
        """(dy, z, relu mask, C, gamma, mean, invstd, acc, dgamma, dbeta, dz):
        this layer's presummed BN-backward apply writing its packed dz (the
        operands of bn_backward_pair); ``dy_masked``: dy arrives masked."""
        return (dy, self.z, self.y if self.relu and not dy_masked else None, self.shp.Co, self.gamma, self.mean,
                self.invstd, self.ws.acc(self.acc_b), self.dgamma, self.dbeta, self.dz)

    def backward(self, dy: torch.Tensor, dx: torch.Tensor | None, accumulate: bool = False,
                 dres: torch.Tensor | None = None, presummed: bool = False,
                 bnb: K.BnBwdTarget | None = None, side: K.BnSide | None = None,
                 bn_done: bool = False, dy_masked: bool = False) -> None:
        """dy: gradient w.r.t. this layer's output.  Writes dgamma/dbeta/dW into
        the flat gradient buffer and (if dx is given) d input into dx; ``dres``
        receives the ReLU-masked dy that the residual branch needs.
        ``presummed``: dy's producer already accumulated this BN's backward
        reductions; ``bnb``: the BN whose upstream gradient ``dx`` is (its
        reductions are fused into this layer's dgrad epilogue); ``bn_done``:
        the BN backward already wrote dz (a paired apply launch);
        ``dy_masked``: dy arrives multiplied by this layer's ReLU mask (see
        :func:`premasked`)."""
        s = self.shp
        if bn_done:
            pk = self.dz.is_cuda and self.dz.dtype == torch.float32 and K.conv_products() == "bf16x3"
            self._conv_backward(dx, accumulate, bnb, pk)
            return
        if (STEM_FUSED and dx is None and dres is None and presummed and side is None and self.relu
                and ((self.z.dtype == torch.float32 and (self.z.is_cuda or FUSED_FILL_CPU))
                     or (self.z.dtype == torch.bfloat16 and self.z.is_cuda))
                and K.stem_backward_ok(s, self.z.device)):
            # no dgrad (the stem): BN backward + weight gradient in one launch,
            # which also carries the optimizer of everything still pending
            # but the stem's own variables
            K.stem_backward(dy, self.z, self.y, self.x, s, self.gamma, self.mean, self.invstd,
                            self.ws.acc(self.acc_b), self.dgamma, self.dbeta, self.dw,
                            opt=self.ws.take_opt_tail(everything=True) if STEM_TAIL else None)
            return
        if (HALO_DGRAD and dx is not None and presummed and side is None and self.hconv_ok()
                and self.z.dtype == torch.float32):
            # halo dgrad: the BN backward runs in its operand fill and its
            # owner tiles write dz packed for the wgrad.  Opt-in: measured on
            # MI355X (scripts/hdgrad_bench.py) the halo dgrad beats BN apply +
            # im2col dgrad (19.9 vs 23.7 us at 32x32x64), but the wgrad then
            # runs alone (19.4 us) instead of inside the paired launch, where
            # dgrad + wgrad take 27.6 us: 38.9 vs 36.1 us per layer
            bnp = K.BnParams(self.ws.acc(self.acc_b), self.gamma, self.beta, self.mean, self.invstd, None, None)
            dzp = self.dz.view(torch.int32) if self.dz.is_cuda else self.dz
            K.hconv_dgrad(dy, self.y if self.relu else None, self.z, self.wp, self.w16, dx, s, bnp,
                          dgamma=self.dgamma, dbeta=self.dbeta, ws=self._split(), dres=dres, dzp=dzp,
                          accumulate=accumulate, bnb=bnb)
            K.conv_wgrad(self.x, self.dz, self.dw, s, accumulate=True, dy_packed=self.dz.is_cuda, xp=self.xp)
            return
        # bf16x3 conv products: dz is only ever read by this layer's dgrad and
        # wgrad, so the BN backward writes it as their packed operand encoding
        pk = self.dz.is_cuda and self.dz.dtype == torch.float32 and K.conv_products() == "bf16x3"
        K.bn_backward(dy, self.z, self.y if self.relu and not dy_masked else None, s.Co, self.gamma, self.mean,
                      self.invstd, self.ws.acc(self.acc_b), self.dgamma, self.dbeta, self.dz, dres,
                      presummed=presummed, side=side, dx_packed=pk)
        self._conv_backward(dx, accumulate, bnb, pk)

    def _conv_backward(self, dx, accumulate: bool, bnb, pk: bool) -> None:
        s = self.shp
        # weight gradient: off the critical path -> side stream (joined before
        # the optimizer); the gradient buffer is zero on entry (re-zeroed by
        # the optimizer launch), so split-K slices accumulate atomically
        if dx is not None and not self.ws.overlap:
            # both GEMMs in one launch (their workgroups share the CUs); the
            # fp32 launch also carries the next optimizer tail, if any
            K.conv_backward_pair(self.x, self.dz, self.dw, self.w16, dx, s, self._split(), accumulate,
                                 bnb=bnb, wp=self.wp, dy_packed=pk, xp=self.xp, opt=self.ws.take_opt_tail())
            return
        with self.ws.fork():
            K.conv_wgrad(self.x, self.dz, self.dw, s, accumulate=True, dy_packed=pk, xp=self.xp)
        if dx is not None:
            K.conv_dgrad(self.dz, self.w16, dx, s, self._split(), accumulate, bnb=bnb, wp=self.wp, dy_packed=pk)


class BasicBlock(Layer):
    """ResNet basic block: relu(bn2(conv2(relu(bn1(conv1(x))))) + shortcut(x))."""

    def __init__(self, name: str, N: int, H: int, W: int, cin: int, cout: int, stride: int):
        self.name = name
        self.c1 = ConvBN(f"{name}.conv1", N, H, W, cin, cout, 3, stride, relu=True)
        P, Q = self.c1.P, self.c1.Q
        self.c2 = ConvBN(f"{name}.conv2", N, P, Q, cout, cout, 3, 1, relu=True, residual=True)
        self.sc = None
        if stride != 1 or cin != cout:
            self.sc = ConvBN(f"{name}.shortcut", N, H, W, cin, cout, 1, stride, relu=False)
            self.sc.alt_workspace = True
        self.out_shape = self.c2.out_shape
        self.in_shape = (N, H, W, cin)

    def sublayers(self):
        return [l for l in (self.c1, self.c2, self.sc) if l is not None]

    def specs(self):
        return [v for l in self.sublayers() for v in l.specs()]

    def bind(self, st, ws, device):
        for l in self.sublayers():
            l.bind(st, ws, device)
        self.da = torch.zeros(self.c1.out_shape, dtype=ws.dtype, device=device)
        self.dres = None
        if self.sc is not None:
            self.dres = torch.zeros(self.out_shape, dtype=ws.dtype, device=device)

    def prepare_backward(self):
        for l in self.sublayers():
            l.prepare_backward()

    def out_p(self):
        return self.c2.out_p()

    def forward(self, x, train=True, xp=None):
        """``xp``: the packed mirror of ``x`` (bf16x3 fp32 path) or None."""
        if self.sc is None:
            a = self.c1.forward(x, train=train, xp=xp)
            return self.c2.forward(a, residual=x, train=train, xp=self.c1.out_p())
        if not self.c1.ws.overlap and self.c1.shp.R == 3 and self.c1.shp.stride == 2:
            # conv1 and the projection shortcut in one paired launch
            c1, sc = self.c1, self.sc
            c1.x = sc.x = x
            c1.xp = sc.xp = xp
            K.conv_forward_pair(x, c1.w16, c1.z, c1._split(), c1.ws.acc(c1.acc_f) if train else None,
                                sc.w16, sc.z, sc._split(), sc.ws.acc(sc.acc_f) if train else None, c1.shp,
                                wp1=c1.wp, wp2=sc.wp, xp=xp)
            if x.is_cuda and not sc.relu and c1.relu:
                # ... and their two BatchNorms in one launch (the shortcut's
                # output only feeds the residual add: no packed mirror)
                f32 = x.dtype == torch.float32
                pair = K.ops().bn32_apply_pair if f32 else K.ops().bn_apply_pair
                pair(sc.z, sc.gamma, sc.beta, sc.mean, sc.invstd, sc.rmean, sc.rvar,
                     sc.ws.acc(sc.acc_f) if train else None, sc.y,
                     c1.z, c1.gamma, c1.beta, c1.mean, c1.invstd, c1.rmean, c1.rvar,
                     c1.ws.acc(c1.acc_f) if train else None, c1.y,
                     c1.shp.Co, train, c1.momentum, c1.eps, *((c1.out_p(),) if f32 else ()))
                r, a = sc.y, c1.y
            else:
                r = sc.bn_forward(train=train)
                a = c1.bn_forward(train=train)
            return self.c2.forward(a, residual=r, train=train, xp=c1.out_p())
        # projection shortcut runs concurrently with conv1 (side stream, own
        # split-K workspace); conv2 consumes both after the join
        with self.c1.ws.fork():
            r = self.sc.forward(x, train=train, xp=xp)
        a = self.c1.forward(x, train=train, xp=xp)
        self.c1.ws.join()
        return self.c2.forward(a, residual=r, train=train, xp=self.c1.out_p())

    def forward_fused(self, src: Pending, train: bool = True) -> Pending:
        """Forward with every BatchNorm apply deferred into its consumer's
        operand fill: ``src`` is this block's (not yet materialised) input; the
        returned Pending is its output relu(BN2(z2) + shortcut)."""
        c1, c2, sc = self.c1, self.c2, self.sc
        if sc is None:
            # identity block: conv1's fill materialises x (the residual)
            a = c1.forward_fused(src, train) if c1.hconv_ok() else self._plain(c1, src, train)
            out = c2.forward_fused(a, train) if c2.hconv_ok() else self._plain(c2, a, train)
            out.res = src.y
            return out
        # downsampling block: the paired stride-2 conv1 + 1x1 shortcut read x
        # packed, so x is materialised by a BatchNorm apply first
        x = src.materialize(train)
        c1.x = sc.x = x
        c1.xp = sc.xp = src.yp
        K.conv_forward_pair(x, c1.w16, c1.z, c1._split(), c1.ws.acc(c1.acc_f) if train else None,
                            sc.w16, sc.z, sc._split(), sc.ws.acc(sc.acc_f) if train else None, c1.shp,
                            wp1=c1.wp, wp2=sc.wp, xp=src.yp)
        a = Pending.of(c1)
        out = c2.forward_fused(a, train) if c2.hconv_ok() else self._plain(c2, a, train)
        # the shortcut's BatchNorm rides in the consumer of z2 (residual BN_r(z_sc))
        return Pending(c2, res_layer=sc)

    @staticmethod
    def _plain(layer: ConvBN, src: Pending, train: bool) -> Pending:
        x = src.materialize(train)
        layer.forward(x, train=train, xp=src.yp, bn=False)
        return Pending.of(layer)

    def backward(self, dout, dx, presummed: bool = False, prev: K.BnBwdTarget | None = None,
                 dout_masked: bool = False):
        """``presummed``: conv2's BN reductions were fused into dout's producer;
        ``prev``: the BN consuming dx (the previous block's conv2 or the stem),
        whose reductions are fused into the LAST dgrad writing dx (conv1's);
        ``dout_masked``: dout arrives multiplied by conv2's ReLU mask."""
        pm = premasked(self.da)  # conv2's dgrad stores da masked for conv1's BN
        if self.sc is None:
            # identity shortcut: masked dout goes straight into dx, conv1's
            # dgrad then accumulates onto it (no add kernel).  A model may give
            # dx the SAME buffer as a masked dout (in-place residual gradient):
            # then there is nothing to copy at all
            inplace = dout_masked and dx.data_ptr() == dout.data_ptr()
            self.c2.backward(dout, self.da, dres=None if inplace else dx, presummed=presummed,
                             bnb=self.c1.bn_target(), dy_masked=dout_masked)
            self.c1.backward(self.da, dx, accumulate=True, presummed=True, bnb=prev, dy_masked=pm)
        else:
            # the shortcut BN's backward sums ride in conv2's BN-backward launch
            # (it writes dres, the shortcut's upstream gradient)
            side = self.sc.bn_side()
            self.c2.backward(dout, self.da, dres=self.dres, presummed=presummed, bnb=self.c1.bn_target(),
                             side=side, dy_masked=dout_masked)
            if side is not None and BN_BWD_PAIR and not HALO_DGRAD and self.da.dtype == torch.float32:
                # conv1's and the shortcut's sums are both complete now (conv2's
                # dgrad epilogue / its BN backward's side reduction): their two
                # BN-backward applies in one launch
                K.bn_backward_pair(self.c1.bn_backward_args(self.da, dy_masked=pm),
                                   self.sc.bn_backward_args(self.dres),
                                   dx_packed=self.da.is_cuda and K.conv_products() == "bf16x3")
                self.sc.backward(self.dres, dx, bn_done=True)
                self.c1.backward(self.da, dx, accumulate=True, bnb=prev, bn_done=True)
                return
            self.sc.backward(self.dres, dx, presummed=side is not None)
            self.c1.backward(self.da, dx, accumulate=True, presummed=True, bnb=prev, dy_masked=pm)


class ClassifierHead(Layer):
    """Global average pool + Linear(C -> K) + softmax cross-entropy, fused."""

    def __init__(self, name: str, N: int, HW: int, C: int, K_: int):
        self.name, self.N, self.HW, self.C, self.K = name, N, HW, C, K_

    def specs(self):
        return [VarSpec(f"{self.name}.kernel", (self.K, self.C), True, "glorot_uniform",
                        fan_in=self.C, fan_out=self.K),
                VarSpec(f"{self.name}.bias", (self.K,), True, "zeros")]

    def bind(self, st, ws, device):
        self.W = st.view(f"{self.name}.kernel")
        self.b = st.view(f"{self.name}.bias")
        self.dW = st.grad(f"{self.name}.kernel")
        self.db = st.grad(f"{self.name}.bias")
        f32 = dict(dtype=torch.float32, device=device)
        self.feat = torch.zeros(self.N * self.C, **f32)
        self.dlogits = torch.zeros(self.N * self.K, **f32)
        self.dx = torch.zeros((self.N, self.HW, self.C), dtype=ws.dtype, device=device)

    # set by forward_backward: the head added the BN-backward sums of its dx
    # into the last block's conv2 accumulator (its backward runs presummed)
    summed_input_bn = False

    def forward_backward(self, x, labels, stats, train=True):
        """``x``: the pooled activation, or the last block's Pending output
        (fp32 path): its BatchNorm + residual + ReLU are applied in the head's
        pooling loop (no BatchNorm apply launch) and the head adds that BN's
        backward sums (no reduce launch)."""
        self.summed_input_bn = False
        if isinstance(x, Pending):
            p = x
            if (p.res is not None and p.zr is None and p.relu
                    and ((p.z.dtype == torch.float32 and (p.z.is_cuda or FUSED_FILL_CPU))
                         or (p.z.dtype == torch.bfloat16 and p.z.is_cuda))):
                lay = p.layer
                acc_b = lay.ws.acc(lay.acc_b) if train else None
                K.head_forward_backward_bn(self.N, self.HW, self.C, self.W, self.b, labels, self.feat, self.dlogits,
                                           self.dx, stats, train, self.dW if train else None,
                                           self.db if train else None, p.z, p.res, p.bn, train, p.y, acc_b)
                self.summed_input_bn = train
                return self.dx
            x = p.materialize(train)
        # the weight gradient rides in the same launch (atomics into the
        # step's zeroed gradient buffer): one kernel for the whole head
        K.head_forward_backward(x, self.N, self.HW, self.C, self.W, self.b, labels, self.feat,
                                self.dlogits, self.dx, stats, backward=train,
                                dW=self.dW if train else None, db=self.db if train else None)
        return self.dx
