"""Sequential static-graph models: the reference's Keras example networks on
the HIP kernel stack.

  * ``CifarCNN``       -- examples/keras/models/cifar_cnn.py:7-52 (1,610,314
                          parameters incl. BN moving statistics)
  * ``FashionMnistFC`` -- examples/keras/models/fashion_mnist_fc.py:6-26
                          (784-128-128-10, 118,282 parameters)
  * ``HousingMLP``     -- examples/keras/models/housing_mlp.py:6-43 (the
                          scalability / stress-test regressor)

Dense layers are 1x1 convolutions on the MFMA implicit-GEMM kernels; widths
that are not a multiple of 8 (10 classes, 13 features, 1 output) are padded
with INERT units -- zero-initialised rows whose output and gradients stay
exactly zero -- and padded logits are masked out of the loss.  Documented
deviation: CifarCNN's reference applies softmax and then a from-logits
cross-entropy (a double softmax); here the last Dense emits logits.
"""
from __future__ import annotations

import math

import torch

from metisfl_amd.models.flat import VarSpec
from metisfl_amd.models.layers import Layer
from metisfl_amd.models.net import StaticNet
from metisfl_amd.ops import nn as K
from metisfl_amd.ops.nn import ConvShape


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


class SeqLayer(Layer):
    """A layer of a Sequential static net: fixed per-sample in/out shapes."""
    in_shape: tuple
    out_shape: tuple

    def forward(self, x, train: bool):
        raise NotImplementedError

    def backward(self, dy, need_dx: bool):
        raise NotImplementedError


class _ConvLike(SeqLayer):
    """conv (k x k, 'same') or dense (1x1 over a flat vector) + bias + act."""

    def __init__(self, name, B, H, W, cin, cout, k, act, live_out=None, init="glorot_uniform"):
        self.name, self.B = name, B
        self.shp = ConvShape(B, H, W, cin, cout, k, k, 1, k // 2)
        self.act = act
        self.live_out = live_out
        self.init = init

    def specs(self):
        s = self.shp
        fan_in = s.R * s.S * s.C
        fan_out = s.R * s.S * (self.live_out or s.Co)
        return [VarSpec(f"{self.name}.kernel", (s.Co, s.R, s.S, s.C), True, self.init, fan_in=fan_in,
                        fan_out=fan_out, live_rows=self.live_out),
                VarSpec(f"{self.name}.bias", (s.Co,), True, "zeros")]

    def bind(self, st, ws, device):
        s = self.shp
        self.ws = ws
        self.w16 = st.bf16(f"{self.name}.kernel")
        self.dw = st.grad(f"{self.name}.kernel")
        self.b = st.view(f"{self.name}.bias")
        self.db = st.grad(f"{self.name}.bias")
        bf = dict(dtype=torch.bfloat16, device=device)
        self.y = torch.zeros((s.N, s.P, s.Q, s.Co), **bf)
        self.dz = torch.zeros_like(self.y)
        self.dx = torch.zeros((s.N, s.H, s.W, s.C), **bf)
        dev = torch.device(device)
        ws.need_split(K.conv_plan(0, s, dev).workspace)
        ws.need_split(K.conv_plan(1, s, dev).workspace)

    def forward(self, x, train):
        s = self.shp
        self.x = x.reshape(s.N, s.H, s.W, s.C)
        K.conv_forward(self.x, self.w16, self.y, s, self.ws.split, None)
        K.bias_act(self.y, self.b, s.Co, self.act)
        return self.y.reshape((s.N,) + self.out_shape)

    def backward(self, dy, need_dx):
        s = self.shp
        K.bias_act_backward(dy.reshape(self.y.shape), self.y, self.dz, self.db, s.Co, self.act)
        K.conv_wgrad(self.x, self.dz, self.dw, s, accumulate=True)
        if not need_dx:
            return None
        K.conv_dgrad(self.dz, self.w16, self.dx, s, self.ws.split, False)
        return self.dx.reshape((s.N,) + self.in_shape)


class Conv2D(_ConvLike):
    def __init__(self, name, B, H, W, cin, cout, k=3, act=K.ACT_RELU):
        super().__init__(name, B, H, W, cin, cout, k, act)
        self.in_shape, self.out_shape = (H, W, cin), (H, W, cout)


class Dense(_ConvLike):
    def __init__(self, name, B, fin, fout, act=K.ACT_RELU, init="glorot_uniform"):
        fp = _pad8(fout)
        super().__init__(name, B, 1, 1, fin, fp, 1, act, live_out=fout if fp != fout else None, init=init)
        self.in_shape, self.out_shape = (fin,), (fp,)


class MaxPool2(SeqLayer):
    def __init__(self, B, H, W, C):
        self.B, self.H, self.W, self.C = B, H, W, C
        self.in_shape, self.out_shape = (H, W, C), (H // 2, W // 2, C)

    def bind(self, st, ws, device):
        bf = dict(dtype=torch.bfloat16, device=device)
        self.y = torch.zeros((self.B,) + self.out_shape, **bf)
        self.dx = torch.zeros((self.B,) + self.in_shape, **bf)

    def forward(self, x, train):
        self.x = x
        K.maxpool2(x, self.y, self.B, self.H, self.W, self.C)
        return self.y

    def backward(self, dy, need_dx):
        K.maxpool2_backward(dy, self.x, self.y, self.dx, self.B, self.H, self.W, self.C)
        return self.dx


class BatchNorm(SeqLayer):
    """Stand-alone BatchNorm (after a pooling layer, no activation)."""

    def __init__(self, name, B, H, W, C, momentum=0.01, eps=1e-3):
        # Keras BatchNormalization defaults: momentum 0.99 (= 0.01 update), eps 1e-3
        self.name, self.B, self.C = name, B, C
        self.in_shape = self.out_shape = (H, W, C)
        self.momentum, self.eps = momentum, eps

    def specs(self):
        n, C = self.name, self.C
        return [VarSpec(f"{n}.gamma", (C,), True, "ones"), VarSpec(f"{n}.beta", (C,), True, "zeros"),
                VarSpec(f"{n}.moving_mean", (C,), False, "zeros"),
                VarSpec(f"{n}.moving_variance", (C,), False, "ones")]

    def bind(self, st, ws, device):
        n = self.name
        self.ws = ws
        self.gamma, self.beta = st.view(f"{n}.gamma"), st.view(f"{n}.beta")
        self.dgamma, self.dbeta = st.grad(f"{n}.gamma"), st.grad(f"{n}.beta")
        self.rmean, self.rvar = st.view(f"{n}.moving_mean"), st.view(f"{n}.moving_variance")
        bf = dict(dtype=torch.bfloat16, device=device)
        self.y = torch.zeros((self.B,) + self.out_shape, **bf)
        self.dx = torch.zeros_like(self.y)
        f32 = dict(dtype=torch.float32, device=device)
        self.mean, self.invstd = torch.zeros(self.C, **f32), torch.zeros(self.C, **f32)
        self.acc_f, self.acc_b = ws.take_acc(2 * self.C), ws.take_acc(2 * self.C)

    def forward(self, x, train):
        self.x = x
        if train:
            K.bn_stats(x, self.C, self.ws.acc(self.acc_f))
        K.bn_apply(x, self.C, self.ws.acc(self.acc_f), self.gamma, self.beta, self.mean, self.invstd,
                   self.rmean, self.rvar, self.y, None, False, train, self.momentum, self.eps)
        return self.y

    def backward(self, dy, need_dx):
        K.bn_backward(dy, self.x, None, self.C, self.gamma, self.mean, self.invstd, self.ws.acc(self.acc_b),
                      self.dgamma, self.dbeta, self.dx, None)
        return self.dx


class Flatten(SeqLayer):
    def __init__(self, in_shape):
        self.in_shape = tuple(in_shape)
        self.out_shape = (math.prod(in_shape),)

    def forward(self, x, train):
        return x.reshape(x.shape[0], -1)

    def backward(self, dy, need_dx):
        return dy.reshape((dy.shape[0],) + self.in_shape)


class Dropout(SeqLayer):
    def __init__(self, B, shape, rate, seed=0x5EED):
        self.B, self.rate, self.seed = B, rate, seed
        self.in_shape = self.out_shape = tuple(shape)

    def bind(self, st, ws, device):
        self.step = st.step
        bf = dict(dtype=torch.bfloat16, device=device)
        self.y = torch.zeros((self.B,) + self.out_shape, **bf)
        self.dx = torch.zeros_like(self.y)

    def forward(self, x, train):
        if not train or self.rate <= 0:
            return x
        K.dropout(x, self.y, self.rate, self.seed, self.step)
        return self.y

    def backward(self, dy, need_dx):
        if self.rate <= 0:
            return dy
        K.dropout(dy, self.dx, self.rate, self.seed, self.step)  # same (seed, step) -> same mask
        return self.dx


class XentHead(Layer):
    """Softmax cross-entropy on (padded) logits; loss / accuracy on device."""

    def __init__(self, B, Kp, K_):
        self.B, self.Kp, self.K = B, Kp, K_

    def bind(self, st, ws, device):
        self.dlogits = torch.zeros((self.B, self.Kp), dtype=torch.bfloat16, device=device)

    def forward_backward(self, x, labels, stats, train=True):
        K.xent(x, labels, self.B, self.Kp, self.K, self.dlogits if train else None, stats)
        return self.dlogits


class MSEHead(Layer):
    def __init__(self, B, Kp):
        self.B, self.Kp = B, Kp

    def bind(self, st, ws, device):
        self.dpred = torch.zeros((self.B, self.Kp), dtype=torch.bfloat16, device=device)

    def forward_backward(self, x, targets, stats, train=True):
        K.mse(x, targets, self.B, self.Kp, self.dpred if train else None, stats)
        return self.dpred


class SequentialNet(StaticNet):
    """``layers`` applied in order, then ``head``; subclasses fill both in
    ``build_layers()``."""

    def build(self):
        self.layers, self.head = self.build_layers()

    def build_layers(self):
        raise NotImplementedError

    def all_layers(self):
        return list(self.layers) + [self.head]

    def forward(self, x, train):
        h = x
        for l in self.layers:
            h = l.forward(h, train)
        return h

    def backward(self, dlast):
        d = dlast
        for i in range(len(self.layers) - 1, -1, -1):
            d = self.layers[i].backward(d, need_dx=i > 0)


class CifarCNN(SequentialNet):
    input_shape = (32, 32, 8)  # 3 channels zero-padded to 8

    def __init__(self, batch_size=32, device="cpu", optimizer=None, seed=0, num_classes=10, dropout=0.2):
        self.num_classes, self.dropout = num_classes, dropout
        super().__init__(batch_size, device, optimizer, seed)

    def build_layers(self):
        B = self.B
        L = [Conv2D("conv2d", B, 32, 32, 8, 64), Conv2D("conv2d_1", B, 32, 32, 64, 64), MaxPool2(B, 32, 32, 64),
             BatchNorm("batch_normalization", B, 16, 16, 64),
             Conv2D("conv2d_2", B, 16, 16, 64, 128), Conv2D("conv2d_3", B, 16, 16, 128, 128),
             MaxPool2(B, 16, 16, 128), BatchNorm("batch_normalization_1", B, 8, 8, 128),
             Conv2D("conv2d_4", B, 8, 8, 128, 128), Conv2D("conv2d_5", B, 8, 8, 128, 128),
             MaxPool2(B, 8, 8, 128), Flatten((4, 4, 128)),
             Dense("dense", B, 2048, 512), Dropout(B, (512,), self.dropout),
             Dense("dense_1", B, 512, self.num_classes, act=K.ACT_NONE)]
        return L, XentHead(B, _pad8(self.num_classes), self.num_classes)


class FashionMnistFC(SequentialNet):
    input_shape = (784,)

    def __init__(self, batch_size=32, device="cpu", optimizer=None, seed=0, num_classes=10):
        self.num_classes = num_classes
        super().__init__(batch_size, device, optimizer, seed)

    def build_layers(self):
        B = self.B
        L = [Dense("dense", B, 784, 128), Dense("dense_1", B, 128, 128),
             Dense("dense_2", B, 128, self.num_classes, act=K.ACT_NONE)]
        return L, XentHead(B, _pad8(self.num_classes), self.num_classes)


class HousingMLP(SequentialNet):
    """Regression MLP; 13 input features are zero-padded to 16."""
    input_shape = (16,)

    def __init__(self, batch_size=32, device="cpu", optimizer=None, seed=0, params_per_layer=10,
                 hidden_layers_num=1):
        self.ppl, self.hidden = params_per_layer, hidden_layers_num
        super().__init__(batch_size, device, optimizer, seed)

    def build_layers(self):
        B, p = self.B, self.ppl
        L = [Dense("dense", B, 16, p, init="normal")]
        for i in range(self.hidden):
            L.append(Dense(f"dense_{i + 1}", B, _pad8(p), p, init="normal"))
        L.append(Dense(f"dense_{self.hidden + 1}", B, _pad8(p), 1, act=K.ACT_NONE, init="normal"))
        return L, MSEHead(B, 8)
