"""ResNet-18 for CIFAR-10 (32x32x3 input, 10 classes) on the static executor.

The north-star config of this framework (BASELINE.json: "8-learner FedAvg
CIFAR-10 ResNet-18").  The reference ships no ResNet-18 -- its CIFAR model
is the VGG-style CifarCNN (examples/keras/models/cifar_cnn.py:7-52, provided
in models/cifar_cnn.py) -- so this is the standard CIFAR ResNet-18 topology:
3x3 stem (64) -> 4 stages of 2 BasicBlocks (64/128/256/512, strides 1/2/2/2)
-> global average pool -> Linear(512, 10).  11.17M parameters, 11.18M
variables including BatchNorm moving statistics.

The 3 input channels are zero-padded to 8 once, at shard upload, so the stem
conv runs on the same 16-B-vectorised MFMA path as every other conv.

Precision: ``dtype="fp32"`` (default) trains at the reference's precision --
Keras trains fp32 (examples/keras/models/cifar_cnn.py:19-41, no
mixed-precision policy; keras_model_ops.py:117-197) -- on the exact fp32 MFMA
kernels (conv32.hip / bn32.hip).  ``dtype="bf16"`` is the mixed-precision
option (bf16 activations and weights, fp32 master / accumulation).

``conv_products`` picks how the fp32 convolutions form their products
(ops/nn.py ``set_conv_products``): ``"exact"`` fp32 MFMA or ``"bf16x3"``
split products with fp32 storage and accumulation (relative error ~4e-6 per
convolution).  Default: ``METISFL_AMD_CONV_PRODUCTS`` or
:data:`DEFAULT_CONV_PRODUCTS`.
"""
from __future__ import annotations

import os

import torch

from metisfl_amd.models.layers import BasicBlock, ClassifierHead, ConvBN, Pending, premasked
from metisfl_amd.models.net import StaticNet
from metisfl_amd.ops.optim import split_pack

DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16}
DEFAULT_CONV_PRODUCTS = "bf16x3"
# identity blocks accumulate the residual gradient in place in dout's buffer
# instead of copying it (profiles/r4/step/inplace/: -0.8 % per update, one
# learner and co-located; MFL_INPLACE_RESGRAD=0 for A/B runs)
INPLACE_RESIDUAL_GRAD = os.environ.get("MFL_INPLACE_RESGRAD", "1") == "1"


def default_conv_products() -> str:
    return os.environ.get("METISFL_AMD_CONV_PRODUCTS", DEFAULT_CONV_PRODUCTS)


class ResNet18(StaticNet):
    input_shape = (32, 32, 8)
    opt_tails_supported = True
    num_classes = 10
    widths = (64, 128, 256, 512)

    def __init__(self, batch_size: int = 32, device="cpu", optimizer=None, seed: int = 0,
                 width_mult: float = 1.0, num_classes: int = 10, dtype: str = "fp32",
                 conv_products: str | None = None, shared_state=None):
        self.compute_dtype = DTYPES[dtype]
        self.conv_products = conv_products or default_conv_products()
        if dtype == "fp32" and torch.device(device).type == "cuda":
            # before any plan / workspace is sized and before graph capture
            from metisfl_amd.ops.nn import set_conv_products
            set_conv_products(self.conv_products)
        self.width_mult = width_mult
        self.num_classes = num_classes
        super().__init__(batch_size, device, optimizer, seed, shared_state=shared_state)

    def _make_eval_twin(self, batch: int, state=None):
        dtype = next(k for k, v in DTYPES.items() if v == self.compute_dtype)
        return ResNet18(batch_size=batch, device=self.device, dtype=dtype, conv_products=self.conv_products,
                        width_mult=self.width_mult, num_classes=self.num_classes,
                        shared_state=self.state if state is None else state)

    def build(self):
        N = self.B
        w = [max(8, int(c * self.width_mult) // 8 * 8) for c in self.widths]
        H = self.input_shape[0]
        self.stem = ConvBN("stem", N, H, H, self.input_shape[2], w[0], 3, 1, relu=True,
                           need_dgrad=False)
        blocks = []
        cin, h = w[0], H
        for i, (c, s) in enumerate(zip(w, (1, 2, 2, 2))):
            b1 = BasicBlock(f"layer{i + 1}.0", N, h, h, cin, c, s)
            h = b1.out_shape[1]
            b2 = BasicBlock(f"layer{i + 1}.1", N, h, h, c, c, 1)
            blocks += [b1, b2]
            cin = c
        self.blocks = blocks
        self.head = ClassifierHead("fc", N, h * h, cin, self.num_classes)

    def all_layers(self):
        return [self.stem] + self.blocks + [self.head]

    def post_bind(self):
        dev = self.device
        # gradient buffers at block boundaries: dx of block i is dout of block i-1.
        # An identity block (not the last: the head's dx arrives unmasked)
        # whose dout arrives pre-masked accumulates its input gradient in place
        # in dout's buffer (layers.BasicBlock.backward): the two share it.
        self.dacts = [torch.zeros(b.in_shape, dtype=self.compute_dtype, device=dev) for b in self.blocks]
        if premasked(self.dacts[0]) and INPLACE_RESIDUAL_GRAD:
            for i in range(len(self.blocks) - 2, -1, -1):
                if self.blocks[i].sc is None:
                    self.dacts[i] = self.dacts[i + 1]
        self._xbp = None  # packed input batch (bf16x3 fp32 path), sized on first use
        if self.stem.yp is not None:
            self._xbp = torch.zeros((self.B,) + self.input_shape, dtype=torch.int32, device=dev)

    def packed_input(self):
        return self._xbp if self.stem.out_p() is not None else None

    def fused_fill(self) -> bool:
        """Every BatchNorm apply rides in its consumer's operand fill where the
        consumer is a halo conv (models/layers.py forward_fused)."""
        return any(c.hconv_ok() for b in self.blocks for c in b.sublayers())

    def forward_to_head(self, x, train):
        # fused-fill path: the last block's BatchNorm is applied by the head
        return self.forward(x, train, to_head=True)

    def forward(self, x, train, to_head: bool = False):
        xp = None
        if self.stem.out_p() is not None:
            # bf16x3 fp32 path: every conv operand arrives packed (hi << 16 |
            # lo); the batch gather packs the input for the stem's forward and
            # wgrad (other callers' inputs are packed here), the BN applies
            # write the rest
            if self._xbp is None or self._xbp.shape != x.shape:
                self._xbp = torch.zeros(x.shape, dtype=torch.int32, device=x.device)
            if x is not getattr(self, "xb", None):
                split_pack(x.reshape(-1), self._xbp.view(-1))
            xp = self._xbp
        if self.fused_fill():
            self.stem.forward(x, train=train, xp=xp, bn=False)
            p = Pending.of(self.stem)
            for b in self.blocks:
                p = b.forward_fused(p, train)
            return p if to_head else p.materialize(train)
        h = self.stem.forward(x, train=train, xp=xp)
        hp = self.stem.out_p()
        for b in self.blocks:
            h = b.forward(h, train=train, xp=hp)
            hp = b.out_p()
        return h

    def backward(self, dlast):
        # BN-backward reductions ride in the dgrad epilogues: every block's
        # conv1 dgrad (the last writer of the block's input gradient) sums for
        # the BN that consumes it -- the previous block's conv2, or the stem.
        # The last block's conv2 (fed by the head) reduces on its own unless
        # the head applied its BatchNorm and added the sums (fused fill).
        # Optimizer tails: the head's and every finished block's variables are
        # updated by later paired launches (StaticNet.grads_final_from).
        d = dlast.view(self.blocks[-1].out_shape)
        self.grads_final_from(self.head.name + ".")
        for i in range(len(self.blocks) - 1, -1, -1):
            prev = self.blocks[i - 1].c2 if i > 0 else self.stem
            last = i == len(self.blocks) - 1
            # dacts[i + 1] was written by block i + 1's conv1 dgrad, which stored
            # it masked for this block's conv2 BN (layers.premasked); the head's
            # dx is not
            self.blocks[i].backward(d, self.dacts[i], presummed=(not last) or self.head.summed_input_bn,
                                    prev=prev.bn_target(), dout_masked=(not last) and premasked(d))
            d = self.dacts[i]
            self.grads_final_from(self.blocks[i].name + ".")
        self.stem.backward(d, None, presummed=True)
