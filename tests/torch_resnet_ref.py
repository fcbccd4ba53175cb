"""Independent fp32/fp64 ``torch.nn`` ResNet-18 (NCHW, nn.Conv2d /
nn.BatchNorm2d / nn.Linear, autograd) used as the whole-model oracle for the
framework's static ResNet-18 executor.  Nothing here touches metisfl_amd's
ops: weights are copied in from a FlatState by variable name and gradients
are read back by the same names."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _relu(t, masks, key, flips=None):
    """ReLU, or -- with ``masks`` -- multiplication by a given 0/1 mask (the
    same function wherever the mask agrees with the sign of ``t``).  Pinning
    the masks to the candidate's own removes ReLU's measure-zero derivative
    jump from a gradient comparison: an element whose pre-activation is
    within rounding of 0 can land on either side in two correct fp32
    evaluations, and its whole upstream gradient then flips in or out."""
    if masks is None or key not in masks:
        return F.relu(t)
    mk = masks[key].to(t.dtype)
    if flips is not None:
        flips[0] += int(((t > 0).to(t.dtype) != mk).sum())
    return t * mk


class _Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.masks, self.key, self.flips = None, "", None
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout, eps=1e-5, momentum=0.1)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout, eps=1e-5, momentum=0.1)
        self.sc = None
        if stride != 1 or cin != cout:
            self.sc = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, 0, bias=False),
                                    nn.BatchNorm2d(cout, eps=1e-5, momentum=0.1))

    def forward(self, x):
        o = _relu(self.bn1(self.conv1(x)), self.masks, f"{self.key}.conv1", self.flips)
        o = self.bn2(self.conv2(o))
        return _relu(o + (self.sc(x) if self.sc is not None else x), self.masks, f"{self.key}.conv2", self.flips)


class TorchResNet18(nn.Module):
    def __init__(self, widths=(64, 128, 256, 512), cin=8, num_classes=10):
        super().__init__()
        self.stem = nn.Conv2d(cin, widths[0], 3, 1, 1, bias=False)
        self.stem_bn = nn.BatchNorm2d(widths[0], eps=1e-5, momentum=0.1)
        blocks, c = [], widths[0]
        for w, s in zip(widths, (1, 2, 2, 2)):
            blocks += [_Block(c, w, s), _Block(w, w, 1)]
            c = w
        self.blocks = nn.ModuleList(blocks)
        self.fc = nn.Linear(c, num_classes)
        self.masks = None
        self.flips = [0]  # pinned mask elements that disagree with the sign

    def pin_relu_masks(self, masks: dict | None) -> None:
        """``masks``: framework ConvBN name -> NCHW 0/1 tensor of that layer's
        ReLU output sign (see ``_relu``)."""
        self.masks = masks
        for i, b in enumerate(self.blocks):
            b.masks, b.key, b.flips = masks, f"layer{i // 2 + 1}.{i % 2}", self.flips

    def forward(self, x):
        h = _relu(self.stem_bn(self.stem(x)), self.masks, "stem", self.flips)
        for b in self.blocks:
            h = b(h)
        return self.fc(h.mean((2, 3)))

    # ---- name map to the framework's variables --------------------------------
    def _convbn(self):
        """(framework ConvBN name, conv module, bn module)"""
        out = [("stem", self.stem, self.stem_bn)]
        for i, b in enumerate(self.blocks):
            n = f"layer{i // 2 + 1}.{i % 2}"
            out += [(f"{n}.conv1", b.conv1, b.bn1), (f"{n}.conv2", b.conv2, b.bn2)]
            if b.sc is not None:
                out.append((f"{n}.shortcut", b.sc[0], b.sc[1]))
        return out

    @torch.no_grad()
    def load_from(self, values: dict) -> None:
        """``values``: FlatState.to_numpy() (conv weights OHWI)."""
        for n, conv, bn in self._convbn():
            conv.weight.copy_(torch.as_tensor(values[f"{n}.conv.weight"]).permute(0, 3, 1, 2))
            bn.weight.copy_(torch.as_tensor(values[f"{n}.bn.gamma"]))
            bn.bias.copy_(torch.as_tensor(values[f"{n}.bn.beta"]))
            bn.running_mean.copy_(torch.as_tensor(values[f"{n}.bn.moving_mean"]))
            bn.running_var.copy_(torch.as_tensor(values[f"{n}.bn.moving_variance"]))
        self.fc.weight.copy_(torch.as_tensor(values["fc.kernel"]))
        self.fc.bias.copy_(torch.as_tensor(values["fc.bias"]))

    def grads(self) -> dict:
        """Gradients keyed by framework variable name (conv weights OHWI)."""
        g = {}
        for n, conv, bn in self._convbn():
            g[f"{n}.conv.weight"] = conv.weight.grad.permute(0, 2, 3, 1).contiguous()
            g[f"{n}.bn.gamma"] = bn.weight.grad
            g[f"{n}.bn.beta"] = bn.bias.grad
        g["fc.kernel"] = self.fc.weight.grad
        g["fc.bias"] = self.fc.bias.grad
        return g

    def running_stats(self) -> dict:
        r = {}
        for n, _, bn in self._convbn():
            r[f"{n}.bn.moving_mean"] = bn.running_mean
            r[f"{n}.bn.moving_variance"] = bn.running_var
        return r


def reference_step(values: dict, x_nhwc8: torch.Tensor, labels: torch.Tensor, dtype=torch.float64,
                   relu_masks: dict | None = None, flips: list | None = None):
    """One training-mode forward/backward of the oracle: returns (loss, grads,
    running stats after the step).  ``relu_masks``: see ``pin_relu_masks``;
    ``flips`` (a one-element list) receives how many pinned mask elements
    disagreed with the oracle's own pre-activation signs."""
    m = TorchResNet18().to(dtype)
    m.load_from(values)
    m.pin_relu_masks(relu_masks)
    m.train()
    x = x_nhwc8.to(dtype).permute(0, 3, 1, 2).contiguous()
    logits = m(x)
    loss = F.cross_entropy(logits, labels.long())
    loss.backward()
    if flips is not None:
        flips[0] = m.flips[0]
    return float(loss.detach()), m.grads(), m.running_stats()
