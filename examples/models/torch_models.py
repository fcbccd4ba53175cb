"""User-model examples on the TorchModelDef path: the
reference's Keras neuroimaging CNNs, IMDB LSTM and PyTorch MLP expressed as
torch ``nn.Module``s.  TorchModelOps trains them on the GPU with the fused
flat-buffer HIP optimizer; the layers themselves are PyTorch-ROCm ops (these
are user models, not framework hot paths).

Reference architectures (studied, not copied):
  * BrainAge2DCNN / BrainAge3DCNN -- examples/keras/models/brainage_cnns.py:
    stacked [conv3 + BN(instance-style) + ReLU + conv3 + BN + ReLU + maxpool2]
    blocks (32..256 filters), a 1x1 projection, average pooling, regression
    head initialised at the cohort mean age (62.68).
  * AlzheimersDisease2D/3D -- alzheimers_disease_cnns.py: the same trunk with
    a sigmoid classification head.
  * ImdbLSTM -- imdb_lstm.py: embedding + LSTM + dense sigmoid.
  * IonosphereMLP -- examples/pytorch/models/mlp.py: MLP 34-10-8-1 (sigmoid).
  * MelanomaFC -- melanoma_fc.py: a FROZEN Xception trunk (entry / 8x middle
    / exit flow of depthwise-separable convolutions with residual 1x1
    projections), global average pooling, Dense 8 + ReLU, Dropout 0.7,
    Dense 1 + sigmoid, binary cross-entropy.  The reference loads
    ImageNet weights into the trunk; none can be fetched here, so the trunk
    is random-init unless ``trunk_weights`` names a local state dict
    (loaded with ``torch.load(weights_only=True)``) -- parity unpinned.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from metisfl_amd.models.model_def import TorchModelDef


def _block(conv, bn, pool, cin, cout):
    return nn.Sequential(conv(cin, cout, 3, padding=1), bn(cout, affine=False), nn.ReLU(inplace=True),
                         conv(cout, cout, 3, padding=1), bn(cout, affine=False), nn.ReLU(inplace=True),
                         pool(2, 2))


class _NeuroCNN(nn.Module):
    def __init__(self, dims: int, filters=(32, 64, 128, 256), out: int = 1, bias0: float = 0.0):
        super().__init__()
        conv, bn, pool, avg = ((nn.Conv2d, nn.BatchNorm2d, nn.MaxPool2d, nn.AdaptiveAvgPool2d) if dims == 2 else
                               (nn.Conv3d, nn.BatchNorm3d, nn.MaxPool3d, nn.AdaptiveAvgPool3d))
        layers, cin = [], 1
        for f in filters:
            layers.append(_block(conv, bn, pool, cin, f))
            cin = f
        self.trunk = nn.Sequential(*layers)
        self.proj = nn.Sequential(conv(cin, 64, 1), bn(64, affine=False), nn.ReLU(inplace=True))
        self.pool = avg(1)
        self.head = nn.Linear(64, out)
        nn.init.constant_(self.head.bias, bias0)

    def forward(self, x):
        return self.head(self.pool(self.proj(self.trunk(x))).flatten(1))


class BrainAge2DCNN(TorchModelDef):
    """Brain-age regression from 2D MRI slices (MSE on years)."""

    def __init__(self, filters=(32, 64, 128, 256)):
        self.filters = filters

    def get_model(self):
        return _NeuroCNN(2, self.filters, 1, 62.68)

    def loss(self, outputs, targets):
        return F.mse_loss(outputs[:, 0], targets.float())


class BrainAge3DCNN(BrainAge2DCNN):
    def get_model(self):
        return _NeuroCNN(3, self.filters, 1, 62.68)


class AlzheimersDisease2DCNN(TorchModelDef):
    def __init__(self, filters=(32, 64, 128, 256)):
        self.filters = filters

    def get_model(self):
        return _NeuroCNN(2, self.filters, 2)


class AlzheimersDisease3DCNN(AlzheimersDisease2DCNN):
    def get_model(self):
        return _NeuroCNN(3, self.filters, 2)


class _LSTMClassifier(nn.Module):
    def __init__(self, vocab: int, emb: int, hidden: int):
        super().__init__()
        self.emb = nn.Embedding(vocab, emb)
        self.lstm = nn.LSTM(emb, hidden, batch_first=True)
        self.out = nn.Linear(hidden, 2)

    def forward(self, x):
        h, _ = self.lstm(self.emb(x.long()))
        return self.out(h[:, -1])


class ImdbLSTM(TorchModelDef):
    """Sentiment classification (IMDB-shaped token ids, 2 classes)."""

    def __init__(self, vocab: int = 10000, emb: int = 64, hidden: int = 64):
        self.vocab, self.emb, self.hidden = vocab, emb, hidden

    def get_model(self):
        return _LSTMClassifier(self.vocab, self.emb, self.hidden)


class IonosphereMLP(TorchModelDef):
    """MLP 34-10-8-2 (the reference's binary MLP with a 2-logit head)."""

    def get_model(self):
        return nn.Sequential(nn.Linear(34, 10), nn.ReLU(), nn.Linear(10, 8), nn.ReLU(), nn.Linear(8, 2))


def synthetic_volumes(n: int, shape, seed: int = 0, classes: int | None = None):
    """MRI-shaped synthetic inputs (N, 1, *shape) with ages or labels."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((n, 1) + tuple(shape), generator=g)
    if classes:
        y = (x.mean(dim=tuple(range(1, x.dim()))) > 0).long()
    else:
        y = 62.68 + 10 * x.mean(dim=tuple(range(1, x.dim()))) * 30
    return x.numpy(), y.numpy()


# ---------------------------------------------------------------------------
class _SepConv(nn.Sequential):
    """Depthwise 3x3 + pointwise 1x1 (Keras SeparableConv2D, no bias) + BN."""

    def __init__(self, cin, cout, relu_first=True):
        layers = [nn.ReLU(inplace=False)] if relu_first else []
        layers += [nn.Conv2d(cin, cin, 3, padding=1, groups=cin, bias=False),
                   nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout)]
        super().__init__(*layers)


class _XBlock(nn.Module):
    """Residual block: [sepconv]*reps (+ maxpool s2) + 1x1 s2 projection."""

    def __init__(self, cin, cout, reps, stride, relu_first=True, grow_first=True):
        super().__init__()
        chans = [cin] + ([cout] * reps if grow_first else [cin] * (reps - 1) + [cout])
        seq = [_SepConv(chans[i], chans[i + 1], relu_first=(i > 0 or relu_first)) for i in range(reps)]
        if stride != 1:
            seq.append(nn.MaxPool2d(3, stride, padding=1))
        self.body = nn.Sequential(*seq)
        self.skip = None if (cin == cout and stride == 1) else nn.Sequential(
            nn.Conv2d(cin, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        return self.body(x) + (x if self.skip is None else self.skip(x))


class Xception(nn.Module):
    """Xception feature extractor (Chollet 2017; keras.applications.Xception
    with include_top=False): 2048 channels at 1/32 resolution."""

    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 32, 3, 2, bias=False), nn.BatchNorm2d(32), nn.ReLU(),
                                  nn.Conv2d(32, 64, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU())
        blocks = [_XBlock(64, 128, 2, 2, relu_first=False), _XBlock(128, 256, 2, 2), _XBlock(256, 728, 2, 2)]
        blocks += [_XBlock(728, 728, 3, 1) for _ in range(8)]
        blocks += [_XBlock(728, 1024, 2, 2, grow_first=False)]
        self.blocks = nn.Sequential(*blocks)
        self.exit = nn.Sequential(_SepConv(1024, 1536, relu_first=False), nn.ReLU(),
                                  _SepConv(1536, 2048, relu_first=False), nn.ReLU())

    def forward(self, x):
        return self.exit(self.blocks(self.stem(x)))


class _MelanomaNet(nn.Module):
    def __init__(self, trunk_weights: str | None):
        super().__init__()
        self.trunk = Xception()
        if trunk_weights:
            self.trunk.load_state_dict(torch.load(trunk_weights, map_location="cpu", weights_only=True))
        for p in self.trunk.parameters():  # base_model.trainable = False
            p.requires_grad_(False)
        self.head = nn.Sequential(nn.Linear(2048, 8), nn.ReLU(), nn.Dropout(0.7), nn.Linear(8, 1))

    def forward(self, x):
        # preprocess_input: [0, 255] -> [-1, 1]; the frozen trunk keeps its BN statistics
        self.trunk.eval()
        f = self.trunk(x / 127.5 - 1.0)
        return self.head(f.mean(dim=(2, 3))).squeeze(-1)


class MelanomaFC(TorchModelDef):
    """Binary melanoma classifier: frozen Xception + small dense head
    (logit output; the loss applies the sigmoid)."""

    def __init__(self, image_size=(1024, 1024), trunk_weights: str | None = None):
        self.image_size = tuple(image_size)
        self.trunk_weights = trunk_weights

    def get_model(self):
        return _MelanomaNet(self.trunk_weights)

    def loss(self, outputs, targets):
        return F.binary_cross_entropy_with_logits(outputs, targets.float())
