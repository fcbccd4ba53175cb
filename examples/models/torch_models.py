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
MelanomaFC (melanoma_fc.py) needs ImageNet-pretrained Xception weights,
which cannot be fetched here; it is not provided.
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
