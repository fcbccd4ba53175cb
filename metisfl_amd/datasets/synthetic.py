"""Synthetic datasets with the shapes of the reference's example datasets
(no network access: CIFAR-10 / FashionMNIST / Boston housing are not
downloadable here).  Labels are a fixed function of the inputs so models can
actually learn."""
from __future__ import annotations

import numpy as np

SHAPES = {"cifar10": (32, 32, 3), "fashionmnist": (28, 28), "housing": (13,)}


def synthetic_classification(name: str, n: int, num_classes: int = 10, seed: int = 0):
    rng = np.random.default_rng(seed)
    shape = SHAPES[name]
    x = rng.standard_normal((n,) + shape).astype(np.float32)
    proj = np.random.default_rng(1234).standard_normal((int(np.prod(shape)), num_classes)).astype(np.float32)
    y = (x.reshape(n, -1) @ proj).argmax(1).astype(np.int64)
    return x, y


def synthetic_regression(n: int, features: int = 13, seed: int = 0):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, features)).astype(np.float32)
    w = np.random.default_rng(4321).standard_normal(features).astype(np.float32)
    return x, (x @ w + 0.1 * rng.standard_normal(n)).astype(np.float32)
