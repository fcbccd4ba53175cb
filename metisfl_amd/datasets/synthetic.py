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


MASK_ID = 103  # [MASK] in the BERT uncased vocabulary


def synthetic_mlm(n: int, seq: int = 128, max_pred: int = 20, vocab: int = 30522, seed: int = 0,
                  rec_stride: int | None = None) -> np.ndarray:
    """Masked-LM records for ``models.bert.BertMLM``: int32 rows
    ``[tokens seq | masked positions max_pred | original ids max_pred |
    inverse map seq (slot or -1) | pad]``.  Token streams follow a fixed
    random bigram chain (so the model has something to learn); ``max_pred``
    distinct positions per sequence (never position 0, the [CLS] slot) are
    replaced by [MASK]."""
    rng = np.random.default_rng(seed)
    stride = rec_stride or ((2 * seq + 2 * max_pred + 3) // 4 * 4)
    lo = min(1000, vocab // 2)
    nxt = np.random.default_rng(777).integers(lo, vocab, size=vocab)
    rec = np.zeros((n, stride), dtype=np.int32)
    tok = np.empty((n, seq), dtype=np.int64)
    tok[:, 0] = 101  # [CLS]
    cur = rng.integers(lo, vocab, size=n)
    for t in range(1, seq):
        jump = rng.random(n) < 0.2
        cur = np.where(jump, rng.integers(lo, vocab, size=n), nxt[cur])
        tok[:, t] = cur
    pos = np.argsort(rng.random((n, seq - 1)), axis=1)[:, :max_pred] + 1
    pos.sort(axis=1)
    ids = np.take_along_axis(tok, pos, axis=1)
    masked = tok.copy()
    np.put_along_axis(masked, pos, MASK_ID, axis=1)
    inv = np.full((n, seq), -1, dtype=np.int64)
    np.put_along_axis(inv, pos, np.broadcast_to(np.arange(max_pred), pos.shape), axis=1)
    rec[:, :seq] = masked
    rec[:, seq:seq + max_pred] = pos
    rec[:, seq + max_pred:seq + 2 * max_pred] = ids
    rec[:, seq + 2 * max_pred:2 * seq + 2 * max_pred] = inv
    return rec
