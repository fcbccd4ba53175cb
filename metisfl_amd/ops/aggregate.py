"""Model-aggregation ops (K1 weighted sum, K2 rolling merge/scale, K8 zero
counts, K9 CKKS private weighted average) over flat device buffers.

Numerics follow the reference exactly (federated_average.cc:14-37,
federated_rolling_average_base.cc:18-171): every scaled term is
``(T)((double)x * w)`` -- integer tensors truncate per term, fp32 tensors
round per term -- and terms are accumulated in T in learner order.
"""
from __future__ import annotations

import numpy as np
import torch

from metisfl_amd.ops._native import ops

MERGE_ADD, MERGE_SUB, SCALE_MUL, SCALE_DIV = range(4)


def _np_term(x: np.ndarray, w: float) -> np.ndarray:
    prod = x.astype(np.float64) * w
    if np.issubdtype(x.dtype, np.integer):
        info = np.iinfo(x.dtype)
        t = np.trunc(prod)
        # C++ double->T conversion truncates; wrap like the narrowing add does
        return (t.astype(np.int64) if info.min < 0 else t.astype(np.uint64)).astype(x.dtype)
    return prod.astype(x.dtype)


def weighted_sum_np(xs: list[np.ndarray], ws: list[float]) -> np.ndarray:
    """Host reference of K1 (bit-exact to the reference's FedAvg)."""
    out = np.zeros_like(xs[0])
    with np.errstate(over="ignore"):
        for x, w in zip(xs, ws):
            out = (out + _np_term(x, w)).astype(xs[0].dtype)
    return out


def weighted_sum(out: torch.Tensor, xs: list[torch.Tensor], ws: list[float]) -> None:
    if out.is_cuda:
        ops().weighted_sum(out, list(xs), [float(w) for w in ws])
        return
    res = weighted_sum_np([x.numpy() for x in xs], list(ws))
    out.copy_(torch.from_numpy(res))


def rolling_op(y: torch.Tensor, x: torch.Tensor | None, op: int, w: float) -> None:
    if y.is_cuda:
        ops().rolling_op(y, x, op, float(w))
        return
    yn = y.numpy()
    with np.errstate(over="ignore"):
        if op == MERGE_ADD:
            r = yn + _np_term(x.numpy(), w)
        elif op == MERGE_SUB:
            r = yn - _np_term(x.numpy(), w)
        elif op == SCALE_MUL:
            r = _np_term(yn, w)
        else:  # (T)((double)y / z)
            r = yn.astype(np.float64) / w
            if np.issubdtype(yn.dtype, np.integer):
                r = np.trunc(r).astype(np.int64)
    y.copy_(torch.from_numpy(np.asarray(r).astype(yn.dtype)))


def count_zeros(x: torch.Tensor, segments: list[tuple[int, int]]) -> list[int]:
    """Zero counts of ``x[beg:end]`` for every (beg, end) segment, one launch."""
    if not x.is_cuda:
        return [int((x[b:e] == 0).sum()) for b, e in segments]
    tile = 1 << 16
    seg, beg, end = [], [], []
    for i, (b, e) in enumerate(segments):
        for s in range(b, e, tile):
            seg.append(i)
            beg.append(s)
            end.append(min(e, s + tile))
    dev = x.device
    counts = torch.zeros(len(segments), dtype=torch.int64, device=dev)
    if seg:
        ops().count_zeros(x, torch.tensor(seg, dtype=torch.int64, device=dev),
                          torch.tensor(beg, dtype=torch.int64, device=dev),
                          torch.tensor(end, dtype=torch.int64, device=dev), counts)
    return counts.cpu().tolist()
