"""Scaling-factor semantics of the reference's controller scalers.

Canonical implementation lives in the C++ engine (csrc/engine/policies.h);
this host mirror exists for engine-less use and for cross-checking in tests.
Reference: scaling/batches_scaler.cc:7-50, participants_scaler.cc:7-43,
train_dataset_size_scaler.cc:7-50.  Quirk kept: a
federation of exactly one learner gets 1.0, but a single participant among
several learners gets its RAW value (examples / batches), not 1.0.
"""
from __future__ import annotations

import numpy as np


def compute(kind: str, num_train, completed_batches, num_all_learners: int) -> list[float]:
    kind = kind.upper()
    n = len(num_train)
    if n == 0:
        return []
    if num_all_learners == 1:
        return [1.0] * n
    if kind == "NUM_PARTICIPANTS":
        return [1.0] if n == 1 else [1.0 / n] * n
    v = np.asarray(completed_batches if kind == "NUM_COMPLETED_BATCHES" else num_train,
                   dtype=np.float64)
    if n == 1:
        return [float(v[0])]
    tot = float(np.sum(v.astype(np.int64)))
    return [float(x) / tot for x in v]
