"""Learner shards for federated experiments (reference:
examples/utils/data_partitioning.py:8-124): IID, non-IID with a fixed number
of classes per learner, and Dirichlet label skew."""
from __future__ import annotations

import numpy as np


class DataPartitioning:

    def __init__(self, x_train, y_train, partitions_num: int, seed: int = 1990):
        self.x = np.asarray(x_train)
        self.y = np.asarray(y_train)
        self.n = partitions_num
        self.rng = np.random.default_rng(seed)

    def _split(self, groups):
        xs = [self.x[g] for g in groups]
        ys = [self.y[g] for g in groups]
        return xs, ys

    def iid_partition(self):
        """Shuffle and split into ``n`` near-equal shards."""
        idx = self.rng.permutation(len(self.y))
        return self._split(np.array_split(idx, self.n))

    def non_iid_partition(self, classes_per_partition: int = 2):
        """Every learner sees ``classes_per_partition`` classes; each class is
        split evenly among the learners holding it."""
        classes = np.unique(self.y)
        if classes_per_partition > len(classes):
            raise ValueError("more classes per partition than classes")
        # round-robin assignment of classes to partitions
        order = self.rng.permutation(classes)
        owners: dict = {c: [] for c in classes}
        assign = []
        k = 0
        for p in range(self.n):
            mine = [order[(k + j) % len(order)] for j in range(classes_per_partition)]
            k += classes_per_partition
            assign.append(mine)
            for c in mine:
                owners[c].append(p)
        groups = [[] for _ in range(self.n)]
        for c, ps in owners.items():
            if not ps:
                continue
            idx = self.rng.permutation(np.nonzero(self.y == c)[0])
            for p, part in zip(ps, np.array_split(idx, len(ps))):
                groups[p].extend(part.tolist())
        return self._split([np.asarray(sorted(g), dtype=np.int64) for g in groups])

    def dirichlet_based_partition(self, a: float = 0.5):
        """Label skew: per class, learner proportions ~ Dirichlet(a)."""
        groups = [[] for _ in range(self.n)]
        for c in np.unique(self.y):
            idx = self.rng.permutation(np.nonzero(self.y == c)[0])
            p = self.rng.dirichlet([a] * self.n)
            cuts = (np.cumsum(p) * len(idx)).astype(int)[:-1]
            for g, part in zip(groups, np.split(idx, cuts)):
                g.extend(part.tolist())
        return self._split([np.asarray(sorted(g), dtype=np.int64) for g in groups])

    @staticmethod
    def to_json_representation(ys) -> dict:
        out = {}
        for i, y in enumerate(ys):
            cls, cnt = np.unique(np.asarray(y), return_counts=True)
            out[i] = {int(c): int(n) for c, n in zip(cls, cnt)}
        return out
