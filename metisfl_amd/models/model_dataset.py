"""Dataset wrappers handed to the learner (same public classes as the
reference, metisfl/models/model_dataset.py:4-71).  ``x`` / ``y`` are host
arrays; the learner uploads them ONCE to device memory (DeviceDataset) and
keeps the shard resident across rounds."""
from __future__ import annotations

import numpy as np


class ModelDataset:
    def __init__(self, x=None, y=None, size: int = 0):
        self._x = x
        self._y = y
        self._size = int(size if size else (len(x) if x is not None else 0))

    def get_x(self, *args, **kwargs):
        return self._x

    def get_y(self, *args, **kwargs):
        return self._y

    def get_size(self, *args, **kwargs) -> int:
        return self._size

    def get_model_dataset_specifications(self, *args, **kwargs) -> dict:
        return {}


class ModelDatasetClassification(ModelDataset):
    def __init__(self, x=None, y=None, size: int = 0, examples_per_class: dict | None = None):
        super().__init__(x, y, size)
        if examples_per_class is None and y is not None:
            cls, cnt = np.unique(np.asarray(y).reshape(-1), return_counts=True)
            examples_per_class = {int(c): int(n) for c, n in zip(cls, cnt)}
        self.examples_per_class = dict(examples_per_class or {})

    def get_model_dataset_specifications(self, *args, **kwargs) -> dict:
        return self.examples_per_class


class ModelDatasetRegression(ModelDataset):
    def __init__(self, x=None, y=None, size: int = 0, min_val=0.0, max_val=0.0, mean_val=0.0,
                 median_val=0.0, mode_val=0.0, stddev_val=0.0):
        super().__init__(x, y, size)
        self.min_val, self.max_val, self.mean_val = min_val, max_val, mean_val
        self.median_val, self.mode_val, self.stddev = median_val, mode_val, stddev_val

    @classmethod
    def from_arrays(cls, x, y):
        yy = np.asarray(y, dtype=np.float64).reshape(-1)
        vals, cnt = np.unique(yy, return_counts=True)
        return cls(x, y, len(yy), float(yy.min()), float(yy.max()), float(yy.mean()),
                   float(np.median(yy)), float(vals[np.argmax(cnt)]), float(yy.std()))

    def get_model_dataset_specifications(self, *args, **kwargs) -> dict:
        return {"min": self.min_val, "max": self.max_val, "mean": self.mean_val,
                "median": self.median_val, "mode": self.mode_val, "stddev": self.stddev}
