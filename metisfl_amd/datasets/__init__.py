"""Data partitioning and synthetic datasets for federated experiments."""
from metisfl_amd.datasets.partitioning import DataPartitioning  # noqa: F401
from metisfl_amd.datasets.synthetic import (  # noqa: F401
    synthetic_classification, synthetic_mlm, synthetic_regression)
