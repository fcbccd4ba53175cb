import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Under pytest-xdist every worker (and the learner/controller processes its
# tests spawn) would otherwise start one OpenMP thread per core: six workers
# on 8 cores oversubscribe 6x, and the spin-waiting OpenMP barriers turn a
# 25 s CPU federation into a >10 min one.  Share the cores instead.
_workers = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1") or 1)
if _workers > 1 and "OMP_NUM_THREADS" not in os.environ:
    os.environ["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // _workers))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
