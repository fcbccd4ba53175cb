"""Tracing / observability.

The reference's only trace is the controller's ``FederatedTaskRuntimeMetadata``
(metis.proto:342-365, recorded at controller.cc:406-1004) and the Keras
PerformanceProfiler callback (models/keras/callbacks/performance_profiler.py:
5-63); it has no profiler integration.  Here:

* ``range(name)`` -- a roctx range (``libroctx64``) around a host phase
  (local steps, scale, all-reduce, eval), so ``rocprofv3 --marker-trace``
  timelines show federation phases next to the HIP kernels.  A no-op when the
  library is absent (CPU containers) or ``METISFL_AMD_ROCTX=0``.
* ``JsonlLog`` -- one JSON object per federation round (the runtime metadata
  plus rounds/s, all-reduce GB/s and HBM usage), append-only so a crashed
  run keeps everything up to its last round.
* ``hbm_usage()`` -- device memory in use / total (``hipMemGetInfo``).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time

_LIB = None
_LOCK = threading.Lock()


def _roctx():
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                lib = False
                if os.environ.get("METISFL_AMD_ROCTX", "1") != "0":
                    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so", "libroctx64.so.4"):
                        try:
                            lib = ctypes.CDLL(name)
                            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                            lib.roctxRangePushA.restype = ctypes.c_int
                            lib.roctxRangePop.restype = ctypes.c_int
                            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                            break
                        except OSError:
                            lib = False
                _LIB = lib
    return _LIB or None


def roctx_available() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx verb
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


def hbm_usage(device=None) -> dict:
    """{"used_bytes", "total_bytes"} of a HIP device ({} on CPU)."""
    try:
        import torch
        if not torch.cuda.is_available():
            return {}
        free, total = torch.cuda.mem_get_info(device)
        return {"used_bytes": int(total - free), "total_bytes": int(total)}
    except Exception:  # pragma: no cover
        return {}


class JsonlLog:
    """Append-only JSON-lines log (one object per line, flushed per write)."""

    def __init__(self, path: str | None):
        self.path = path
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def write(self, obj: dict) -> None:
        if not self.path:
            return
        obj = dict(obj)
        obj.setdefault("logged_at", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(obj, default=_default) + "\n")

    @staticmethod
    def read(path: str) -> list[dict]:
        with open(path) as f:
            return [json.loads(line) for line in f if line.strip()]


def _default(o):
    try:
        import numpy as np
        if isinstance(o, np.ndarray):
            return o.tolist()
        if isinstance(o, (np.floating, np.integer)):
            return o.item()
    except Exception:  # pragma: no cover
        pass
    return str(o)
