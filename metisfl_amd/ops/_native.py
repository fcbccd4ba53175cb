"""Loader for the in-tree HIP kernel extension ``metisfl_amd._ops``.

Device tensors are ALWAYS served by the hand-written gfx950 kernels: if the
extension is missing on a machine with a GPU, :func:`ops` raises instead of
silently falling back to eager PyTorch.  CPU tensors (the host-only test
path) use the plain-PyTorch reference implementations in the sibling modules,
which are also what the GPU numerics tests compare against.
"""
from __future__ import annotations

import importlib

_MOD = None
_ERR: Exception | None = None


def ops():
    global _MOD, _ERR
    if _MOD is not None:
        return _MOD
    try:
        _MOD = importlib.import_module("metisfl_amd._ops")
    except Exception as e:  # pragma: no cover - exercised on a box without a build
        _ERR = e
        raise RuntimeError(
            "metisfl_amd._ops (HIP kernels) is not built or failed to load: "
            f"{e!r}. Run `python -m metisfl_amd.csrc.build` (hipcc, gfx950).") from e
    return _MOD


def available() -> bool:
    try:
        ops()
        return True
    except RuntimeError:
        return False
