"""metisfl_amd: an MI355X-native federated learning framework.

Same capabilities as MetisFL (controller / learner / driver roles, the
``metisfl`` protobuf wire format, sync / semi-sync / async protocols, FedAvg /
FedStride / FedRec / CKKS-PWA aggregation), re-designed for AMD Instinct
MI355X: learners are persistent per-GPU processes whose training step runs on
hand-written gfx950 HIP kernels, and aggregation is an RCCL collective over
xGMI.
"""
__version__ = "0.1.0"


def _share_hip_runtime() -> None:
    """One HIP runtime per process.

    Both torch's bundled ``libamdhip64.so`` and ROCm's ``/opt/rocm/lib/
    libamdhip64.so.7`` carry the soname ``libamdhip64.so.7``.  The native
    extensions (``_engine``: the controller's device aggregation, ``_ops``)
    link against that soname; if one of them is loaded before torch, ROCm's
    copy comes in, torch later loads its own, and whichever runtime
    initialises second sees no device.  Loading torch's copy first (by path,
    without importing torch) makes every later ``libamdhip64.so.7`` lookup --
    and torch's own -- resolve to the same object."""
    import ctypes
    import importlib.util
    import os

    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.origin:
        return
    lib = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(lib):
        try:
            ctypes.CDLL(lib, mode=ctypes.RTLD_GLOBAL)
        except OSError:
            pass


_share_hip_runtime()
