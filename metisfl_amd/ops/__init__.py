"""Hand-written HIP/CDNA4 kernels of metisfl_amd and their Python entry points."""
from metisfl_amd.ops._native import available, ops  # noqa: F401
from metisfl_amd.ops import aggregate, nn, optim  # noqa: F401
