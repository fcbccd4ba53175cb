"""Which HIP runtime does the controller engine bind to when torch is (or is
not) initialised first in the same process?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l})


order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch cuda", torch.cuda.is_available(), torch.cuda.device_count())
from metisfl_amd import _engine as E
print("engine avail", E.device_aggregation_available(), E.device_aggregation_stats())
if order == "engine_first":
    import torch
    print("torch cuda", torch.cuda.is_available(), torch.cuda.device_count())
print("maps", maps())
