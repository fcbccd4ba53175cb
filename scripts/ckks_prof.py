"""Whole-model CKKS secure aggregation on one GPU (ResNet-18 size) for
rocprofv3: keygen on the host, then 5 x (device encrypt -> scale -> decrypt)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.encryption import CKKS
from metisfl_amd.encryption.device import DeviceCKKS
from metisfl_amd.parallel.comm import Comm


def main():
    c = CKKS(4096, 52)
    c.gen_crypto_context_and_keys(tempfile.mkdtemp())
    d = DeviceCKKS(c, "cuda")
    theta = torch.randn(11_173_962, device="cuda") * 0.05
    ref = theta.clone()
    comm = Comm()
    ct = torch.empty(d.ct_numel(theta.numel()), dtype=torch.int64, device="cuda")
    for i in range(5):
        t = d.secure_weighted_allreduce(comm, theta, 1.0, ct=ct)
        print(i, {k: round(v, 3) for k, v in t.items()}, flush=True)
    print("max err", float((theta - ref).abs().max()))


if __name__ == "__main__":
    main()
