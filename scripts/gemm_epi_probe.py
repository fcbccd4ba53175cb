"""Large-tile GEMM fixed costs: the BERT ffn1 output shape (16384 x 3072) at
K = 64 / 128 / 256 / 768 -- the K -> 0 intercept is prologue + epilogue."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.ops._native import ops
from scripts.gemm_micro import graph_us


def main():
    o = ops()
    M, N = 16384, 3072
    for K in (64, 128, 256, 768):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        b = torch.zeros(N, device="cuda")
        r = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        for name, fn in (("plain", lambda: o.gemm_fwd(x, w, y, None, None, None, M, N, K)),
                         ("bias", lambda: o.gemm_fwd(x, w, y, b, None, None, M, N, K)),
                         ("bias+resid", lambda: o.gemm_fwd(x, w, y, b, r, None, M, N, K))):
            us = graph_us(fn)
            print(f"K={K:4d} {name:10s} {us:7.1f} us  {2.0 * M * N * K / us / 1e6:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
