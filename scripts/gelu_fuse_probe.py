"""FFN1 backward at BERT-base size: dgrad + streaming gelu_bwd (+ bias colsum)
against the fused gemm_dgrad_gelu epilogue, graph-replay timed."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.ops import bert as BO
from scripts.gemm_micro import graph_us


def main():
    M, N, K = 16384, 768, 3072  # dy [M][768] . W1^T-side [768][3072] -> dz [M][3072]
    dy = ((torch.rand(M, N, device="cuda") * 2 - 1)).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
    z = ((torch.rand(M, K, device="cuda") * 4 - 2)).bfloat16()
    dh = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    dz = torch.empty_like(dh)
    db = torch.zeros(K, device="cuda")

    def unfused():
        BO.gemm_dgrad(dy, w, dh, M, N, K)
        BO.gelu_bwd(dh, z, dz, M, K, dbias=db)

    def fused():
        BO.gemm_dgrad_gelu(dy, w, dz, z, M, N, K, dbias=db)

    def dgrad_only():
        BO.gemm_dgrad(dy, w, dh, M, N, K)

    for name, fn in (("dgrad", dgrad_only), ("unfused", unfused), ("fused", fused), ("unfused", unfused),
                     ("fused", fused)):
        print(f"{name:8s} {graph_us(fn):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
