"""LayerNorm-backward microbenchmark at the BERT shape (16384 x 768)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.ops import bert as BO


def main():
    M, H = 16384, 768
    x = (torch.randn(M, H, device="cuda") * 2).bfloat16()
    dy = torch.randn(M, H, device="cuda").bfloat16()
    gam, bet = torch.rand(H, device="cuda") + 0.5, torch.randn(H, device="cuda")
    y = torch.empty_like(x)
    mean, rstd = torch.zeros(M, device="cuda"), torch.zeros(M, device="cuda")
    BO.ln_fwd(x, gam, bet, y, mean, rstd, M, H, 1e-12)
    dx, dx2 = torch.empty_like(x), torch.empty_like(x)
    dg, db, dbp = (torch.zeros(H, device="cuda") for _ in range(3))
    fn = lambda: BO.ln_bwd(dy, x, mean, rstd, gam, dx, dg, db, M, H, dx2=dx2, dbias_prev=dbp)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"blocks={os.environ.get('MFL_LN_BWD_BLOCKS', '256')} ln_bwd {us:.1f} us  ({100e6 / us / 1e6:.2f} TB/s)")


if __name__ == "__main__":
    main()
