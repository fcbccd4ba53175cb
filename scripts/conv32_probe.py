"""Targeted conv32 timing probe: for chosen layers, time fwd / dgrad / wgrad
under forced plans (BM, BN, split) and debug modes (MFL_C32_DBG: 1 = no
MFMA, 2 = no operand DMA, 3 = neither) -- to see whether a configuration is
bound by the matrix pipe, the LDS-DMA stream or its fixed costs.
python scripts/conv32_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from metisfl_amd.ops import nn as K  # noqa: E402
from metisfl_amd.ops.nn import ConvShape  # noqa: E402
from scripts.conv32_bench import timed  # noqa: E402

CASES = [  # (shape, mode, [(bm, bn, split)])
    ((32, 4, 4, 512, 512, 3, 1), 0, [(64, 64, 4), (64, 64, 8), (64, 64, 12), (64, 64, 16), (128, 64, 8), (64, 128, 8)]),
    ((32, 32, 32, 64, 64, 3, 1), 0, [(128, 64, 1), (64, 64, 1), (64, 64, 2), (128, 64, 2)]),
    ((32, 16, 16, 128, 128, 3, 1), 1, [(64, 64, 1), (64, 64, 2), (64, 64, 3), (128, 64, 2)]),
    ((32, 32, 32, 64, 64, 3, 1), 2, [(64, 64, 28), (64, 64, 56), (128, 64, 28), (64, 128, 28)]),
]


def main():
    dev = torch.device("cuda")
    ws = torch.zeros(32 << 20, device=dev)
    for t, mode, plans in CASES:
        N, H, W, C, Co, k, s = t
        shp = ConvShape(N, H, W, C, Co, k, k, s, k // 2)
        x = torch.randn(N, H, W, C, device=dev)
        w = torch.randn(Co, k, k, C, device=dev) * 0.05
        y = torch.zeros(N, shp.P, shp.Q, Co, device=dev)
        st = torch.zeros(8 * 2 * Co, dtype=torch.float64, device=dev)
        dy = torch.randn(N, shp.P, shp.Q, Co, device=dev)
        dx = torch.zeros(N, H, W, C, device=dev)
        dw = torch.zeros(Co, k, k, C, device=dev)
        flop = 2.0 * N * shp.P * shp.Q * Co * k * k * C
        run = {0: lambda: K.conv_forward(x, w, y, shp, ws, st),
               1: lambda: K.conv_dgrad(dy, w, dx, shp, ws, False),
               2: lambda: K.conv_wgrad(x, dy, dw, shp, accumulate=True)}[mode]
        for bm, bn, sp in plans:
            os.environ.update(MFL_C32_BM=str(bm), MFL_C32_BN=str(bn), MFL_C32_SPLIT=str(sp))
            p = K.conv_plan(mode, shp, dev, torch.float32)
            if p.splits != sp or p.kchunk == 0:
                print(f"{'fdw'[mode]} {'x'.join(map(str, t))} {bm}x{bn} s{sp}: infeasible")
                continue
            res = []
            for dbg in (0, 1, 2, 3):
                os.environ["MFL_C32_DBG"] = str(dbg)
                res.append(timed(run, 30))
            os.environ["MFL_C32_DBG"] = "0"
            print(f"{'fdw'[mode]} {'x'.join(map(str, t)):22s} {bm}x{bn} s{sp:<3d} full {res[0]:6.1f} "
                  f"({flop / res[0] / 1e6:5.1f} TF)  dma-only {res[1]:6.1f}  mfma-only {res[2]:6.1f}  "
                  f"skeleton {res[3]:6.1f} us", flush=True)
    for k_ in ("MFL_C32_BM", "MFL_C32_BN", "MFL_C32_SPLIT"):
        os.environ.pop(k_, None)


if __name__ == "__main__":
    main()
