"""Upper bound of running a layer's wgrad beside its dgrad (ResNet-18 CIFAR
shapes, batch 32): a graph of 20 (wgrad, dgrad) pairs in sequence, against
the 20 wgrads on one captured stream and the 20 dgrads on another with no
joins between pairs (maximum overlap, not a legal training schedule)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.ops import nn as K

SHAPES = [(32, 32, 32, 64, 64, 3, 1), (32, 16, 16, 128, 128, 3, 1), (32, 8, 8, 256, 256, 3, 1),
          (32, 4, 4, 512, 512, 3, 1)]


def timed(g):
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / 3


def main(iters=20):
    dev = torch.device("cuda")
    for (N, H, W, C, Co, k, s) in SHAPES:
        shp = K.ConvShape(N, H, W, C, Co, k, k, s, k // 2)
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, k, k, C, device=dev) * 0.05).bfloat16()
        dy = torch.randn(N, shp.P, shp.Q, Co, device=dev).bfloat16()
        dx = torch.empty_like(x)
        dw = torch.zeros(Co, k, k, C, device=dev)
        ws = torch.zeros(max(4, K.conv_plan(1, shp, dev).workspace), device=dev)
        wg = lambda: K.conv_wgrad(x, dy, dw, shp, accumulate=True)
        dg = lambda: K.conv_dgrad(dy, w, dx, shp, ws, False)
        wg(); dg()
        torch.cuda.synchronize()
        res = {}
        for name in ("wgrad", "dgrad", "seq", "two_streams"):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if name == "two_streams":
                    s1 = torch.cuda.Stream()
                    s1.wait_stream(torch.cuda.current_stream())
                    for _ in range(iters):
                        dg()
                    with torch.cuda.stream(s1):
                        for _ in range(iters):
                            wg()
                    torch.cuda.current_stream().wait_stream(s1)
                else:
                    for _ in range(iters):
                        if name in ("wgrad", "seq"):
                            wg()
                        if name in ("dgrad", "seq"):
                            dg()
            res[name] = timed(g) / iters
        print(f"{H}x{W}x{C}->{Co}: " + "  ".join(f"{k} {v:6.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
