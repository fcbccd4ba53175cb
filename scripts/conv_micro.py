"""Per-layer conv microbenchmark (ResNet-18 CIFAR shapes, batch 32): times
fwd / dgrad / wgrad of every distinct layer with HIP events and prints a
table; also the workload for rocprofv3 --pmc counter runs."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch

from metisfl_amd.ops import nn as K

SHAPES = [(32, 32, 32, 8, 64, 3, 1), (32, 32, 32, 64, 64, 3, 1), (32, 32, 32, 64, 128, 3, 2),
          (32, 32, 32, 64, 128, 1, 2), (32, 16, 16, 128, 128, 3, 1), (32, 16, 16, 128, 256, 3, 2),
          (32, 16, 16, 128, 256, 1, 2), (32, 8, 8, 256, 256, 3, 1), (32, 8, 8, 256, 512, 3, 2),
          (32, 8, 8, 256, 512, 1, 2), (32, 4, 4, 512, 512, 3, 1)]


def graph_us(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main(iters=50):
    dev = torch.device("cuda")
    one = torch.zeros(1, device=dev)
    print(f"trivial kernel (1-element add_) per launch in a graph: {graph_us(lambda: one.add_(1), 200):.2f}us")
    for (N, H, W, C, Co, k, s) in SHAPES:
        shp = K.ConvShape(N, H, W, C, Co, k, k, s, k // 2)
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(Co, k, k, C, device=dev) * 0.05).bfloat16()
        y = torch.empty(N, shp.P, shp.Q, Co, dtype=torch.bfloat16, device=dev)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.zeros(Co, k, k, C, device=dev)
        ws = torch.zeros(max(4, K.conv_plan(0, shp, dev).workspace, K.conv_plan(1, shp, dev).workspace), device=dev)
        res = []
        for name, fn in (("fwd", lambda: K.conv_forward(x, w, y, shp, ws, None)),
                         ("dgrad", lambda: K.conv_dgrad(dy, w, dx, shp, ws, False)),
                         ("wgrad", lambda: K.conv_wgrad(x, dy, dw, shp, accumulate=True))):
            if name == "dgrad" and C == 8:
                res.append(f"{name} -")
                continue
            fn()
            torch.cuda.synchronize()
            # replay a captured graph of `iters` launches: per-launch CPU
            # overhead is out of the measurement, as in the training step
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(iters):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / iters
            fl = 2.0 * shp.N * shp.P * shp.Q * Co * C * k * k
            res.append(f"{name} {us:6.1f}us {fl / us / 1e6:6.1f}TF")
        print((N, H, W, C, Co, k, s), " | ".join(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
