"""Hot- vs cold-input conv timing: the same conv launched back to back (input
L2-resident on every XCD) vs preceded by a kernel that rewrites its input (as
in the training graph, where a BN-apply kernel produced it)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.ops import nn as K

SHAPES = [(32, 32, 32, 64, 64, 3, 1), (32, 16, 16, 128, 128, 3, 1), (32, 8, 8, 256, 256, 3, 1),
          (32, 4, 4, 512, 512, 3, 1)]


def graph_us(fn, iters=40):
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


def main():
    dev = torch.device("cuda")
    for (N, H, W, C, Co, k, s) in SHAPES:
        shp = K.ConvShape(N, H, W, C, Co, k, k, s, k // 2)
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        x2 = torch.randn_like(x)
        w = (torch.randn(Co, k, k, C, device=dev) * 0.05).bfloat16()
        y = torch.empty(N, shp.P, shp.Q, Co, dtype=torch.bfloat16, device=dev)
        dy = torch.randn_like(y)
        dy2 = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.zeros(Co, k, k, C, device=dev)
        ws = torch.zeros(max(4, K.conv_plan(0, shp, dev).workspace, K.conv_plan(1, shp, dev).workspace), device=dev)
        big = torch.empty(64 << 20, dtype=torch.uint8, device=dev)  # 64 MiB: evicts the L2s
        res = {}
        res["copy"] = graph_us(lambda: x.copy_(x2))
        res["fwd_hot"] = graph_us(lambda: K.conv_forward(x, w, y, shp, ws, None))
        res["fwd_cold"] = graph_us(lambda: (x.copy_(x2), K.conv_forward(x, w, y, shp, ws, None))) - res["copy"]
        res["dgrad_hot"] = graph_us(lambda: K.conv_dgrad(dy, w, dx, shp, ws, False))
        res["dgrad_cold"] = graph_us(lambda: (dy.copy_(dy2), K.conv_dgrad(dy, w, dx, shp, ws, False))) - res["copy"] * dy.numel() / x.numel()
        res["wgrad_hot"] = graph_us(lambda: K.conv_wgrad(x, dy, dw, shp, accumulate=True))
        res["wgrad_cold"] = graph_us(lambda: (x.copy_(x2), K.conv_wgrad(x, dy, dw, shp, accumulate=True))) - res["copy"]
        stats = torch.zeros(2 * Co, dtype=torch.float64, device=dev)
        res["fwd_stats_hot"] = graph_us(lambda: K.conv_forward(x, w, y, shp, ws, stats))
        bz = torch.randn_like(x)
        bnb = K.BnBwdTarget(bz, None, torch.zeros(C, device=dev), torch.ones(C, device=dev),
                            torch.zeros(2 * C, dtype=torch.float64, device=dev))
        res["dgrad_bnb_hot"] = graph_us(lambda: K.conv_dgrad(dy, w, dx, shp, ws, False, bnb=bnb))
        res["fill64M"] = graph_us(lambda: big.fill_(1))
        res["fwd_evicted"] = graph_us(lambda: (big.fill_(1), K.conv_forward(x, w, y, shp, ws, None))) - res["fill64M"]
        print((N, H, W, C, Co, k, s), " ".join(f"{k_}={v:.1f}" for k_, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
