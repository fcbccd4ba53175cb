"""Per-layer timing of the fp32 conv kernels (conv32.hip) on the ResNet-18
CIFAR shapes at batch 32: the planner's choice, and with --sweep every
(BM, BN, split) candidate via the MFL_C32_* plan overrides.
python scripts/conv32_bench.py [--sweep] [--iters 50]"""
import argparse
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from metisfl_amd.ops import nn as K  # noqa: E402
from metisfl_amd.ops.nn import ConvShape  # noqa: E402

SHAPES = [  # N, H, W, C, Co, k, stride
    (32, 32, 32, 8, 64, 3, 1), (32, 32, 32, 64, 64, 3, 1), (32, 32, 32, 64, 128, 3, 2),
    (32, 32, 32, 64, 128, 1, 2), (32, 16, 16, 128, 128, 3, 1), (32, 16, 16, 128, 256, 3, 2),
    (32, 16, 16, 128, 256, 1, 2), (32, 8, 8, 256, 256, 3, 1), (32, 8, 8, 256, 512, 3, 2),
    (32, 8, 8, 256, 512, 1, 2), (32, 4, 4, 512, 512, 3, 1),
]
# how many times each shape runs per training step (fwd; dgrad skips the stem)
PER_STEP = [1, 4, 1, 1, 3, 1, 1, 3, 1, 1, 3]


def set_plan(bm=0, bn=0, sp=0):
    os.environ["MFL_C32_BM"] = str(bm)
    os.environ["MFL_C32_BN"] = str(bn)
    os.environ["MFL_C32_SPLIT"] = str(sp)


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--products", default="exact", choices=("exact", "bf16x3"))
    ap.add_argument("--stats-reps", type=int, default=1,
                    help="forward BN-statistics accumulator replicas (0: no statistics)")
    a = ap.parse_args()
    K.set_conv_products(a.products)
    print("conv products:", a.products)
    dev = torch.device("cuda")
    ws = torch.zeros(16 << 20, device=dev)
    total = {0: 0.0, 1: 0.0, 2: 0.0}
    for t, mult in zip(SHAPES, PER_STEP):
        N, H, W, C, Co, k, s = t
        shp = ConvShape(N, H, W, C, Co, k, k, s, k // 2)
        x = torch.randn(N, H, W, C, device=dev)
        w = torch.randn(Co, k, k, C, device=dev) * 0.05
        y = torch.zeros(N, shp.P, shp.Q, Co, device=dev)
        st = torch.zeros(2 * Co * max(1, a.stats_reps), dtype=torch.float64, device=dev) if a.stats_reps else None
        dy = torch.randn(N, shp.P, shp.Q, Co, device=dev)
        dx = torch.zeros(N, H, W, C, device=dev)
        dw = torch.zeros(Co, k, k, C, device=dev)
        flop = 2.0 * N * shp.P * shp.Q * Co * k * k * C
        if a.products == "bf16x3":
            # as in the model: operands arrive as packed hi|lo mirrors written
            # by their producers (no per-call packing inside the timing)
            from metisfl_amd.ops.optim import split_pack
            wp = torch.zeros(w.shape, dtype=torch.int32, device=dev)
            split_pack(w.reshape(-1), wp.view(-1))
            xp = torch.zeros(x.shape, dtype=torch.int32, device=dev)
            split_pack(x.reshape(-1), xp.view(-1))
            dyp = torch.zeros(dy.shape, dtype=torch.int32, device=dev)
            split_pack(dy.reshape(-1), dyp.view(-1))
            dyv = dyp.view(torch.float32)
            runs = {0: lambda: K.conv_forward(x, w, y, shp, ws, st, wp=wp, xp=xp),
                    1: lambda: K.conv_dgrad(dyv, w, dx, shp, ws, False, wp=wp, dy_packed=True),
                    2: lambda: K.conv_wgrad(x, dyv, dw, shp, accumulate=True, dy_packed=True, xp=xp)}
        else:
            runs = {0: lambda: K.conv_forward(x, w, y, shp, ws, st),
                    1: lambda: K.conv_dgrad(dy, w, dx, shp, ws, False),
                    2: lambda: K.conv_wgrad(x, dy, dw, shp, accumulate=True)}
        for mode in map(int, a.modes.split(",")):
            if mode == 1 and C == 8:
                continue
            set_plan()
            p = K.conv_plan(mode, shp, dev, torch.float32)
            us = timed(runs[mode], a.iters)
            total[mode] += us * mult
            line = (f"{'fdw'[mode]} {'x'.join(map(str, t)):22s} plan {p.bm}x{p.bn} s{p.splits:<3d} "
                    f"{us:7.1f} us {flop / us / 1e6:6.1f} TF")
            if a.sweep:
                best = (us, p.bm, p.bn, p.splits)
                for bm, bn, sp in itertools.product((64, 128), (64, 128), (1, 2, 3, 4, 6, 7, 8, 12, 14, 16, 24, 28, 32, 48, 64)):
                    set_plan(bm, bn, sp)
                    q = K.conv_plan(mode, shp, dev, torch.float32)
                    if q.kchunk == 0 or q.splits != sp or q.bm != bm or q.bn != bn:
                        continue
                    if q.workspace > ws.numel():
                        continue
                    u = timed(runs[mode], a.iters)
                    if u < best[0]:
                        best = (u, bm, bn, sp)
                set_plan()
                line += f" | best {best[1]}x{best[2]} s{best[3]} {best[0]:7.1f} us {flop / best[0] / 1e6:6.1f} TF"
            print(line, flush=True)
    print(f"per-step conv time (planner): fwd {total[0]:.0f} us, dgrad {total[1]:.0f} us, wgrad {total[2]:.0f} us, "
          f"sum {sum(total.values()):.0f} us", flush=True)


if __name__ == "__main__":
    main()
