"""Per-stage timing of a 3x3 / stride-1 layer's backward: the round-2 path
(bn32 backward apply + paired conv32 dgrad / wgrad) against the halo dgrad
with the BatchNorm backward in its operand fill (hconv.hip) + the wgrad, and
each kernel alone.  Graph replay, interleaved rounds, median us per call.

    python scripts/hdgrad_bench.py [--iters 200]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from metisfl_amd.ops import nn as K  # noqa: E402
from metisfl_amd.ops.optim import split_pack  # noqa: E402

STAGES = [(32, 32, 64), (16, 16, 128), (8, 8, 256), (4, 4, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--eager", type=int, default=0, help="profiling: N eager calls of the paired backward per stage")
    args = ap.parse_args()
    K.set_conv_products("bf16x3")
    dev = torch.device("cuda")
    N = args.batch
    for H, W, C in STAGES:
        shp = K.ConvShape(N, H, W, C, C, 3, 3, 1, 1)
        r = lambda: torch.randn(N, H, W, C, device=dev)  # noqa: E731
        dy, z, ym, x = r(), r(), r().clamp_min(0), r().clamp_min(0)
        xp = torch.empty(x.shape, dtype=torch.int32, device=dev)
        split_pack(x.reshape(-1), xp.reshape(-1))
        w = torch.randn(C, 3, 3, C, device=dev) / (9 * C) ** 0.5
        wp = torch.zeros(w.numel(), dtype=torch.int32, device=dev)
        split_pack(w.reshape(-1), wp)
        acc = torch.zeros(16 * C, dtype=torch.float64, device=dev)
        acc[:C] = dy.reshape(-1, C).double().sum(0)
        acc[C:2 * C] = (dy.reshape(-1, C).double() * z.reshape(-1, C).double()).sum(0)
        one, zero = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        bn = K.BnParams(acc, one, zero, zero, one, None, None)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dz = torch.empty_like(z)
        dzp = dz.view(torch.int32)
        dres = torch.empty_like(z)
        dx, dw = torch.empty_like(z), torch.zeros_like(w)
        bacc = torch.zeros(16 * C, dtype=torch.float64, device=dev)
        bnb = K.BnBwdTarget(r(), r().clamp_min(0), zero, one, bacc)
        pd = K.conv_plan(1, shp, dev, torch.float32)
        ws = torch.zeros(max(4, pd.workspace, K.hconv_workspace(shp, dev)), device=dev)

        def bnbwd():
            K.bn_backward(dy, z, ym, C, one, zero, one, acc, dg, db, dzp, dy_masked=dres, presummed=True,
                          dx_packed=True)

        def pair():
            K.conv_backward_pair(x, dz, dw, w, dx, shp, ws, False, bnb=bnb, wp=wp, dy_packed=True, xp=xp)

        def dgrad():
            K.conv_dgrad(dz, w, dx, shp, ws, False, bnb=bnb, wp=wp, dy_packed=True)

        def wgrad():
            K.conv_wgrad(x, dz, dw, shp, accumulate=True, dy_packed=True, xp=xp)

        def hdgrad():
            K.hconv_dgrad(dy, ym, z, wp, w, dx, shp, bn, dgamma=dg, dbeta=db, ws=ws, dres=dres, dzp=dzp, bnb=bnb)

        if args.eager:
            for _ in range(args.eager):
                pair()
            torch.cuda.synchronize()
            continue
        side = torch.cuda.Stream()

        def hdgrad_par_wgrad():  # the wgrad on a second stream, concurrent with the halo dgrad
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                wgrad()
            hdgrad()
            cur.wait_stream(side)

        fns = (("hdgrad||wgrad", hdgrad_par_wgrad), ("bnbwd+pair", lambda: (bnbwd(), pair())), ("bnbwd", bnbwd), ("pair", pair), ("dgrad", dgrad),
               ("wgrad", wgrad), ("hdgrad", hdgrad), ("hdgrad+wgrad", lambda: (hdgrad(), wgrad())))
        graphs = {}
        for name, fn in fns:
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(20):
                    fn()
            graphs[name] = g
        torch.cuda.synchronize()
        samples = {k: [] for k, _ in fns}
        reps = max(1, args.iters // 20)
        for _ in range(args.rounds):
            for name, _ in fns:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    graphs[name].replay()
                e1.record()
                torch.cuda.synchronize()
                samples[name].append(e0.elapsed_time(e1) * 1000.0 / (reps * 20))
        print(json.dumps({"stage": f"{N}x{H}x{W}x{C}",
                          "us_per_call": {k: round(statistics.median(v), 2) for k, v in samples.items()}}), flush=True)


if __name__ == "__main__":
    main()
