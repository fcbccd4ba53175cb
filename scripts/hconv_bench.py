"""Per-stage timing: BatchNorm apply + im2col conv32 forward (round-2 path)
against the halo conv with the BN fused into its operand fill (hconv.hip).

    python scripts/hconv_bench.py [--iters 200]

Both sides run the same work: y = relu(BN(z) + res) materialised (fp32 y +
packed yp), out = conv3x3(y, W), output BN sums.  Interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24); median per call in us.
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
    ap.add_argument("--eager", type=int, default=0,
                    help="profiling: run only the halo conv, N eager calls per stage, no timing")
    ap.add_argument("--stamps", action="store_true", help="in-kernel phase stamps of the halo conv")
    args = ap.parse_args()
    K.set_conv_products("bf16x3")
    dev = torch.device("cuda")
    N = args.batch
    for H, W, C in STAGES:
        shp = K.ConvShape(N, H, W, C, C, 3, 3, 1, 1)
        z = torch.randn(N, H, W, C, device=dev)
        res = torch.randn(N, H, W, C, device=dev)
        w = torch.randn(C, 3, 3, C, device=dev) / (9 * C) ** 0.5
        wp = torch.zeros(w.numel(), dtype=torch.int32, device=dev)
        split_pack(w.reshape(-1), wp)
        acc = torch.zeros(16 * C, dtype=torch.float64, device=dev)
        acc[:C] = z.reshape(-1, C).double().sum(0)
        acc[C:2 * C] = (z.reshape(-1, C).double() ** 2).sum(0)
        bn = K.BnParams(acc, torch.ones(C, device=dev), torch.zeros(C, device=dev), torch.zeros(C, device=dev),
                        torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.ones(C, device=dev))
        y = torch.empty_like(z)
        yp = torch.empty(z.shape, dtype=torch.int32, device=dev)
        out = torch.empty_like(z)
        stats = torch.zeros(16 * C, dtype=torch.float64, device=dev)
        pf = K.conv_plan(0, shp, dev, torch.float32)
        ws = torch.zeros(max(4, pf.workspace, K.hconv_workspace(shp, dev)), device=dev)

        def old():
            K.bn_apply(z, C, acc, bn.gamma, bn.beta, bn.mean, bn.invstd, bn.run_mean, bn.run_var, y,
                       residual=res, relu=True, train=True, yp=yp)
            K.conv_forward(y, w, out, shp, ws, stats, wp=wp, xp=yp)

        def new():
            K.hconv_forward(z, wp, w, out, shp, bn, True, True, ws=ws, stats=stats, res=res, y=y, yp=yp)

        def conv_only():
            K.conv_forward(y, w, out, shp, ws, stats, wp=wp, xp=yp)

        if args.eager:
            for _ in range(args.eager):
                new()
            torch.cuda.synchronize()
            continue
        if args.stamps:  # per-phase cycle stamps of every workgroup (median over workgroups)
            st = torch.zeros(2048 * 16, dtype=torch.int64, device=dev)
            for _ in range(3):
                K.hconv_forward(z, wp, w, out, shp, bn, True, True, ws=ws, stats=stats, res=res, y=y, yp=yp,
                                stamps=st)
            torch.cuda.synchronize()
            t = st.view(-1, 16)[:, :9].cpu().double()
            t = t[t[:, 0] > 0]
            base = t[:, 0].min()
            rel = t - base
            ph = ["coef", "fill0", "chunk0_mfma", "chunk0_store", "loop_rest", "epi_tile", "out_store",
                  "stats"]
            d = (t[:, 1:] - t[:, :-1]).median(0).values
            print(json.dumps({"stage": f"{N}x{H}x{W}x{C}", "wg": int(t.shape[0]),
                              "phase_cycles_median": {p: float(v) for p, v in zip(ph, d)},
                              "start_spread": float(rel[:, 0].max()), "end_max": float(rel[:, 8].max())}),
                  flush=True)
            continue
        res_t = {}
        fns = (("bn+conv32", old), ("conv32", conv_only), ("hconv", new))
        graphs = {}
        for name, fn in fns:  # graph replay, as in the training step (no host launch gaps)
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
        for k, v in samples.items():
            res_t[k] = round(statistics.median(v), 2)
        print(json.dumps({"stage": f"{N}x{H}x{W}x{C}", "us_per_call": res_t}), flush=True)


if __name__ == "__main__":
    main()
