"""GPU diagnostic: split-K hand-off under hipGraph replay.

Runs conv layers with in-kernel split-K reductions back to back on one shared
workspace (as the ResNet step does), eagerly and inside a captured graph, and
reports any output that differs from the eager reference (the reduction order
is fixed, so results must be bit-identical)."""
import sys

import torch

from metisfl_amd.ops import nn as K

DEV = "cuda"


def main():
    torch.manual_seed(0)
    shapes = [K.ConvShape(32, 4, 4, 512, 512, 3, 3, 1, 1),   # layer4
              K.ConvShape(32, 8, 8, 256, 256, 3, 3, 1, 1),   # layer3
              K.ConvShape(32, 8, 8, 256, 512, 3, 3, 2, 1),   # layer4 entry
              K.ConvShape(32, 16, 16, 128, 128, 3, 3, 1, 1)]  # layer2
    dev = torch.device(DEV)
    need = 4
    for s in shapes:
        need = max(need, K.conv_plan(0, s, dev).workspace, K.conv_plan(1, s, dev).workspace)
        print("plan fwd", s, K.conv_plan(0, s, dev), "dgrad", K.conv_plan(1, s, dev))
    ws = torch.zeros(need, device=DEV)
    xs = [torch.randn(s.N, s.H, s.W, s.C, device=DEV).bfloat16() for s in shapes]
    wts = [(torch.randn(s.Co, s.R, s.S, s.C, device=DEV) * 0.05).bfloat16() for s in shapes]
    dys = [torch.randn(s.N, s.P, s.Q, s.Co, device=DEV).bfloat16() for s in shapes]
    ys = [torch.empty(s.N, s.P, s.Q, s.Co, dtype=torch.bfloat16, device=DEV) for s in shapes]
    dxs = [torch.empty_like(x) for x in xs]

    def body():
        for i, s in enumerate(shapes):
            K.conv_forward(xs[i], wts[i], ys[i], s, ws, None)
            K.conv_dgrad(dys[i], wts[i], dxs[i], s, ws, False)

    body()
    torch.cuda.synchronize()
    ref_y = [y.clone() for y in ys]
    ref_dx = [d.clone() for d in dxs]
    bad = 0
    for it in range(20):
        body()
        torch.cuda.synchronize()
        for i in range(len(shapes)):
            bad += int(not torch.equal(ys[i], ref_y[i])) + int(not torch.equal(dxs[i], ref_dx[i]))
    print("eager repeat mismatches:", bad)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        body()
    badg = 0
    for it in range(50):
        for y in ys:
            y.zero_()
        g.replay()
        torch.cuda.synchronize()
        for i in range(len(shapes)):
            my = not torch.equal(ys[i], ref_y[i])
            md = not torch.equal(dxs[i], ref_dx[i])
            if (my or md) and badg < 10:
                print(f"replay {it} layer {i}: y {'BAD' if my else 'ok'} "
                      f"({(ys[i].float() - ref_y[i].float()).abs().max().item():.3g}) dx {'BAD' if md else 'ok'}")
            badg += int(my) + int(md)
    print("graph replay mismatches:", badg)
    sys.exit(1 if (bad or badg) else 0)


if __name__ == "__main__":
    main()
