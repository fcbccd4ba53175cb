"""Per-call device time of the latency-regime fp32 (bf16x3) backward kernels
(conv32.hip: dgrad, wgrad and the paired launch) at the 3x3 / stride-1
ResNet-18 CIFAR shapes (graph-replayed, one stream and 8 learners' launches over 4 streams).
python scripts/conv32_ref_times.py [batch] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from metisfl_amd.ops import nn as K  # noqa: E402
from metisfl_amd.ops.nn import ConvShape  # noqa: E402
from metisfl_amd.ops.optim import split_pack  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def timed_conc(fns, iters, nstreams=4):
    """fns[l]: learner l's launch; each learner's ``iters`` calls captured in
    one hipGraph (as the learners replay their step graphs) and the graphs
    replayed over nstreams streams (co-located regime) -> us per learner call."""
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    cur = torch.cuda.current_stream()
    graphs = []
    for fn in fns:
        fn()
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            for _ in range(iters):
                fn()
        graphs.append(gph)
    for l, gph in enumerate(graphs):  # warm replay
        with torch.cuda.stream(streams[l % nstreams]):
            gph.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for s in streams:
        s.wait_stream(cur)
    for l, gph in enumerate(graphs):
        with torch.cuda.stream(streams[l % nstreams]):
            gph.replay()
    for s in streams:
        cur.wait_stream(s)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (iters * len(fns))


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    K.set_conv_products("bf16x3")
    dev = torch.device("cuda")
    ws = torch.zeros(64 << 20, device=dev)
    for H, C in ((32, 64), (16, 128), (8, 256), (4, 512)):
        s = ConvShape(batch, H, H, C, C, 3, 3, 1, 1)
        x = torch.randn(batch, H, H, C, device=dev)
        dy = torch.randn(batch, H, H, C, device=dev) * 0.01
        w = torch.randn(C, 3, 3, C, device=dev) * 0.05
        xp = torch.empty(x.shape, dtype=torch.int32, device=dev)
        dyp = torch.empty(dy.shape, dtype=torch.int32, device=dev)
        wp = torch.empty(w.shape, dtype=torch.int32, device=dev)
        split_pack(x.reshape(-1), xp.view(-1))
        split_pack(dy.reshape(-1), dyp.view(-1))
        split_pack(w.reshape(-1), wp.view(-1))
        dyf = dyp.view(torch.float32)
        dw = torch.zeros_like(w)
        dx = torch.zeros_like(x)
        tw = timed(lambda: K.conv_wgrad(x, dyf, dw, s, accumulate=True, dy_packed=True, xp=xp), iters)
        td = timed(lambda: K.conv_dgrad(dyf, w, dx, s, ws, False, wp=wp, dy_packed=True), iters)
        tp = timed(lambda: K.conv_backward_pair(x, dyf, dw, w, dx, s, ws, False, wp=wp, dy_packed=True, xp=xp),
                   iters)
        flop = 2.0 * batch * H * H * C * 9 * C
        # 8 co-located learners on 4 streams, each with its own buffers
        L = 8
        bufs = [(x.clone(), xp.clone(), dyf.clone(), w.clone(), wp.clone(), torch.zeros_like(w), torch.zeros_like(x),
                 torch.zeros(16 << 20, device=dev)) for _ in range(L)]
        cw = timed_conc([lambda b=b: K.conv_wgrad(b[0], b[2], b[5], s, accumulate=True, dy_packed=True, xp=b[1])
                         for b in bufs], iters)
        cd = timed_conc([lambda b=b: K.conv_dgrad(b[2], b[3], b[6], s, b[7], False, wp=b[4], dy_packed=True)
                         for b in bufs], iters)
        cp = timed_conc([lambda b=b: K.conv_backward_pair(b[0], b[2], b[5], b[3], b[6], s, b[7], False, wp=b[4],
                                                          dy_packed=True, xp=b[1]) for b in bufs], iters)
        print(f"conv32 N={batch} {H}x{H} C={C}: wgrad {tw:.2f} us ({flop / tw * 1e-6:.0f} TF) | "
              f"dgrad {td:.2f} us ({flop / td * 1e-6:.0f} TF) | pair {tp:.2f} us || 8 on 4 streams: "
              f"wgrad {cw:.2f} dgrad {cd:.2f} pair {cp:.2f} us per learner", flush=True)


if __name__ == "__main__":
    main()
