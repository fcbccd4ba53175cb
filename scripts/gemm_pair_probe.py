"""Does running an output-heavy GEMM (the FFN2 dgrad with the GELU backward
fused: reads z, writes dz, 100 MB each) next to a compute-heavy one (the FFN2
weight gradient, split-K) beat running them one after the other?  Both kernels
occupy one workgroup per CU; on two streams the dispatcher interleaves their
workgroups, so the first one's output bursts no longer happen on every CU at
once.  Prints us per pair: each alone, serial, and on two streams."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.ops._native import ops

M, N, K = 16384, 768, 3072


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    o = ops()
    dev = "cuda"
    dy = ((torch.rand(M, N, device=dev) * 2 - 1) * 0.1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
    z = (torch.randn(M, K, device=dev)).bfloat16()
    h = (torch.randn(M, K, device=dev)).bfloat16()
    dz = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    dbias = torch.zeros(K, device=dev)
    dw = torch.zeros(N, K, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def dgrad():
        o.gemm_dgrad_gelu(dy, w, dz, z, dbias, M, N, K)

    def wgrad():
        o.gemm_wgrad(h, dy, dw, M, N, K, False, False)

    def serial():
        dgrad()
        wgrad()

    def streams():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            dgrad()
        with torch.cuda.stream(s2):
            wgrad()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def streams_rev():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            wgrad()
        with torch.cuda.stream(s1):
            dgrad()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    r = {}
    for name, fn in (("dgrad_gelu", dgrad), ("wgrad", wgrad), ("serial", serial), ("two_streams", streams),
                     ("two_streams_wgrad_first", streams_rev), ("serial_again", serial)):
        r[name] = round(timed(fn), 2)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
