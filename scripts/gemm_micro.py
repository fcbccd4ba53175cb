"""BERT-base GEMM microbenchmark (M = 128 x 128 tokens): fwd / dgrad / wgrad of
every projection shape on the large-tile path (gemm_big.hip), the conv-core
path, and torch.matmul (hipBLASLt) for reference; TFLOP/s per call, timed as
graph replays of 20 launches."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from metisfl_amd.ops._native import ops

M = 16384
SHAPES = [("qkv", 2304, 768), ("attn_out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)]


def graph_us(fn, iters=20):
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
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * iters)


def main():
    o = ops()
    res = []
    for name, N, K in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16()
        dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
        dw = torch.zeros(N, K, device="cuda")
        bias = torch.zeros(N, device="cuda")
        fl = 2.0 * M * N * K
        row = {"shape": name, "M": M, "N": N, "K": K}
        for path in (("big",) if os.environ.get("BIG_ONLY") else ("big", "conv")):
            o.set_gemm_big(path == "big")
            for op, fn in (("fwd", lambda: o.gemm_fwd(x, w, y, bias, None, None, M, N, K)),
                           ("dgrad", lambda: o.gemm_dgrad(dy, w, dx, M, N, K, False)),
                           ("wgrad", lambda: o.gemm_wgrad(x, dy, dw, M, N, K, True, True))):
                us = graph_us(fn)
                row[f"{path}_{op}_us"] = round(us, 2)
                row[f"{path}_{op}_tf"] = round(fl / us / 1e6, 1)
        if os.environ.get("BIG_ONLY"):
            print(json.dumps(row), flush=True)
            continue
        for op, fn in (("fwd", lambda: torch.matmul(x, w.t(), out=y)),
                       ("dgrad", lambda: torch.matmul(dy, w, out=dx)),
                       ("wgrad", lambda: torch.matmul(dy.t(), x))):
            us = graph_us(fn)
            row[f"hipblaslt_{op}_us"] = round(us, 2)
            row[f"hipblaslt_{op}_tf"] = round(fl / us / 1e6, 1)
        print(json.dumps(row), flush=True)
        res.append(row)
    o.set_gemm_big(True)
    return res


if __name__ == "__main__":
    main()
