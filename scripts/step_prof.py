"""Time the ResNet-18 local-update step (the hipGraph the bench replays
6,252 times per round) for one precision; short enough to run under
rocprofv3.  python scripts/step_prof.py [--dtype fp32|bf16] [--steps N]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from metisfl_amd.models.resnet import ResNet18  # noqa: E402
from metisfl_amd.ops.optim import OptimizerSpec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--conv-products", default=None, choices=(None, "exact", "bf16x3"))
    a = ap.parse_args()
    net = ResNet18(batch_size=a.batch, device="cuda", seed=7, dtype=a.dtype, conv_products=a.conv_products,
                   optimizer=OptimizerSpec("momentum_sgd", 0.005, momentum=0.75))
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn((2048, 32, 32, 3), generator=g, device="cuda")
    y = torch.randint(0, 10, (2048,), generator=g, device="cuda")
    ds = net.make_dataset(x, y)
    net.train_steps(ds, a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    net.train_steps(ds, a.steps, a.warmup)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e3 / a.steps
    tag = f"{a.dtype}/{net.conv_products}" if a.dtype == "fp32" else a.dtype
    print(f"{tag} batch {a.batch}: {dt:.4f} ms per local update "
          f"({a.batch / dt * 1e3:.0f} samples/s), loss {net.train_stats()['loss']:.4f}", flush=True)


if __name__ == "__main__":
    main()
