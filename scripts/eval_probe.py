"""Time a test-set evaluation (10,000 CIFAR-shaped samples, BN in inference
mode) of the fp32 ResNet-18 at several evaluation micro-batch sizes.
python scripts/eval_probe.py [--batches 32,64,128]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from metisfl_amd.models.resnet import ResNet18  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="32,64,128")
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn((a.n, 32, 32, 3), generator=g, device="cuda")
    y = torch.randint(0, 10, (a.n,), generator=g, device="cuda")
    for b in [int(v) for v in a.batches.split(",")]:
        net = ResNet18(batch_size=b, device="cuda", seed=7, dtype="fp32")
        ds = net.make_dataset(x, y, shuffle=False)
        net.evaluate(ds)  # capture + warm
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r = net.evaluate(ds)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"eval batch {b}: {min(ts):.2f} ms (runs {', '.join(f'{t:.2f}' for t in ts)}), "
              f"{ds.steps_per_epoch} batches, loss {r['loss']:.5f} acc {r['accuracy']:.4f}", flush=True)
        del net, ds
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
