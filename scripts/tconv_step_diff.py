"""One fp32 ResNet-18 step with the paired latency-regime backward and with
the throughput backward (tconv.hip): per-tensor gradient differences."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from metisfl_amd.models.resnet import ResNet18  # noqa: E402
from metisfl_amd.ops.optim import OptimizerSpec  # noqa: E402


def run(tput, eager=True):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((32, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, 32)
    net = ResNet18(batch_size=32, device="cuda", optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=4,
                   conv_products="bf16x3")
    net.set_throughput_conv(tput)
    ds = net.make_dataset(x, y, shuffle=False)
    net.zero_grad_in_optimizer = False
    net._train_body(ds)
    torch.cuda.synchronize()
    return net


a, b = run(False), run(True)
rows = []
for s in a.state.specs:
    if not s.trainable:
        continue
    ga, gb = a.state.grad(s.name).double(), b.state.grad(s.name).double()
    rows.append((float((ga - gb).norm() / (ga.norm() + 1e-30)), s.name, float(ga.norm()), float(gb.norm())))
for r in rows:
    print(f"{r[1]:32s} rel {r[0]:.3e}  |paired| {r[2]:.4e} |tconv| {r[3]:.4e}")
