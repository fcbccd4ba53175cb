"""Graph replay vs eager for the ResNet-18 learner: per-step max |diff| of
the flat fp32 model, eager-vs-eager and graph-vs-graph as noise references."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from metisfl_amd.models.resnet import ResNet18  # noqa: E402
from metisfl_amd.ops.optim import OptimizerSpec  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "fp32"
lr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
rng = np.random.default_rng(0)
x = rng.standard_normal((64, 32, 32, 3)).astype(np.float32)
y = rng.integers(0, 10, 64)


def make():
    n = ResNet18(batch_size=8, device="cuda", optimizer=OptimizerSpec("vanilla_sgd", lr), seed=3,
                 width_mult=0.25, dtype=dtype)
    return n, n.make_dataset(x, y, shuffle=False)


nets = [make() for _ in range(4)]  # eager, eager, graph, graph
for step in range(4):
    for i, (n, d) in enumerate(nets):
        if i < 2:
            n._train_body(d)
        else:
            n.train_steps(d, 1, step)
    torch.cuda.synchronize()
    m = [n.state.model32 for n, _ in nets]
    f = lambda a, b: float((a - b).abs().max())
    print(f"step {step + 1}: eager-eager {f(m[0], m[1]):.2e} graph-graph {f(m[2], m[3]):.2e} "
          f"eager-graph {f(m[0], m[2]):.2e}", flush=True)
