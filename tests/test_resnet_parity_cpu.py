"""The static ResNet-18 executor (host reference ops, fp32) vs an independent
torch.nn ResNet-18 (tests/torch_resnet_ref.py, fp64): same loss, same
gradient for every variable, same BN running statistics.  This pins the
layer graph itself -- residual wiring, BN-backward fusion targets, the
presummed reductions, head -- independently of the kernels (the GPU twin is
tests/test_fp32_gpu.py)."""
import numpy as np
import torch
import torch.nn.functional as F


def _rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / (b.norm() + 1e-300))


def test_cpu_executor_matches_torch_nn_resnet18():
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    from tests.torch_resnet_ref import reference_step
    rng = np.random.default_rng(3)
    B = 4
    x = rng.standard_normal((B, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, B)
    net = ResNet18(batch_size=B, device="cpu", optimizer=OptimizerSpec("vanilla_sgd", 0.0), seed=2)
    values = net.state.to_numpy()
    ds = net.make_dataset(x, y, shuffle=False)
    net.zero_grad_in_optimizer = False
    net._train_body(ds)
    loss = net.train_stats()["loss"]
    ref_loss, ref_g, ref_run = reference_step(values, F.pad(torch.as_tensor(x), (0, 5)), torch.as_tensor(y))
    assert abs(loss - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
    for name, rg in ref_g.items():
        assert _rel(net.state.grad(name), rg) <= 1e-4, name
    for name, rv in ref_run.items():
        assert _rel(net.state.view(name), rv) <= 1e-5, name
