"""Example-model layers and models on the HIP kernels vs the CPU reference
ops (layers.hip; Dense as 1x1 MFMA conv)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def test_bias_act_forward_backward():
    from metisfl_amd.ops import nn as K
    torch.manual_seed(0)
    M, N = 300, 136
    for act in (K.ACT_NONE, K.ACT_RELU):
        y = torch.randn(M, N).bfloat16()
        b = torch.randn(N)
        yc, yg = y.clone(), y.to(DEV)
        K.bias_act(yc, b, N, act)
        K.bias_act(yg, b.to(DEV), N, act)
        assert rel(yg, yc) < 1e-2
        dy = torch.randn(M, N).bfloat16()
        dzc, dzg = torch.empty_like(dy), torch.empty_like(dy).to(DEV)
        dbc, dbg = torch.zeros(N), torch.zeros(N, device=DEV)
        K.bias_act_backward(dy, yc, dzc, dbc, N, act)
        K.bias_act_backward(dy.to(DEV), yg, dzg, dbg, N, act)
        assert torch.equal(dzg.cpu(), dzc)
        assert torch.allclose(dbg.cpu(), dbc, rtol=1e-4, atol=1e-3)


def test_maxpool_forward_backward():
    from metisfl_amd.ops import nn as K
    torch.manual_seed(1)
    N, H, W, C = 4, 8, 6, 16
    x = torch.randn(N, H, W, C).bfloat16()
    x[0, 0, 0, :] = x[0, 0, 1, :]  # ties: the first maximum takes the gradient
    yc = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16)
    yg = yc.to(DEV)
    K.maxpool2(x, yc, N, H, W, C)
    K.maxpool2(x.to(DEV), yg, N, H, W, C)
    assert torch.equal(yg.cpu(), yc)
    dy = torch.randn_like(yc)
    dxc, dxg = torch.empty_like(x), torch.empty_like(x).to(DEV)
    K.maxpool2_backward(dy, x, yc, dxc, N, H, W, C)
    K.maxpool2_backward(dy.to(DEV), x.to(DEV), yg, dxg, N, H, W, C)
    assert torch.equal(dxg.cpu(), dxc)


def test_dropout_matches_host_mask():
    from metisfl_amd.ops import nn as K
    x = torch.randn(8192).bfloat16()
    step = torch.tensor([5], dtype=torch.int32)
    yc, yg = torch.empty_like(x), torch.empty_like(x).to(DEV)
    K.dropout(x, yc, 0.2, 1234, step)
    K.dropout(x.to(DEV), yg, 0.2, 1234, step.to(DEV))
    assert torch.equal(yg.cpu(), yc)


def test_xent_and_mse_heads():
    from metisfl_amd.ops import nn as K
    torch.manual_seed(2)
    B, Kp, Kv = 33, 16, 10
    z = torch.randn(B, Kp).bfloat16()
    lab = torch.randint(0, Kv, (B,), dtype=torch.int32)
    sc, sg = torch.zeros(4), torch.zeros(4, device=DEV)
    dc, dg = torch.empty_like(z), torch.empty_like(z).to(DEV)
    K.xent(z, lab, B, Kp, Kv, dc, sc)
    K.xent(z.to(DEV), lab.to(DEV), B, Kp, Kv, dg, sg)
    assert torch.allclose(sg.cpu(), sc, rtol=1e-3, atol=1e-3)
    assert rel(dg, dc) < 1e-2 and float(dg[:, Kv:].abs().sum()) == 0.0
    t = torch.randn(B)
    sc, sg = torch.zeros(4), torch.zeros(4, device=DEV)
    K.mse(z, t, B, Kp, dc, sc)
    K.mse(z.to(DEV), t.to(DEV), B, Kp, dg, sg)
    assert torch.allclose(sg.cpu(), sc, rtol=1e-3, atol=1e-3) and rel(dg, dc) < 1e-2


@pytest.mark.parametrize("family", ["fashion_mnist_fc", "cifar_cnn", "housing_mlp"])
def test_model_step_gpu_vs_cpu(family):
    from metisfl_amd.models.model_def import StaticModelDef
    from metisfl_amd.ops.optim import OptimizerSpec
    mdef = StaticModelDef(family)
    opt = OptimizerSpec("vanilla_sgd", 0.0)
    cpu = mdef.get_model(batch_size=8, device="cpu", seed=4)
    gpu = mdef.get_model(batch_size=8, device=DEV, seed=4)
    for n in (cpu, gpu):
        n.state.set_optimizer(opt)
        n.zero_grad_in_optimizer = False
    rng = np.random.default_rng(3)
    shape = {"fashion_mnist_fc": (8, 28, 28), "cifar_cnn": (8, 32, 32, 3), "housing_mlp": (8, 13)}[family]
    x = rng.standard_normal(shape).astype(np.float32)
    y = rng.standard_normal(8).astype(np.float32) if family == "housing_mlp" else rng.integers(0, 10, 8)
    dc, dg = cpu.make_dataset(x, y, shuffle=False), gpu.make_dataset(x, y, shuffle=False)
    cpu._train_body(dc)
    gpu._train_body(dg)
    torch.cuda.synchronize()
    a, b = cpu.state.grad32.double(), gpu.state.grad32.double().cpu()
    cos = float((a @ b) / (a.norm() * b.norm() + 1e-30))
    assert cos > 0.98, cos
    assert abs(float(cpu.stats[0]) - float(gpu.stats[0].cpu())) < 0.05 * abs(float(cpu.stats[0])) + 1e-3
