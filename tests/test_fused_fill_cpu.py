"""The fused-fill forward orchestration (every BatchNorm apply deferred into its
consumer's halo-conv operand fill, models/layers.py forward_fused) on the CPU
references: the same training steps as the BatchNorm-apply orchestration --
identical activations, gradients, BN statistics and running averages (up to
the fp64-vs-fp32 coefficient rounding of the two reference paths)."""
import numpy as np
import pytest
import torch

from metisfl_amd.models import layers as L
from metisfl_amd.ops import nn as K
from metisfl_amd.ops.optim import OptimizerSpec


def _net(fused: bool, monkeypatch, halo_dgrad: bool = False):
    from metisfl_amd.models.resnet import ResNet18
    monkeypatch.setattr(L, "FUSED_FILL_CPU", fused)
    monkeypatch.setattr(L, "HALO_DGRAD", halo_dgrad)
    net = ResNet18(batch_size=8, optimizer=OptimizerSpec("momentum_sgd", 0.01, momentum=0.9), seed=5)
    net.zero_grad_in_optimizer = False
    return net


def test_hconv_workspace_covers_the_resnet_stages():
    dev = torch.device("cpu")
    for h, c in ((32, 64), (16, 128), (8, 256), (4, 512)):
        assert K.hconv_workspace(K.ConvShape(8, h, h, c, c, 3, 3, 1, 1), dev) >= 0
    assert K.hconv_workspace(K.ConvShape(8, 32, 32, 64, 128, 3, 3, 2, 1), dev) == -1  # stride 2
    assert K.hconv_workspace(K.ConvShape(8, 32, 32, 8, 64, 3, 3, 1, 1), dev) == -1    # stem
    assert K.hconv_workspace(K.ConvShape(4, 4, 4, 512, 512, 3, 3, 1, 1), dev) == -1  # 8-image tiles


@pytest.mark.parametrize("halo_dgrad", [False, True], ids=["pair_bwd", "halo_dgrad"])
def test_fused_fill_matches_bn_apply_orchestration(monkeypatch, halo_dgrad):
    rng = np.random.default_rng(3)
    x = rng.standard_normal((16, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, 16)
    ref = _net(False, monkeypatch)
    fus = _net(True, monkeypatch, halo_dgrad)
    assert not ref.fused_fill() and fus.fused_fill()
    assert torch.equal(ref.state.model32, fus.state.model32)
    for net in (ref, fus):
        ds = net.make_dataset(x, y, seed=1)
        net.reset_train_stats()
        net.train_steps(ds, 2)
    torch.testing.assert_close(fus.state.grad32, ref.state.grad32, rtol=2e-4, atol=2e-6)
    torch.testing.assert_close(fus.state.model32, ref.state.model32, rtol=1e-5, atol=1e-6)
    for a, b in zip(fus.blocks, ref.blocks):
        for la, lb in zip(a.sublayers(), b.sublayers()):
            torch.testing.assert_close(la.z, lb.z, rtol=1e-4, atol=1e-5)
            torch.testing.assert_close(la.mean, lb.mean, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(la.invstd, lb.invstd, rtol=1e-5, atol=1e-6)
            if la.relu:  # materialised activations (ReLU masks of the backward)
                torch.testing.assert_close(la.y, lb.y, rtol=1e-4, atol=1e-5)
    assert fus.train_stats()["loss"] == pytest.approx(ref.train_stats()["loss"], rel=1e-5)
    # evaluation (running statistics in the fills)
    ev = fus.make_dataset(x, y, shuffle=False)
    er = ref.make_dataset(x, y, shuffle=False)
    assert fus.evaluate(ev)["loss"] == pytest.approx(ref.evaluate(er)["loss"], rel=1e-4)
