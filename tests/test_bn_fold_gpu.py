"""BatchNorm-backward applies folded into the preceding paired conv backward
launch (conv32.hip folded_bn_bwd, models/layers.py BN_FOLD): the same
training step with and without the fold -- every gradient, the updated model
and the BN statistics agree up to the fp32 atomic-order noise the unfolded
path already has (the folded apply runs the same arithmetic as
bn32_bwd_apply; its upstream gradient is read device-scope while the dgrad of
the same launch is still finishing other tiles)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return float((a - b).norm() / (b.norm() + 1e-300))


def _step(fold, monkeypatch, products, steps=3):
    from metisfl_amd.models import layers as L
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    monkeypatch.setattr(L, "BN_FOLD", fold)
    net = ResNet18(batch_size=32, device="cuda", seed=11, conv_products=products,
                   optimizer=OptimizerSpec("momentum_sgd", 0.05, momentum=0.9))
    net.zero_grad_in_optimizer = False
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn((256, 32, 32, 3), generator=g, device="cuda")
    y = torch.randint(0, 10, (256,), generator=g, device="cuda")
    ds = net.make_dataset(x, y, seed=3)
    net.train_steps(ds, steps)
    torch.cuda.synchronize()
    syncs = [l.fold_sync.clone() for b in net.blocks for l in b.sublayers()]
    return net, syncs


@pytest.mark.parametrize("products", ["bf16x3", "exact"])
def test_bn_fold_step_matches_unfolded(monkeypatch, products):
    ref, _ = _step(False, monkeypatch, products)
    fol, syncs = _step(True, monkeypatch, products)
    # every carried launch re-armed its arrival counters
    assert all(int(s.abs().sum()) == 0 for s in syncs)
    assert _rel(fol.state.grad32, ref.state.grad32) <= 1e-4
    assert _rel(fol.state.model32, ref.state.model32) <= 1e-5
    for a, b in zip(fol.blocks, ref.blocks):
        for la, lb in zip(a.sublayers(), b.sublayers()):
            assert _rel(la.dgamma, lb.dgamma) <= 1e-4, la.name
            assert _rel(la.dbeta, lb.dbeta) <= 1e-4, la.name
            assert _rel(la.dw, lb.dw) <= 1e-4, la.name
    assert fol.train_stats()["loss"] == pytest.approx(ref.train_stats()["loss"], rel=1e-4)
    from metisfl_amd.ops import nn as K
    K.set_conv_products("bf16x3")
