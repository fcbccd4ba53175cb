"""The example model families on the static executor (CPU reference ops):
parameter counts vs the reference's Keras models, local training reduces the
loss, dropout / pooling / padded-unit semantics."""
import numpy as np
import pytest
import torch

from metisfl_amd.ops.optim import OptimizerSpec


def _train(net, x, y, steps):
    ds = net.make_dataset(x, y, shuffle=True)
    net.reset_train_stats()
    net.train_steps(ds, 1)
    first = net.train_stats()["loss"]
    for _ in range(steps):
        net.reset_train_stats()
        net.train_steps(ds, ds.steps_per_epoch)
    return first, net.train_stats()["loss"]


def test_fashion_mnist_fc_learns_and_counts():
    from metisfl_amd.models.sequential import FashionMnistFC
    net = FashionMnistFC(batch_size=16, optimizer=OptimizerSpec("vanilla_sgd", 0.1), seed=1)
    live = {s.name: s for s in net.state.specs}
    # 784*128+128 + 128*128+128 + 128*10+10 = 118,282 live parameters (reference count)
    n_live = sum(s.numel if s.live_rows is None else s.live_rows * (s.numel // s.shape[0]) for s in live.values())
    n_live_bias = sum(s.numel - 10 for s in live.values() if s.name == "dense_2.bias")
    assert n_live - n_live_bias == 118_282
    rng = np.random.default_rng(0)
    x = rng.standard_normal((64, 28, 28)).astype(np.float32)
    y = (x.reshape(64, -1)[:, :10].argmax(1)).astype(np.int64)  # learnable labels
    first, last = _train(net, x, y, 15)
    assert last < first * 0.8
    # padded (inert) output units stay zero
    k = net.state.view("dense_2.kernel")
    assert float(k[10:].abs().sum()) == 0.0


def test_cifar_cnn_counts_and_step():
    from metisfl_amd.models.sequential import CifarCNN
    net = CifarCNN(batch_size=4, optimizer=OptimizerSpec("momentum_sgd", 0.01, momentum=0.9), seed=2)
    names = [s.name for s in net.state.specs]
    assert "batch_normalization.moving_mean" in names and "dense.kernel" in names
    rng = np.random.default_rng(1)
    x = rng.standard_normal((8, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, 8)
    before = net.state.model32.clone()
    first, last = _train(net, x, y, 2)
    assert np.isfinite(last) and not torch.equal(before, net.state.model32)


def test_housing_mlp_regression():
    from metisfl_amd.models.sequential import HousingMLP
    net = HousingMLP(batch_size=16, optimizer=OptimizerSpec("adam", 0.01), seed=3, params_per_layer=16)
    rng = np.random.default_rng(2)
    x = rng.standard_normal((64, 13)).astype(np.float32)
    y = (x @ rng.standard_normal(13)).astype(np.float32)
    first, last = _train(net, x, y, 30)
    assert last < first * 0.5


def test_dropout_mask_is_reproducible_and_scaled():
    from metisfl_amd.ops import nn as K
    x = torch.ones(4096, dtype=torch.bfloat16)
    y1, y2 = torch.empty_like(x), torch.empty_like(x)
    step = torch.tensor([7], dtype=torch.int32)
    K.dropout(x, y1, 0.25, 11, step)
    K.dropout(x, y2, 0.25, 11, step)
    assert torch.equal(y1, y2)
    kept = (y1 != 0).float().mean().item()
    assert 0.7 < kept < 0.8 and float(y1.max()) == pytest.approx(1 / 0.75, rel=1e-2)
    step[0] = 8
    K.dropout(x, y2, 0.25, 11, step)
    assert not torch.equal(y1, y2)


def test_model_zoo_families():
    from metisfl_amd.models.model_def import StaticModelDef, families
    assert {"resnet18", "cifar_cnn", "fashion_mnist_fc", "housing_mlp"} <= set(families())
    net = StaticModelDef("fashion_mnist_fc").get_model(batch_size=8)
    assert net.B == 8


@pytest.mark.parametrize("n", [10_000, 1_250, 10])
def test_evaluation_counts_every_sample(n):
    """evaluation covers every test sample (the last batch's
    tail is padding the statistics skip), not floor(n / B) full batches."""
    from metisfl_amd.models.sequential import FashionMnistFC
    net = FashionMnistFC(batch_size=32, seed=0)
    rng = np.random.default_rng(n)
    x = rng.standard_normal((n, 28, 28)).astype(np.float32)
    y = rng.integers(0, 10, n)
    ds = net.make_dataset(x, y, shuffle=False)
    assert ds.steps_per_epoch == -(-n // 32)
    net.evaluate(ds)
    assert int(net.stats[2]) == n
    # the same accuracy as counting by hand over all n samples
    net.stats.zero_()
    acc = net.evaluate(ds)["accuracy"]
    assert 0.0 <= acc <= 1.0
    # drop_last keeps the old full-batches-only behaviour on request
    if n >= 32:
        assert net.make_dataset(x, y, shuffle=False, drop_last=True).steps_per_epoch == n // 32
