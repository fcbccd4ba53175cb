"""Test-set evaluation through the wide-batch twin (models/net.py eval_batch):
the twin shares the model's parameters and BatchNorm running statistics, so
its loss / accuracy equal the training-batch pass over the same samples (every
sample once, the padded tail skipped), and it tracks the model as it trains."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(n):
    from metisfl_amd.models.resnet import ResNet18
    from metisfl_amd.ops.optim import OptimizerSpec
    net = ResNet18(batch_size=32, device="cuda", seed=3, optimizer=OptimizerSpec("momentum_sgd", 0.05, momentum=0.9))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn((n, 32, 32, 3), generator=g, device="cuda")
    y = torch.randint(0, 10, (n,), generator=g, device="cuda")
    return net, net.make_dataset(x, y, shuffle=False), net.make_dataset(x, y, seed=2)


@pytest.mark.parametrize("n", [1000, 256])
def test_eval_twin_matches_training_batch_pass(n):
    net, test_ds, train_ds = _pair(n)
    net.train_steps(train_ds, 12)  # non-trivial running statistics
    net.eval_batch = 0
    ref = net.evaluate(test_ds)
    net.eval_batch = 512
    got = net.evaluate(test_ds)
    # 1000 samples: two batches of 512 (2.4 % padding); 256: one of 256
    twin = net._eval_twins[{1000: 512, 256: 256}[n]]
    assert twin is not False and twin.B == {1000: 512, 256: 256}[n]
    assert twin.state is net.state
    # the wider batch may pick other split-K plans (fp32 summation order):
    # a near-tie argmax may flip, the loss agrees to fp32 rounding
    assert abs(got["accuracy"] - ref["accuracy"]) <= 2.0 / n
    assert got["loss"] == pytest.approx(ref["loss"], rel=1e-5)
    # the twin follows the shared parameters after more training
    net.train_steps(train_ds, 8, 12)
    net.eval_batch = 0
    ref2 = net.evaluate(test_ds)
    net.eval_batch = 512
    got2 = net.evaluate(test_ds)
    assert got2["loss"] == pytest.approx(ref2["loss"], rel=1e-5)
    assert abs(got2["accuracy"] - ref2["accuracy"]) <= 2.0 / n
    assert got2["loss"] != pytest.approx(got["loss"], rel=1e-9)
