"""Built-in model families (registered for StaticModelDef)."""
from __future__ import annotations

from metisfl_amd.models.model_def import register_family


@register_family("resnet18")
def _resnet18(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    from metisfl_amd.models.resnet import ResNet18
    return ResNet18(batch_size=batch_size, device=device, optimizer=optimizer, seed=seed, **kw)


@register_family("cifar_cnn")
def _cifar_cnn(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    from metisfl_amd.models.sequential import CifarCNN
    return CifarCNN(batch_size=batch_size, device=device, optimizer=optimizer, seed=seed, **kw)


@register_family("fashion_mnist_fc")
def _fashion_mnist_fc(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    from metisfl_amd.models.sequential import FashionMnistFC
    return FashionMnistFC(batch_size=batch_size, device=device, optimizer=optimizer, seed=seed, **kw)


@register_family("housing_mlp")
def _housing_mlp(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    from metisfl_amd.models.sequential import HousingMLP
    return HousingMLP(batch_size=batch_size, device=device, optimizer=optimizer, seed=seed, **kw)


@register_family("bert_base")
def _bert_base(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    from metisfl_amd.models.bert import BertMLM
    return BertMLM(batch_size=batch_size, device=device, optimizer=optimizer, seed=seed, **kw)


@register_family("bert_tiny")
def _bert_tiny(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    from metisfl_amd.models.bert import BERT_TINY, BertMLM
    return BertMLM(batch_size=batch_size, device=device, optimizer=optimizer, seed=seed,
                   config=kw.pop("config", BERT_TINY), **kw)


@register_family("mnist_fc")
def _mnist_fc(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    """MNIST dense model (examples/keras/models/mnist_fc.py: 784-128-128-10,
    the FashionMNIST topology; its SGD lr 0.02 is the learner's optimizer)."""
    from metisfl_amd.models.sequential import FashionMnistFC
    from metisfl_amd.ops.optim import OptimizerSpec
    return FashionMnistFC(batch_size=batch_size, device=device,
                          optimizer=optimizer or OptimizerSpec("vanilla_sgd", 0.02), seed=seed, **kw)
