"""Built-in model families (registered for StaticModelDef)."""
from __future__ import annotations

from metisfl_amd.models.model_def import register_family


@register_family("resnet18")
def _resnet18(batch_size, device="cpu", optimizer=None, seed=0, **kw):
    from metisfl_amd.models.resnet import ResNet18
    return ResNet18(batch_size=batch_size, device=device, optimizer=optimizer, seed=seed, **kw)
