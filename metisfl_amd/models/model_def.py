"""Model definitions the learner can instantiate (reference:
metisfl/models/model_def.py:8-23 ``ModelDef`` / ``PyTorchDef``).

The reference ships model *code* to learners as a Keras SavedModel or a
cloudpickled torch class.  Here the built-in families are named in a small
JSON document (family + constructor kwargs) that is safe to load anywhere,
and the learner builds the static-graph network for its own GPU:

    {"family": "resnet18", "kwargs": {"num_classes": 10}}

``TorchModelDef`` keeps the reference's PyTorch contract for arbitrary user
``nn.Module``s (get_model / fit / evaluate)."""
from __future__ import annotations

import abc
import json
import os


class ModelDef(abc.ABC):
    @abc.abstractmethod
    def get_model(self, *args, **kwargs):
        ...


_FAMILIES = {}


def register_family(name):
    def deco(fn):
        _FAMILIES[name] = fn
        return fn
    return deco


def families() -> list[str]:
    _load_builtin()
    return sorted(_FAMILIES)


def _load_builtin():
    # import for the registration side effect
    from metisfl_amd.models import zoo  # noqa: F401


class StaticModelDef(ModelDef):
    """A built-in family on the static hipGraph executor."""

    FILENAME = "model_definition.json"

    def __init__(self, family: str, **kwargs):
        self.family = family
        self.kwargs = kwargs

    def get_model(self, batch_size: int, device="cpu", optimizer=None, seed: int = 0):
        _load_builtin()
        if self.family not in _FAMILIES:
            raise KeyError(f"unknown model family {self.family!r}; known: {sorted(_FAMILIES)}")
        return _FAMILIES[self.family](batch_size=batch_size, device=device, optimizer=optimizer,
                                      seed=seed, **self.kwargs)

    def to_json(self) -> str:
        return json.dumps({"family": self.family, "kwargs": self.kwargs})

    @classmethod
    def from_json(cls, s: str) -> "StaticModelDef":
        d = json.loads(s)
        return cls(d["family"], **d.get("kwargs", {}))

    def save(self, model_dir: str) -> str:
        os.makedirs(model_dir, exist_ok=True)
        p = os.path.join(model_dir, self.FILENAME)
        with open(p, "w") as f:
            f.write(self.to_json())
        return p

    @classmethod
    def load(cls, model_dir: str) -> "StaticModelDef":
        with open(os.path.join(model_dir, cls.FILENAME)) as f:
            return cls.from_json(f.read())


class TorchModelDef(ModelDef):
    """User PyTorch model (reference PyTorchDef): ``get_model()`` returns an
    ``nn.Module`` producing logits; ``fit`` / ``evaluate`` may be overridden,
    otherwise TorchModelOps runs a standard cross-entropy loop with the fused
    HIP optimizer."""

    def get_model(self):
        raise NotImplementedError

    def loss(self, outputs, targets):
        import torch.nn.functional as F
        return F.cross_entropy(outputs, targets.long())
