"""Metric dictionary helpers (reference: metisfl/utils/formatting.py:7-45).

Model metrics travel as ``map<string, string>`` (metis.proto ModelEvaluation),
so numbers are stringified, NaN as "NaN".  ``normalize`` flattens nested
dicts with "_" separators (the reference uses pandas.json_normalize; this is
the same flattening without the pandas dependency on the hot path)."""
from __future__ import annotations

import math


def _str(v) -> str:
    if isinstance(v, str):
        return v
    if isinstance(v, float) and math.isnan(v):
        return "NaN"
    return str(v)


class DictionaryFormatter:
    @classmethod
    def normalize(cls, d: dict, sep: str = "_") -> dict:
        out = {}

        def walk(prefix, obj):
            if isinstance(obj, dict) and obj:
                for k, v in obj.items():
                    walk(f"{prefix}{sep}{k}" if prefix else str(k), v)
            else:
                out[prefix] = _str(obj) if not isinstance(obj, (list, tuple)) else str(list(obj))
        walk("", d)
        return out

    @classmethod
    def stringify(cls, d: dict, stringify_nan: bool = True) -> dict:
        out = {}
        for k, v in d.items():
            if isinstance(v, (list, tuple)):
                out[k] = [_str(x) if stringify_nan else str(x) for x in v]
            else:
                out[k] = _str(v) if stringify_nan else str(v)
        return out

    @classmethod
    def listify_values(cls, d: dict) -> dict:
        return {k: v if isinstance(v, list) else [v] for k, v in d.items()}
