"""Convergence / timing plots from a driver ``experiment.json`` (reference:
examples/utils/convergence_plots.py:15-211, which plots the community model's
test metric per round and the round / aggregation times recorded in the
federation runtime metadata, :49-60).

    python examples/utils/convergence_plots.py /tmp/metis_amd_fashionmnist/experiment.json --out plots/

Writes ``metric.png`` and ``timing.png`` (matplotlib, Agg backend) plus
``rounds.csv`` with one row per round.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
from datetime import datetime


def _ts(s: str | None) -> float | None:
    if not s:
        return None
    s = s.rstrip("Z")
    if "." in s:
        head, frac = s.split(".", 1)
        s = head + "." + frac[:6].ljust(6, "0")  # protobuf ns -> the us fromisoformat takes
    return datetime.fromisoformat(s).timestamp()


def rounds_table(stats: dict, metric: str = "accuracy") -> list[dict]:
    evals = {e["global_iteration"]: e for e in stats.get("community_model_results", {}).get(
        "community_evaluation", [])}
    rows = []
    for m in stats.get("federation_runtime_metadata", {}).get("metadata", []):
        gi = m.get("global_iteration")
        t0, t1 = _ts(m.get("started_at")), _ts(m.get("completed_at"))
        agg = m.get("model_aggregation_total_duration_ms")
        vals = []
        for ev in evals.get(gi, {}).get("evaluations", {}).values():
            v = ev.get("test_evaluation", {}).get("metric_values", {}).get(metric)
            if v is not None:
                try:
                    vals.append(float(v))
                except ValueError:
                    pass
        rows.append({"round": gi, "round_s": (t1 - t0) if t0 and t1 else None,
                     "aggregation_ms": float(agg) if agg is not None else None,
                     f"test_{metric}_mean": sum(vals) / len(vals) if vals else None})
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("experiment")
    ap.add_argument("--metric", default="accuracy")
    ap.add_argument("--out", default=".")
    a = ap.parse_args(argv)
    with open(a.experiment) as f:
        stats = json.load(f)
    rows = rounds_table(stats, a.metric)
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "rounds.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) if rows else ["round"])
        w.writeheader()
        w.writerows(rows)
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:  # pragma: no cover
        print("matplotlib unavailable: wrote rounds.csv only")
        return rows
    key = f"test_{a.metric}_mean"
    pts = [(r["round"], r[key]) for r in rows if r[key] is not None]
    if pts:
        plt.figure(figsize=(5, 3.5))
        plt.plot(*zip(*pts), marker="o")
        plt.xlabel("federation round")
        plt.ylabel(f"community model test {a.metric}")
        plt.tight_layout()
        plt.savefig(os.path.join(a.out, "metric.png"), dpi=120)
        plt.close()
    pts = [(r["round"], r["round_s"]) for r in rows if r["round_s"] is not None]
    if pts:
        plt.figure(figsize=(5, 3.5))
        plt.bar(*zip(*pts))
        plt.xlabel("federation round")
        plt.ylabel("round time (s)")
        plt.tight_layout()
        plt.savefig(os.path.join(a.out, "timing.png"), dpi=120)
        plt.close()
    return rows


if __name__ == "__main__":
    main()
