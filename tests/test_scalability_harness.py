"""Orchestration at scale (reference: examples/keras/scalability_testing.py
with test/learner_notrain_noeval.py echo learners): the harness in
benchmarks/scalability.py drives 24 echo learners in 4 worker processes
through synchronous FedAvg rounds against the gRPC controller and reports
dispatch / collect / aggregation / round times from the runtime metadata."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))


def test_scalability_harness_24_echo_learners(tmp_path):
    import scalability

    r = scalability.run_case(24, 0.5, rounds=2, workers=4, tmpdir=str(tmp_path))
    assert r["learners"] == 24 and r["workers"] == 4
    assert r["rounds_measured"] >= 2, r
    for k in ("dispatch_ms", "collect_ms", "aggregation_ms", "round_ms"):
        assert r[k] is not None and r[k] > 0, (k, r)
    assert r["dispatch_ms"] <= r["collect_ms"] <= r["round_ms"]
    for rd in r["per_round"]:
        assert rd["dispatch_ms"] is not None  # every learner received every round's task
