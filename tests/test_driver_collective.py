"""The driver-launched collective (DataPlane: rccl) federation beyond plain
synchronous rounds (gloo on the CPU, real processes):

* community-model evaluation after every all-reduce, recorded with the round:
  a low MetricCutoffScore terminates the federation on "metric" and the
  statistics carry community_model_results (controller.cc:469-485,
  driver_session.py:423-467 in the reference);
* the asynchronous protocol: FedRec over point-to-point transfers with
  uneven learner speeds (staleness > 0), one runtime-metadata record per
  community version, clean shutdown at the FederationRounds cutoff;
* a lost rank: rank 2 of 3 dies at round 2, the driver relaunches the two
  survivors as fresh processes from the round-1 FederatedModel checkpoint and
  the federation completes its rounds on 2 learners with recomputed weights.
"""
import json
import os

import numpy as np
import pytest

from tests.test_driver import env_dict, eval_recipe, train_recipe


def _session(tmp_path, n, rounds, protocol="Synchronous", metric_cutoff=2.0, **opts):
    from metisfl_amd.driver.driver_session import DriverSession, free_port
    from metisfl_amd.models.model_def import StaticModelDef
    from metisfl_amd.utils.fedenv_parser import FederationEnvironment
    d = env_dict([free_port() for _ in range(n)], rounds=rounds, protocol=protocol)
    d["FederationEnvironment"]["DataPlane"] = "rccl"
    d["FederationEnvironment"]["TerminationSignals"]["MetricCutoffScore"] = metric_cutoff
    fe = FederationEnvironment(config=d)
    return DriverSession(fe, StaticModelDef("resnet18", width_mult=0.125), train_recipe, None, eval_recipe,
                         working_dir=str(tmp_path / "w"), device="cpu", collective_options=opts)


def test_collective_community_evaluation_and_metric_cutoff(tmp_path):
    sess = _session(tmp_path, 2, rounds=5, metric_cutoff=0.0)
    try:
        sess.initialize_federation()
        reason = sess.monitor_federation(request_every_secs=0.3)
    finally:
        sess.shutdown_federation(timeout=60)
    assert reason == "metric"
    stats = sess.get_federation_statistics()
    res = stats["community_model_results"]["community_evaluation"]
    assert res and all(len(r["evaluations"]) == 2 for r in res)
    for r in res:
        for ev in r["evaluations"].values():
            acc = float(ev["test_evaluation"]["metric_values"]["accuracy"])
            assert 0.0 <= acc <= 1.0
    md = stats["federation_runtime_metadata"]["metadata"]
    assert max(int(m["global_iteration"]) for m in md) < 5  # stopped early
    sess.save_statistics(str(tmp_path / "experiment.json"))
    assert json.load(open(tmp_path / "experiment.json"))["community_model_results"]["community_evaluation"]


def test_collective_asynchronous_protocol_through_the_driver(tmp_path):
    sess = _session(tmp_path, 3, rounds=8, protocol="Asynchronous",
                    extra={"debug_delay_s": {"2": 0.6, "1": 0.1}})
    stats = sess.run_collective(request_every_secs=0.3)
    md = stats["federation_runtime_metadata"]["metadata"]
    gis = sorted(int(m["global_iteration"]) for m in md)
    assert gis[:8] == list(range(1, 9))  # one record per community version (FedRec update)
    lineages = stats["learners_models_results"]["learner_task"]
    assert len(lineages) == 3 and all(len(v["task_metadata"]) >= 1 for v in lineages.values())
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async]")][-1]
    stal = json.loads(line.split("staleness ")[1])
    assert max(stal) > 0  # the slow learner trained on an older community model
    assert stats["community_model_results"]["community_evaluation"]


def test_collective_recovers_from_a_lost_rank(tmp_path):
    sess = _session(tmp_path, 3, rounds=3, fault={"rank": 2, "round": 2}, heartbeat_timeout_s=10)
    stats = sess.run_collective(request_every_secs=0.3)
    assert len(sess.recoveries) == 1
    rc = sess.recoveries[0]
    assert rc["failed"] == ["learner_localhost-2"] and rc["survivors"] == 2 and rc["resumed_from_round"] == 1
    md = stats["federation_runtime_metadata"]["metadata"]
    assert sorted({int(m["global_iteration"]) for m in md}) == [1, 2, 3]
    # round 1 had three contributors, rounds 2-3 the two survivors
    by_gi = {}
    for m in md:
        by_gi.setdefault(int(m["global_iteration"]), m)
    assert len(by_gi[1]["completed_by_learner_id"]) == 3
    assert len(by_gi[3]["completed_by_learner_id"]) == 2
    assert len(stats["learners_descriptor"]["learner"]) == 2
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    assert "resumed at round 1 on 2 learners (checkpoint of 3)" in log
    w = [json.loads(l.split("weights ")[1]) for l in log.splitlines() if l.startswith("[collective] round 3")]
    assert w and np.isclose(sum(w[-1]), 1.0) and len(w[-1]) == 2
