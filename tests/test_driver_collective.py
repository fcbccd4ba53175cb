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
    assert sess.termination_reason == "rounds", sess.termination_reason  # not the time cutoff
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
    sess = _session(tmp_path, 3, rounds=3, fault={"rank": 2, "round": 2}, heartbeat_timeout_s=10,
                    checkpoint_every=1)
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason  # not the time cutoff
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


def _recovered(sess, tmp_path, failed, resumed_round, world_after):
    assert len(sess.recoveries) == 1, sess.recoveries
    rc = sess.recoveries[0]
    assert rc["failed"] == [failed] and rc["survivors"] == world_after and rc["resumed_from_round"] == resumed_round
    return rc


def test_collective_recovers_from_a_sigkilled_rank(tmp_path):
    """A rank killed by SIGKILL (exit -9, as the OOM killer does) is the failed
    rank, not a peer the driver stopped."""
    sess = _session(tmp_path, 3, rounds=3, fault={"rank": 1, "round": 2, "signal": "KILL"}, heartbeat_timeout_s=10,
                    checkpoint_every=1)
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason  # not the time cutoff
    rc = _recovered(sess, tmp_path, "learner_localhost-1", 1, 2)
    assert rc["exit_code"] == -9
    md = stats["federation_runtime_metadata"]["metadata"]
    assert sorted({int(m["global_iteration"]) for m in md}) == [1, 2, 3]


def test_collective_recovers_when_rank0_dies(tmp_path):
    """Rank 0 hosts the rendezvous store and the controller bridge: when it
    dies the survivors' watchdogs lose the store, exit as peers, and are
    relaunched with the old rank 1 as the new rank 0."""
    sess = _session(tmp_path, 3, rounds=3, fault={"rank": 0, "round": 2}, heartbeat_timeout_s=8,
                    checkpoint_every=1)
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason  # not the time cutoff
    _recovered(sess, tmp_path, "learner_localhost-0", 1, 2)
    md = stats["federation_runtime_metadata"]["metadata"]
    by_gi = {}
    for m in md:
        by_gi.setdefault(int(m["global_iteration"]), m)
    assert sorted(by_gi) == [1, 2, 3] and len(by_gi[3]["completed_by_learner_id"]) == 2
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-1.log")).read()
    assert "resumed at round 1 on 2 learners (checkpoint of 3)" in log


def test_async_collective_recovers_from_a_lost_rank(tmp_path):
    """Asynchronous protocol: rank 2 of 3 dies at its second task; the
    survivors continue from the last checkpointed community version (FedRec
    state restored, the lost learner's contribution dropped), not from the
    initial model, and the federation reaches its version budget."""
    sess = _session(tmp_path, 3, rounds=10, protocol="Asynchronous", fault={"rank": 2, "round": 2},
                    heartbeat_timeout_s=8, checkpoint_every=1, extra={"debug_delay_s": {"0": 0.3, "1": 0.3}})
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason  # not the time cutoff
    rc = _recovered(sess, tmp_path, "learner_localhost-2", sess.recoveries[0]["resumed_from_round"], 2)
    assert rc["resumed_from_round"] is not None and rc["resumed_from_round"] >= 1
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async] resumed at version")]
    assert line and int(line[-1].split("version ")[1].split()[0]) == rc["resumed_from_round"]
    assert "dropped learners ['localhost-2']" in line[-1]
    md = stats["federation_runtime_metadata"]["metadata"]
    assert max(int(m["global_iteration"]) for m in md) >= 10
    # BOTH survivors were served after the resume (before the fix rank 1
    # never was, and the run ended on the time cutoff)
    after = {lid for m in md if int(m["global_iteration"]) > rc["resumed_from_round"]
             for lid in m.get("completed_by_learner_id", [])}
    assert len(after) == 2, after


def test_community_model_lineage_is_current_mid_run(tmp_path):
    """Rank 0 hands every round's community model to the controller (in the
    background): GetCommunityModelLineage serves the latest round while the
    federation is still running (the reference replaces its community model
    every global iteration, controller.cc:466)."""
    import time
    sess = _session(tmp_path, 2, rounds=4, extra={"debug_slow_s": {"0": 0.0}})
    seen = set()
    try:
        sess.initialize_federation()
        c = sess._driver_controller_grpc_client
        end = time.time() + 300
        while time.time() < end:
            running = any(p.poll() is None for n, p in sess._procs.items() if n.startswith("learner_"))
            lin = c.get_community_model_lineage(1)
            if running and len(lin.federated_models):
                fm = lin.federated_models[-1]
                if fm.global_iteration >= 1:
                    seen.add(int(fm.global_iteration))
                    assert len(fm.model.variables) > 10
            if not running:
                break
            time.sleep(0.1)
        sess.monitor_federation(request_every_secs=0.3)
    finally:
        sess.shutdown_federation(timeout=60)
    assert any(1 <= g < 4 for g in seen), seen  # an intermediate round's model, while the ranks ran


def test_learner_joins_a_running_collective_federation(tmp_path):
    """The reference's AddLearner admits a learner at any time
    (controller.cc:98-168).  2 learners run; a third joins during round 1;
    the ranks checkpoint at the round boundary, the driver relaunches 3 ranks
    from it, and the following rounds have 3 contributors with weights over
    the 3 shards."""
    import time
    from metisfl_amd.driver.driver_session import free_port
    sess = _session(tmp_path, 2, rounds=4, extra={"debug_slow_s": {"0": 0.0}})
    try:
        sess.initialize_federation()
        c = sess._driver_controller_grpc_client
        end = time.time() + 120
        while time.time() < end:  # wait until round 1 is under way
            if c.get_runtime_metadata(num_backtracks=0).metadata:
                break
            time.sleep(0.2)
        sess.join_collective_learner({"LearnerID": "localhost-2", "ProjectHome": ".",
                                      "GRPCServicer": {"Hostname": "127.0.0.1", "Port": free_port()}})
        reason = sess.monitor_federation(request_every_secs=0.3)
    finally:
        sess.shutdown_federation(timeout=60)
    assert reason == "rounds"
    assert len(sess.regroups) == 1 and sess.regroups[0]["joined"] == ["localhost-2"]
    at = sess.regroups[0]["at_round"]
    assert 1 <= at < 4
    stats = sess.get_federation_statistics()
    md = stats["federation_runtime_metadata"]["metadata"]
    by_gi = {}
    for m in md:
        by_gi[int(m["global_iteration"])] = m  # the last record of each round
    assert sorted(by_gi) == [1, 2, 3, 4]
    assert len(by_gi[at]["completed_by_learner_id"]) == 2
    assert len(by_gi[4]["completed_by_learner_id"]) == 3
    assert len(stats["learners_descriptor"]["learner"]) == 3
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    assert f"resumed at round {at} on 3 learners (checkpoint of 2)" in log
    w = [json.loads(l.split("weights ")[1]) for l in log.splitlines() if l.startswith("[collective] round 4")]
    assert w and len(w[-1]) == 3 and np.isclose(sum(w[-1]), 1.0)


def test_learners_sharing_a_device_are_colocated_in_one_rank(tmp_path):
    """The reference runs several learners per GPU (10 learners on 5 GPUs in
    examples/config/cifar10/...momentumsgd.yaml).  RCCL runs one rank per
    GPU, so learners naming the same device are hosted by ONE process
    (models/colocated.py): 3 learners on 2 "devices" -> 2 ranks, 3
    contributors per round, weights over 3 shards."""
    from metisfl_amd.driver.driver_session import DriverSession, free_port
    from metisfl_amd.models.model_def import StaticModelDef
    from metisfl_amd.utils.fedenv_parser import FederationEnvironment
    d = env_dict([free_port() for _ in range(3)], rounds=2)
    d["FederationEnvironment"]["DataPlane"] = "rccl"
    for l, dev in zip(d["FederationEnvironment"]["Learners"], ([0], [0], [1])):
        l["Devices"] = dev
    sess = DriverSession(FederationEnvironment(config=d), StaticModelDef("resnet18", width_mult=0.125), train_recipe,
                         None, eval_recipe, working_dir=str(tmp_path / "w"), device="cpu",
                         collective_options={"checkpoint_every": 1})
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason  # not the time cutoff
    assert [len(g) for g in sess._collective_groups] == [2, 1]
    job = json.load(open(os.path.join(str(tmp_path / "w"), "collective_job.json")))
    assert job["ranks"] == [[0, 1], [2]]
    md = stats["federation_runtime_metadata"]["metadata"]
    by_gi = {int(m["global_iteration"]): m for m in md}
    assert sorted(by_gi) == [1, 2] and len(by_gi[2]["completed_by_learner_id"]) == 3
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    w = [json.loads(l.split("weights ")[1]) for l in log.splitlines() if l.startswith("[collective] round 2")]
    assert w and len(w[-1]) == 3 and np.isclose(sum(w[-1]), 1.0)
    assert not os.path.exists(os.path.join(str(tmp_path / "w"), "learner_localhost-1.log"))  # hosted by rank 0
    from metisfl_amd.parallel.checkpoint import resolve
    ck = resolve(os.path.join(str(tmp_path / "w"), "collective_checkpoint"))
    assert sorted(f for f in os.listdir(ck) if f.startswith("learner_")) == [
        "learner_localhost-0.safetensors", "learner_localhost-1.safetensors",
        "learner_localhost-2.safetensors"]


def _session_devices(tmp_path, devices, rounds, protocol="Asynchronous", he=False, **opts):
    """Learners placed on devices (learners naming the same device share one
    rank: co-located).  ``he``: PWA under CKKS."""
    from metisfl_amd.driver.driver_session import DriverSession, free_port
    from metisfl_amd.models.model_def import StaticModelDef
    from metisfl_amd.utils.fedenv_parser import FederationEnvironment
    d = env_dict([free_port() for _ in range(len(devices))], rounds=rounds, protocol=protocol,
                 rule="PWA" if he else "FedAvg")
    d["FederationEnvironment"]["DataPlane"] = "rccl"
    if he:
        d["FederationEnvironment"]["HomomorphicEncryption"] = {"Scheme": "CKKS", "BatchSize": 4096,
                                                               "ScalingFactorBits": 52}
    for l, dev in zip(d["FederationEnvironment"]["Learners"], devices):
        l["Devices"] = dev
    return DriverSession(FederationEnvironment(config=d), StaticModelDef("resnet18", width_mult=0.125), train_recipe,
                         None, eval_recipe, working_dir=str(tmp_path / "w"), device="cpu", collective_options=opts)


def test_async_colocated_learners_through_the_driver(tmp_path):
    """The reference's asynchronous configs place several learners on one GPU
    (examples/config/fashionmnist/test_localhost_asynchronous_vanillasgd.yaml:
    all 10 on GPU 0) and schedule each learner on its own
    (asynchronous_scheduler.h:12-18).  4 learners on 2 devices -> 2 ranks of 2
    co-located learners, each learner a FedRec participant: one
    runtime-metadata record per community version up to the budget, every
    learner contributing, stale updates from the slower rank."""
    sess = _session_devices(tmp_path, [[0], [0], [1], [1]], rounds=12, checkpoint_every=2,
                            extra={"debug_delay_s": {"1": 0.3}})
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason
    job = json.load(open(os.path.join(str(tmp_path / "w"), "collective_job.json")))
    assert job["ranks"] == [[0, 1], [2, 3]]
    md = stats["federation_runtime_metadata"]["metadata"]
    gis = sorted(int(m["global_iteration"]) for m in md)
    assert gis[:12] == list(range(1, 13))
    who = {lid for m in md for lid in m.get("completed_by_learner_id", [])}
    assert len(who) == 4, who
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async]")][-1]
    assert "over 4 learners on 2 ranks" in line
    stal = json.loads(line.split("staleness ")[1])
    assert max(stal) > 0
    assert stats["community_model_results"]["community_evaluation"]


def test_async_secure_pwa_through_the_driver(tmp_path):
    """asynchronous PWA (CKKS) on the collective data plane.  3
    learners on 2 devices (rank 0 hosts two), PWA + HomomorphicEncryption:
    the ranks load the driver's key files, every finisher submits a
    ciphertext, rank 0 aggregates over the latest ciphertexts (checkpointing
    them), and the federation reaches its version budget with every learner
    contributing."""
    sess = _session_devices(tmp_path, [[0], [0], [1]], rounds=6, he=True, checkpoint_every=2,
                            extra={"debug_delay_s": {"1": 0.2}})
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason
    job = json.load(open(os.path.join(str(tmp_path / "w"), "collective_job.json")))
    fj = job["federation"]
    assert fj["secure_aggregation"] and fj["he_key_dir"] and os.path.exists(
        os.path.join(fj["he_key_dir"], "key-private.txt"))
    md = stats["federation_runtime_metadata"]["metadata"]
    assert sorted(int(m["global_iteration"]) for m in md)[:6] == list(range(1, 7))
    who = {lid for m in md for lid in m.get("completed_by_learner_id", [])}
    assert len(who) == 3, who
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async]")][-1]
    assert "over 3 learners on 2 ranks" in line and "secure PWA over ciphertexts" in line
    from metisfl_amd.parallel import checkpoint as ck
    d = ck.resolve(job["checkpoint_dir"])
    meta = json.load(open(os.path.join(d, "federation.json")))
    assert meta["secure_aggregation"] and not os.path.exists(os.path.join(d, "community_model.pb"))


def test_async_colocated_rank_lost_resumes_from_checkpoint(tmp_path):
    """Rank 1 (hosting learners 2 and 3) dies at its learners' second task;
    the driver relaunches the survivors (learners 0 and 1, now one rank) from
    the last checkpointed community version, their FedRec contributions kept
    by learner id and the lost learners' dropped, and the federation reaches
    its version budget."""
    sess = _session_devices(tmp_path, [[0], [0], [1], [1]], rounds=14, fault={"rank": 1, "round": 2},
                            heartbeat_timeout_s=8, checkpoint_every=1, extra={"debug_delay_s": {"0": 0.2}})
    stats = sess.run_collective(request_every_secs=0.3)
    assert sess.termination_reason == "rounds", sess.termination_reason
    rc = sess.recoveries[0]
    assert len(sess.recoveries) == 1 and rc["failed"] == ["learner_localhost-2"]
    assert sorted(rc["lost_learners"]) == ["localhost-2", "localhost-3"] and rc["survivors"] == 2
    assert rc["resumed_from_round"] is not None and rc["resumed_from_round"] >= 1
    log = open(os.path.join(str(tmp_path / "w"), "learner_localhost-0.log")).read()
    line = [l for l in log.splitlines() if l.startswith("[collective-async] resumed at version")]
    assert line and int(line[-1].split("version ")[1].split()[0]) == rc["resumed_from_round"]
    # the lost learners' contributions leave the running sum (a learner whose
    # first task had not finished contributed nothing yet)
    dropped = json.loads(line[-1].split("dropped learners ")[1].rstrip(")").replace("'", '"'))
    assert dropped and set(dropped) <= {"localhost-2", "localhost-3"}, dropped
    md = stats["federation_runtime_metadata"]["metadata"]
    assert max(int(m["global_iteration"]) for m in md) >= 14
    after = {lid for m in md if int(m["global_iteration"]) > rc["resumed_from_round"]
             for lid in m.get("completed_by_learner_id", [])}
    assert len(after) == 2, after  # both survivors served after the resume
