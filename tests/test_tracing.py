"""Observability: roctx ranges degrade to no-ops without
the library, the per-round JSONL log carries the runtime metadata."""
import numpy as np

from metisfl_amd.utils import tracing


def test_roctx_range_is_safe_anywhere():
    with tracing.range("metisfl.test"):
        tracing.mark("inside")
    assert isinstance(tracing.roctx_available(), bool)


def test_jsonl_round_log(tmp_path):
    from metisfl_amd.models.sequential import HousingMLP
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig
    comm = Comm(backend="gloo")
    net = HousingMLP(batch_size=4, device="cpu", seed=0, optimizer=OptimizerSpec("vanilla_sgd", 0.01))
    rng = np.random.default_rng(0)
    ds = net.make_dataset(rng.standard_normal((16, 13)).astype(np.float32),
                          rng.standard_normal(16).astype(np.float32))
    log = tmp_path / "rounds.jsonl"
    cfg = FederationConfig(batch_size=4, local_epochs=1, evaluate_test=False, jsonl_log=str(log))
    fed = CollectiveFederation(comm, net, ds, cfg)
    for _ in range(3):
        fed.run_round()
    rows = tracing.JsonlLog.read(str(log))
    assert [r["global_iteration"] for r in rows] == [1, 2, 3]
    assert all(r["kind"] == "round" and r["rounds_per_s"] > 0 and "allreduce_gbps" in r for r in rows)
    assert rows[0]["num_local_updates"] == [4]
