"""Controller-side device aggregation (engine/device_agg.*): every rule the
engine runs on the GPU must be BYTE-identical to its host implementation
(aggregation.cc, the reference's federated_average.cc / federated_stride.cc /
federated_recency.cc / private_weighted_average.cc semantics), and staged
models must be aggregated from HBM without a second upload."""
import numpy as np
import pytest

from metisfl_amd import _engine as E
from metisfl_amd.proto import model_pb2
from metisfl_amd.utils.tensor_codec import model_from_arrays

pytestmark = pytest.mark.gpu

MIXED = [("w", np.float32, (257, 131)), ("b", np.float64, (1001,)), ("steps", np.int64, (3,)),
         ("q", np.int8, (4099,)), ("u", np.uint16, (77,)), ("i", np.int32, (12345,)),
         ("empty", np.float32, (0,)), ("big", np.float32, (300_001,))]


def _rand_model(rng, spec=MIXED):
    names, arrs = [], []
    for name, dt, shape in spec:
        if np.issubdtype(dt, np.integer):
            info = np.iinfo(dt)
            lo, hi = max(info.min // 4, -10_000), min(info.max // 4, 10_000)
            a = rng.integers(lo, hi, size=shape).astype(dt)
        else:
            a = rng.standard_normal(shape).astype(dt)
        names.append(name)
        arrs.append(a)
    return model_from_arrays(names, arrs).SerializeToString()


@pytest.fixture(autouse=True)
def _device_on():
    assert E.device_aggregation_available(), "no HIP device visible to the controller engine"
    E.set_device_aggregation(True, 0)
    yield
    E.set_device_aggregation(True, 1 << 20)


def _host_and_device(fn):
    E.set_device_aggregation(False)
    host = fn()
    E.set_device_aggregation(True, 0)
    before = E.device_aggregation_stats()
    dev = fn()
    after = E.device_aggregation_stats()
    return host, dev, before, after


@pytest.mark.parametrize("n", [1, 8, 37])  # 37 > 32 inputs per launch: accumulate path
def test_fedavg_device_is_byte_identical(n):
    rng = np.random.default_rng(n)
    ms = [_rand_model(rng) for _ in range(n)]
    ws = list(rng.random(n) / n)
    host, dev, b, a = _host_and_device(lambda: E.aggregate_models("fed_avg", ms, ws))
    assert a["fedavg_calls"] == b["fedavg_calls"] + 1
    assert host == dev


@pytest.mark.parametrize("stride", [1, 3])
def test_fedstride_device_is_byte_identical(stride):
    rng = np.random.default_rng(10 + stride)
    ms = [_rand_model(rng) for _ in range(7)]
    ws = list(rng.random(7))
    host, dev, b, a = _host_and_device(lambda: E.aggregate_models("fed_stride", ms, ws, stride))
    assert a["rolling_calls"] > b["rolling_calls"]
    assert host == dev


def test_fedrec_device_is_byte_identical():
    rng = np.random.default_rng(3)
    m = [_rand_model(rng) for _ in range(4)]
    seq = [([m[0]], [1.0]), ([m[1]], [2.0]), ([m[0], m[2]], [1.0, 1.5]), ([m[1], m[3]], [2.0, 0.5]),
           ([m[2], m[0]], [1.5, 3.0])]

    def run():
        agg = E.FedRec()
        return [agg.aggregate(models, ws) for models, ws in seq]

    host, dev, b, a = _host_and_device(run)
    assert a["rolling_calls"] > b["rolling_calls"]
    assert host == dev


def test_staged_models_are_aggregated_from_hbm():
    rng = np.random.default_rng(5)
    spec = [("w%d" % i, np.float32, (65_536,)) for i in range(6)]
    ms = [_rand_model(rng, spec) for _ in range(8)]
    ws = list(rng.random(8) / 8)
    staged = E.StagedModels([f"L{i}" for i in range(8)], ms)
    s0 = E.device_aggregation_stats()
    dev = staged.aggregate("fed_avg", ws)
    s1 = E.device_aggregation_stats()
    assert s1["resident_hits"] - s0["resident_hits"] == 8
    assert s1["cold_uploads"] == s0["cold_uploads"]
    E.set_device_aggregation(False)
    assert staged.aggregate("fed_avg", ws) == dev
    fm = model_pb2.FederatedModel()
    fm.ParseFromString(dev)
    assert fm.num_contributors == 8 and len(fm.model.variables) == 6


def test_pwa_device_is_byte_identical(tmp_path):
    c = E.CKKS(4096, 52)
    c.gen_crypto_context_and_keys(str(tmp_path))
    rng = np.random.default_rng(9)
    xs = [rng.standard_normal(20_000) for _ in range(5)]
    cts = [c.encrypt(x) for x in xs]
    ws = [0.1, 0.2, 0.3, 0.15, 0.25]
    host, dev, b, a = _host_and_device(lambda: c.compute_weighted_average(cts, ws))
    assert a["pwa_calls"] == b["pwa_calls"] + 1
    assert host == dev
    out = c.decrypt(dev, 20_000)
    assert np.abs(out - sum(w * x for w, x in zip(ws, xs))).max() < 1e-6


def test_grpc_controller_stages_and_aggregates_on_device(tmp_path):
    """End to end: a gRPC controller with 6 echo learners (worker processes,
    benchmarks/scalability.py) and a 4 MB model -- every learner's model is
    staged into HBM on arrival and the rounds aggregate from there."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "benchmarks"))
    import scalability
    E.set_device_aggregation(True, 1 << 20)
    s0 = E.device_aggregation_stats()
    r = scalability.run_case(6, 4.0, rounds=2, workers=3, tmpdir=str(tmp_path))
    s1 = r["device_aggregation"]
    assert r["rounds_measured"] >= 2, r
    assert s1["available"]
    assert s1["staged_models"] - s0.get("staged_models", 0) >= 6 * 2
    assert s1["fedavg_calls"] - s0.get("fedavg_calls", 0) >= 2
    assert s1["resident_hits"] - s0.get("resident_hits", 0) >= 6 * 2
    assert s1["cold_uploads"] == s0.get("cold_uploads", 0)


def test_rolling_state_falls_back_to_host_when_hbm_budget_is_exhausted(tmp_path):
    """FedStride with a device budget that holds the rolling state but not the
    next operand: the merge continues on the host from the device's scaled
    sum instead of failing, byte-identical to the host rule (own process: the
    budget is read when the device aggregator starts)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys
sys.path.insert(0, {root!r})
import numpy as np
from metisfl_amd import _engine as E
from tests.test_device_aggregation_gpu import _rand_model
rng = np.random.default_rng(11)
ms = [_rand_model(rng) for _ in range(5)]
ws = list(rng.random(5))
E.set_device_aggregation(False)
host = E.aggregate_models("fed_stride", ms, ws, 1)
E.set_device_aggregation(True, 0)
dev = E.aggregate_models("fed_stride", ms, ws, 1)
st = E.device_aggregation_stats()
print("RESULT", host == dev, st["rolling_calls"], flush=True)
"""
    env = dict(os.environ, METISFL_AMD_DEVICE_AGG_MAX_GB=str(2.2e6 / (1 << 30)), PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][0].split()
    assert line[1] == "True"
    assert int(line[2]) >= 1  # the rolling state did start on the device
